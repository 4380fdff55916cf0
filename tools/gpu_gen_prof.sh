#!/bin/bash
# rocprofv3 kernel stats of the device generator (tools/gen_device_timing.py, 1M samples)
set -e
mkdir -p gpurun_out/genprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/genprof -o gen -- python3 $GRAFT_REPO_ROOT/tools/gen_device_timing.py 1000000 2 > $GRAFT_REPO_ROOT/gpurun_out/genprof/run.log 2>&1
