#!/bin/bash
# Round-4 measurement record, run ON THE GPU BOX:
#   1) the default bench line (what the driver runs) -> gpurun_out/r04_bench_default.json
#   2) rocprofv3 --kernel-trace --stats of that same default command
#   3) the per-config profile set (stats + PMC passes) for c2 c3 c5
#   4) calibrate(300, 3) medians of both optimizer drivers on c1 c2 c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_default.json 2> gpurun_out/r04_bench_default.err \
    || { echo "default bench failed rc=$?"; tail -5 gpurun_out/r04_bench_default.err; exit 1; }
echo "default bench ok"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r04_default_stats --output-format csv \
    -- python bench.py > gpurun_out/prof/r04_default_stats.log 2>&1 || { echo "default stats failed rc=$?"; exit 1; }
echo "default stats ok"
TAG=r04 CONFIGS="c2 c3 c5" bash tools/gpu_profile.sh || exit 1
bash tools/gpu_calib_drivers.sh || exit 1
echo done
