#!/bin/bash
# Round-5 measurement set, run ON THE GPU BOX (gpurun): the driver's default bench command, its
# rocprofv3 --stats, and the per-config stats + PMC passes (tools/gpu_profile.sh) whose summary
# (tools/summarize_profiles.py, run afterwards in the build container) feeds profiles/ and
# profiles/pmc_traffic.json (bench.py's executed-flop roofline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r05}
mkdir -p gpurun_out/prof
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err \
    || { echo "default bench failed"; tail -5 gpurun_out/bench_${TAG}_default.err; exit 1; }
tail -c 600 gpurun_out/bench_${TAG}_default.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o ${TAG}_default_cmd --output-format csv \
    -- python3 bench.py > gpurun_out/prof/${TAG}_default_cmd.log 2>&1 || { echo "profiled default bench failed"; exit 1; }
echo "default stats ok"
TAG=$TAG CONFIGS="${CONFIGS:-c3 c2 c5}" bash tools/gpu_profile.sh
