#!/bin/bash
# Round-6 measurement set, run ON THE GPU BOX (gpurun): the driver's default bench command under
# rocprofv3 --stats, then the per-config stats + PMC passes (tools/gpu_profile.sh), then an
# instruction-cache pass of C3 when the counters exist.  tools/summarize_profiles.py (in the build
# container) turns gpurun_out/prof into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r06}
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
if [ -z "$NODEFAULT" ]; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o ${TAG}_default_cmd --output-format csv \
    -- python3 bench.py > gpurun_out/prof/${TAG}_default_cmd.log 2>&1 || { echo "profiled default bench failed"; exit 1; }
echo "default stats ok"
fi
TAG=$TAG CONFIGS="${CONFIGS:-c3 c2 c1 c4}" bash tools/gpu_profile.sh || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/prof/counters_avail.txt 2>&1
grep -o "SQC_ICACHE_[A-Z_]*" gpurun_out/prof/counters_avail.txt | sort -u | head -8
if grep -q "SQC_ICACHE_MISSES" gpurun_out/prof/counters_avail.txt; then
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/prof -o ${TAG}_c3_icache --output-format csv \
      -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --no-calib --no-side > gpurun_out/prof/${TAG}_c3_icache.log 2>&1 && echo "icache ok"
fi

# the per-dispatch traces are not needed by summarize_profiles.py and would pass the 64 MiB merge cap
gzip -f gpurun_out/prof/${TAG}_default_cmd_kernel_trace.csv 2>/dev/null; rm -f gpurun_out/prof/*_kernel_trace.csv
gzip -f gpurun_out/prof/*_counter_collection.csv 2>/dev/null
du -sh gpurun_out
echo done
