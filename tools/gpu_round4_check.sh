#!/bin/bash
# Round-4 GPU check, run ON THE GPU BOX (gpurun): the -m gpu suite, the round-3 library on the
# small vol-of-vol CF-cut test (expected to fail there: the fp32 cancellation ADVICE r3 found),
# and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_r03.so timeout -k 10 120 \
    python -u -m pytest tests/test_gpu_parity.py -m gpu -k small_vol -v --timeout 100 \
    --timeout-method thread > gpurun_out/r03lib_small_vol.log 2>&1
echo "r03 lib small-vol rc=$? (1 = the old bound fails the test)" >> gpurun_out/r03lib_small_vol.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
DHCOS_GEN_TIMING=1 timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1
timeout -k 10 300 python3 tools/occupancy_probe.py c3 > gpurun_out/occ_c3.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 tools/occupancy_probe.py c2 > gpurun_out/occ_c2.jsonl 2>&1 || exit 1
echo done
