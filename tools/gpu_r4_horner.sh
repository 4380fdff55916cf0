#!/bin/bash
# Round-4: Horner angle sums on block-wide tiles. Parity tests (fused == split bitwise, C3 full
# size vs the exact kernel, oracle rows), then the A/B against the previous library on C3 / C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/horner_tests.log 2>&1
rc=$?; tail -3 gpurun_out/horner_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/horner_tests.log | head -20; exit $rc; }
LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c4 STEPS=50 LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
echo done
