#!/bin/bash
# Round-4 multi-table kernel check: parity (bitwise vs fused / split, the 5x5 ensemble, lockstep),
# then A/B of tables per block (mt0 = single-table fused kernel) and the G-cap variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu \
    -k "fused_equals_split or 5x5 or lockstep" -v -s --timeout 240 --timeout-method thread \
    > gpurun_out/t_mt.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/t_mt.log; tail -3 gpurun_out/t_mt.log
[ $rc -eq 0 ] || exit $rc
LIBS="mt0 mt2 mt4 t128:mt0 t128:mt2 t128:mt4 g5" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c4 STEPS=50 LIBS="mt0 mt2 mt4 pk" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c1 LIBS="mt0 t128:mt0" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="mt2 mt4" BPATH=mt bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="base" bash tools/gpu_lib_ab.sh || exit 1
echo done
