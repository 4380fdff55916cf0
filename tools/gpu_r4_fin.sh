#!/bin/bash
# Round-4: the full -m gpu suite, then A/B of the lane-parallel finalisation (base) against the
# previous library (libdhcos_prev.so) on C3 / C2 / C4, and the C3 PMC pass of both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gputests.log; tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c4 STEPS=50 LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
LIBS="prev base" bash tools/gpu_r4_pmc_ab.sh || exit 1
echo done
