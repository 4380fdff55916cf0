#!/bin/bash
# Round-6 fused-kernel changes on the GPU box: the bitwise tests of the fused path, then A/B of the
# committed library (libdhcos_head.so) against the working one, and of the new switches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
TAG=${TAG:-r6k}
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_fullsize.py::test_c3_request_full_size tests/test_gpu_fullsize.py::test_c4_request_fused_split_bitwise \
    "tests/test_gpu_parity.py::test_fused_equals_split_bitwise" tests/test_gpu_fullsize.py::test_c3_objective_and_fd_gradient_match_oracle \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
fi
LIBS="head base" CONFIG=c3 bash tools/gpu_lib_ab.sh || exit 1
VARIANTS="base DHCOS_DEFER=1" CONFIG=c3 bash tools/gpu_env_ab.sh || exit 1
LIBS="head base" CONFIG=c2 bash tools/gpu_lib_ab.sh || exit 1
VARIANTS="base DHCOS_XCD_REMAP=0" CONFIG=c2 bash tools/gpu_env_ab.sh || exit 1
LIBS="head base" CONFIG=c1 bash tools/gpu_lib_ab.sh || exit 1
