#!/bin/bash
# Round-6 A/B on the GPU box: bitwise tests of the fused path (unless NOTESTS), then LIBS for each
# config in CONFIGS (tools/gpu_lib_ab.sh: base = libdhcos.so, X = libdhcos_X.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
TAG=${TAG:-r6ab}
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_fullsize.py::test_c3_request_full_size tests/test_gpu_fullsize.py::test_c4_request_fused_split_bitwise \
    "tests/test_gpu_parity.py::test_fused_equals_split_bitwise" tests/test_gpu_fullsize.py::test_c3_objective_and_fd_gradient_match_oracle \
    ${EXTRA_TESTS} > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
fi
for c in ${CONFIGS:-c3 c2}; do
  LIBS="${LIBS:-head base}" CONFIG=$c bash tools/gpu_lib_ab.sh || exit 1
done
