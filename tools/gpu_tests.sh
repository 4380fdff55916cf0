#!/bin/bash
# GPU test pass, run ON THE GPU BOX (gpurun): smoke(), then `pytest -m gpu` (one process, per-test
# time limit), logs under gpurun_out/.  TESTS= narrows the files.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 ${BUDGET:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
