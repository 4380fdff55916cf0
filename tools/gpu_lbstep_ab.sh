#!/bin/bash
# Device-driver step-kernel change check: GPU tests of the device L-BFGS-B and parity suites, then
# calibration per-iteration A/B (device driver) and bench A/B against dhcos/libdhcos_base.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_device_lbfgs.py tests/test_gpu_parity.py -m gpu > gpurun_out/t_lb.log 2>&1 || { tail -30 gpurun_out/t_lb.log; exit 1; }
tail -2 gpurun_out/t_lb.log
CONFIGS="${CONFIGS:-c1 c2}" DRIVERS=device bash tools/gpu_calib_ab.sh || exit 1
CONFIGS="${CONFIGS:-c1 c2}" bash tools/gpu_ab_libs.sh
