#!/bin/bash
# Round-4: SciPy-driver host path. Calibration GPU tests, then calibrate(300, 3) medians of both
# drivers on c1 c2 c3, and the host split of the SciPy driver (tools/scipy_host_split.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "lockstep or calibrate or fg" > gpurun_out/scipy_tests.log 2>&1
rc=$?; tail -3 gpurun_out/scipy_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_calib_drivers.sh || exit 1
for c in c1 c2 c3; do
  timeout -k 10 120 python tools/scipy_host_split.py --config $c --pipeline "${PIPE:-}" 2>&1 | grep -v amdgpu.ids || exit 1
done
echo done
