#!/bin/bash
# Quick GPU check of a kernel change (run ON THE GPU BOX via gpurun): microbenchmarks, the
# full-size and parity GPU tests, and the C3 bench line without the CPU / calibration legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for u in ${UBENCH:-}; do
  timeout -k 10 60 ./tools/ubench/$u > gpurun_out/ub_$u.txt 2>&1 || { echo "ubench $u failed"; exit 1; }
done
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_fullsize.py tests/test_gpu_parity.py} -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
for c in ${CONFIGS:-c3}; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-calib --steps 200 --warmup 20 \
      > gpurun_out/quick_$c.json 2> gpurun_out/quick_$c.err || { echo "bench $c failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/quick_$c.json'));r=d['roofline'];print('$c', 'step_us', round(d['ms_per_step']*1e3,2), 'kernel_us', round(r['kernel_ms']*1e3,2), 'value', '%.4g'%d['value'])"
done
