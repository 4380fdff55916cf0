#!/bin/bash
# One GPU session: parity tests, smoke, bench (+ occupancy variants), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT/prof
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -ge 128 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -s ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if fatal $rc; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; if fatal $rc; then exit $rc; fi
for v in ${VARIANTS}; do
  DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_$v.so timeout -k 10 200 \
    python bench.py --no-cpu --no-calib --steps 200 > $OUT/bench_$v.log 2>&1
  rc=$?; echo "bench $v rc=$rc"; if fatal $rc; then exit $rc; fi
done
if [ -n "${PROF}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ${PROF} --output-format csv \
    -- python bench.py --no-cpu --no-calib --steps 200 > $OUT/bench_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
fi
exit 0
