#!/bin/bash
# GPU tests, then the bench's calibration leg (calibrate(300, 3), seed 0) on c1 and c2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-c1 c2}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 50 > gpurun_out/cal_$c.log 2>&1 || { tail -5 gpurun_out/cal_$c.log; exit 1; }
  python - gpurun_out/cal_$c.log $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["calibration"]
print(sys.argv[2], f"calibrate {c['seconds']*1e3:.1f} ms  launches {c['lockstep_launches_rank0']}  "
      f"per launch {c['seconds']/max(1,c['lockstep_launches_rank0'])*1e6:.0f} us  nit {c['iterations']}  "
      f"loss {c['final_loss']:.6e}  {c['message']}  | request {d['roofline']['kernel_ms']*1e3:.1f} us")
PY
done
