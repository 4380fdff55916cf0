#!/bin/bash
# Full bench lines (CPU baseline included) for every config -> gpurun_out/bench_<cfg>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for c in ${CONFIGS:-c2 c1 c3 c4 c5}; do
  if [ $c = c5 ]; then ST="--steps 5 --warmup 1"; elif [ $c = c4 ]; then ST="--steps 50 --warmup 5"; else ST=""; fi
  timeout -k 10 400 python bench.py --config $c $ST > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log > gpurun_out/bench_$c.json
  python - gpurun_out/bench_$c.json $c <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; c = d.get("calibration", {})
print(sys.argv[2], f"value {d['value']:.3e} {d['unit']}  step {d['ms_per_step']*1e3:.1f} us  frac {r['frac']}  basis {r.get('flop_basis', '')[:20]}  "
      f"cpu {d.get('cpu_baseline', {}).get('value', 0):.0f}/s x{d.get('cpu_baseline', {}).get('cores')}  calib {c.get('seconds', 0)*1e3:.1f} ms")
PY
done
