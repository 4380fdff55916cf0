#!/bin/bash
# rocprofv3 kernel-trace stats of bench configs (per-kernel average durations).
#   CONFIGS="c1 c2" TAG=x bash tools/gpu_kstats.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for c in ${CONFIGS:-c1 c2}; do
  if [ $c = c5 ]; then ST="--steps 3 --warmup 1"; else ST="--steps 200 --warmup 20"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o ${TAG:-x}_${c} --output-format csv \
      -- python bench.py --config $c $ST --no-cpu --no-calib ${BENCH_ARGS} > $OUT/${TAG:-x}_${c}.log 2>&1 \
      || { echo "prof $c failed"; tail -5 $OUT/${TAG:-x}_${c}.log; exit 1; }
  f=$(ls $OUT/${TAG:-x}_${c}_kernel_stats.csv 2>/dev/null || find $OUT -name "${TAG:-x}_${c}_kernel_stats.csv" | head -1)
  echo "== $c"; python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "cos_" in r["Name"] or "loss" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1e3:9.2f} us  min {float(r["MinNs"])/1e3:9.2f}  max {float(r["MaxNs"])/1e3:9.2f}')
PY
  tail -1 $OUT/${TAG:-x}_${c}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('step us', d['ms_per_step']*1e3, 'request us', d['roofline']['kernel_ms']*1e3)"
done
