#!/bin/bash
# A/B of several builds of libdhcos.so (LIBS="name ..." -> dhcos/libdhcos_<name>.so; "new" is the
# working tree's libdhcos.so), bench lines without the CPU and calibration legs, alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
D=option-pricing-ffn-lbfgs_amd/dhcos
for c in ${CONFIGS:-c1 c2 c3}; do
  if [ $c = c5 ]; then ST="--steps 5 --warmup 1"; elif [ $c = c4 ]; then ST="--steps 50 --warmup 5"; else ST="--steps 300"; fi
  for rep in 1 2; do for lib in ${LIBS:-base new}; do
    if [ $lib = new ]; then L=$PWD/$D/libdhcos.so; else L=$PWD/$D/libdhcos_$lib.so; fi
    DHCOS_LIB=$L timeout -k 10 200 python bench.py --config $c $ST --no-cpu --no-calib > gpurun_out/ab_${c}_$lib.log 2>&1 || { echo "bench $c $lib failed"; tail -3 gpurun_out/ab_${c}_$lib.log; exit 1; }
    python - gpurun_out/ab_${c}_$lib.log $c $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]} {sys.argv[3]:6s} step {d['ms_per_step']*1e3:9.2f} us  kernel {r['kernel_ms']*1e3:9.2f} us  frac {r['frac']}")
PY
  done; done
done
