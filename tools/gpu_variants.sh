#!/bin/bash
# GPU tests on the default library, then request time (HIP events) of each library variant on
# each config:  LIBS="libdhcos.so libdhcos_ilp1.so" CONFIGS="c2 c3 c5" bash tools/gpu_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
D=option-pricing-ffn-lbfgs_amd/dhcos
for c in ${CONFIGS:-c2 c3 c5}; do for lib in ${LIBS:-libdhcos.so}; do for p in ${PATHS:-auto}; do
  if [ $c = c5 ]; then ST="--steps 5 --warmup 1"; else ST="--steps 200"; fi
  DHCOS_LIB=$PWD/$D/$lib timeout -k 10 300 python bench.py --config $c --path $p --no-cpu --no-calib $ST \
    > gpurun_out/v_${c}_${lib}_$p.log 2>&1 || { echo "fail $c $lib $p"; tail -5 gpurun_out/v_${c}_${lib}_$p.log; exit 1; }
  python - gpurun_out/v_${c}_${lib}_$p.log $c $lib $p <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]} {sys.argv[3]:22s} {sys.argv[4]:5s} value {d['value']:.3e}  step {d['ms_per_step']*1e3:9.1f} us  "
      f"request {r['kernel_ms']*1e3:9.1f} us  frac {r['frac']:.4f}  {r['kernel']}")
PY
done; done; done
