#!/bin/bash
# Per-iteration time of calibrate(300, starts) for several builds (LIBS="name ..." ->
# dhcos/libdhcos_<name>.so, "new" = the working tree's), both drivers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/caldrv
D=$PWD/option-pricing-ffn-lbfgs_amd/dhcos
for c in ${CONFIGS:-c1 c2}; do for d in ${DRIVERS:-device scipy}; do for lib in ${LIBS:-base new}; do
  if [ $lib = new ]; then L=$D/libdhcos.so; else L=$D/libdhcos_$lib.so; fi
  DHCOS_LIB=$L timeout -k 10 200 python tools/calib_profile.py --config $c --driver $d ${CAL_ARGS} > gpurun_out/caldrv/${c}_${d}_$lib.log 2>&1 || { tail -5 gpurun_out/caldrv/${c}_${d}_$lib.log; exit 1; }
  echo "$c $d $lib: $(grep -E 'median of 7' gpurun_out/caldrv/${c}_${d}_$lib.log)"
done; done; done
