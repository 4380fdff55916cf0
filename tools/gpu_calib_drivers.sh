#!/bin/bash
# calibrate(300, starts) medians for both optimizer drivers on the bench surfaces; scipy_py is the
# SciPy driver with the Python request loop (DHCOS_NATIVE_LOOP=0) instead of the native one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/caldrv
for c in ${CONFIGS:-c1 c2 c3}; do for d in ${DRIVERS:-scipy scipy_py device}; do
  drv=${d%_py}; nl=1; [ "$d" = scipy_py ] && nl=0
  DHCOS_NATIVE_LOOP=$nl timeout -k 10 200 python tools/calib_profile.py --config $c --driver $drv ${CAL_ARGS} > gpurun_out/caldrv/${c}_$d.log 2>&1 || { tail -5 gpurun_out/caldrv/${c}_$d.log; exit 1; }
  echo "== $c $d: $(grep -E 'driver:' gpurun_out/caldrv/${c}_$d.log)"; grep -E "median" gpurun_out/caldrv/${c}_$d.log
done; done
