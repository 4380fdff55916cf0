#!/bin/bash
# calibrate(300, starts) medians per optimizer driver and environment variant on the bench
# surfaces.  VARIANTS: driver[:VAR=val,VAR=val] items, e.g. "scipy scipy:DHCOS_NATIVE_LOOP=0
# device" (the default; scipy with the Python request loop in the middle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/caldrv
for c in ${CONFIGS:-c1 c2 c3}; do for v in ${VARIANTS:-scipy scipy:DHCOS_NATIVE_LOOP=0 device}; do
  drv=${v%%:*}; envs=""; [ "$v" != "$drv" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  tag=$(echo "$v" | tr '=,:/.' '_____')
  env $envs timeout -k 10 200 python tools/calib_profile.py --config $c --driver $drv ${CAL_ARGS} > gpurun_out/caldrv/${c}_$tag.log 2>&1 || { tail -5 gpurun_out/caldrv/${c}_$tag.log; exit 1; }
  echo "== $c $v: $(grep -E 'driver:' gpurun_out/caldrv/${c}_$tag.log)"; grep -E "median" gpurun_out/caldrv/${c}_$tag.log
done; done
