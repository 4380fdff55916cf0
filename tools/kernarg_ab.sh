#!/bin/bash
# A/B of HIP_FORCE_DEV_KERNARG (unset / 0 / 1) on the C2 and C1 bench requests, run ON THE GPU BOX.
cd "${GRAFT_REPO_ROOT}"
for rep in 1 2; do for v in unset 0 1; do
  if [ $v = unset ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$v"; fi
  for c in c2 c1; do
    env $E timeout -k 10 200 python bench.py --config $c --steps 300 --no-cpu --no-calib > gpurun_out/ka_${c}_$v.log 2>&1 || { echo fail; tail -3 gpurun_out/ka_${c}_$v.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ka_${c}_$v.log').read().strip().splitlines()[-1]); print('$c', '$v', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_ms']*1e3,2))"
  done
done; done
