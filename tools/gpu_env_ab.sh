#!/bin/bash
# A/B of environment settings on one box: VARIANTS="DHCOS_AHEAD=0 DHCOS_AHEAD=1" CONFIG=c3
# tools/gpu_env_ab.sh (each variant: space-free VAR=VALUE[,VAR=VALUE]; "base" = none); REPS
# alternations, ms_per_step and kernel_ms per run (bench.py without the CPU / calibration legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
CONFIG=${CONFIG:-c3}
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    out=gpurun_out/ab/${CONFIG}_$(echo "$v" | tr '=,/.' '____')_$rep
    timeout -k 10 150 env $envs python3 bench.py --config $CONFIG --no-cpu --no-calib --no-side \
        --steps ${STEPS:-200} --warmup 20 > $out.json 2> $out.err || { echo "$v failed"; tail -3 $out.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$out.json').read().strip().splitlines()[-1])
print('$CONFIG $v rep $rep', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_ms']*1e3,2), 'us kernel')"
  done
done
