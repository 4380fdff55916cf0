#!/bin/bash
# A/B of library variants on one box: LIBS="base g5 ..." CONFIG=c3 tools/gpu_lib_ab.sh
# (base = libdhcos.so, X = libdhcos_X.so); two alternations, ms_per_step and kernel_ms per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
CONFIG=${CONFIG:-c3}
for rep in 1 2; do
  for v in ${LIBS:-base}; do
    unset DHCOS_LIB
    [ "$v" != base ] && export DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_$v.so
    timeout -k 10 120 python3 bench.py --config $CONFIG --path ${BPATH:-auto} --no-cpu --no-calib --no-side --steps ${STEPS:-200} --warmup 20 \
        > gpurun_out/ab/${CONFIG}_${v}_$rep.json 2> gpurun_out/ab/${CONFIG}_${v}_$rep.err || { echo "$v failed"; tail -3 gpurun_out/ab/${CONFIG}_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab/${CONFIG}_${v}_$rep.json').read().strip().splitlines()[-1])
print('$CONFIG $v rep $rep', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_ms']*1e3,2), 'us kernel')"
  done
done
