#!/bin/bash
# C3 with the separate prologue kernel ahead of the fused kernel (libdhcos_pk2048.so): the two
# kernels' durations (rocprofv3 kernel trace) against the default library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pk
for v in base pk2048; do
  if [ $v = base ]; then unset DHCOS_LIB; else export DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pk -o $v --output-format csv -- python bench.py --config c3 --no-cpu --no-calib --no-side --steps 100 --warmup 10 > gpurun_out/pk/$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/pk/$v.log; exit 1; }
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/pk/${v}_kernel_stats.csv')):
    if 'fused' in r['Name'] or 'prologue' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
