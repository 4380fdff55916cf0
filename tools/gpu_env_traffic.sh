#!/bin/bash
# Fetched bytes (the L2's read requests by size) and WRITE_SIZE of one config's request under each
# environment variant: VARIANTS="DHCOS_XCD_REMAP=1 DHCOS_XCD_REMAP=2" CONFIG=c3 tools/gpu_env_traffic.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
CONFIG=${CONFIG:-c3}
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for v in ${VARIANTS:-base}; do
  envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
  tag=et_$(echo "$v" | tr '=,/.' '____')
  for grp in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE"; do
    g=$(echo $grp | cut -c1-12)
    export $envs
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/prof -o ${tag}_${CONFIG}_$g --output-format csv \
        -- python3 bench.py --config $CONFIG --steps 20 --warmup 3 --no-cpu --no-calib --no-side \
        > gpurun_out/prof/${tag}_${CONFIG}_$g.log 2>&1 || { echo "pmc $v $g failed"; exit 1; }
    for e in $envs; do unset ${e%%=*}; done
    rm -f gpurun_out/prof/${tag}_${CONFIG}_${g}_kernel_trace.csv
    python3 - <<PY
import csv, collections
size = {'TCC_EA0_RDREQ_32B_sum': 32, 'TCC_EA0_RDREQ_64B_sum': 64, 'TCC_EA0_RDREQ_128B_sum': 128}
v = collections.defaultdict(float)
for r in csv.DictReader(open('gpurun_out/prof/${tag}_${CONFIG}_${g}_counter_collection.csv')):
    if 'cos_fused' in r['Kernel_Name']:
        v[r['Dispatch_Id']] += float(r['Counter_Value']) * size.get(r['Counter_Name'], 1024)
x = sorted(v.values())
print('$v ${CONFIG} $g bytes per request (median)', x[len(x) // 2] if x else None)
PY
  done
done
