#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of one config's request (separate --pmc passes), for the library in
# $DHCOS_LIB (default libdhcos.so): TAG=x CONFIG=c3 tools/gpu_r6_traffic.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-tr}; CONFIG=${CONFIG:-c3}
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/prof -o ${TAG}_${CONFIG}_$c --output-format csv \
      -- python bench.py --config $CONFIG --steps 20 --warmup 3 --no-cpu --no-calib --no-side > gpurun_out/prof/${TAG}_${CONFIG}_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  rm -f gpurun_out/prof/${TAG}_${CONFIG}_${c}_kernel_trace.csv
  python3 - <<PY
import csv, collections
v=collections.defaultdict(float)
for r in csv.DictReader(open('gpurun_out/prof/${TAG}_${CONFIG}_${c}_counter_collection.csv')):
    if 'cos_fused' in r['Kernel_Name'] or 'loss_partials' in r['Kernel_Name']:
        v[r['Dispatch_Id']] += float(r['Counter_Value'])
x=sorted(v.values()); print('${TAG} ${CONFIG} ${c} KiB median', x[len(x)//2] if x else None)
PY
done
