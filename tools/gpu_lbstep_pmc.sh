#!/bin/bash
# PMC counters of the device L-BFGS step kernel (one pass, SQ block only) on the c2 calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
mkdir -p gpurun_out/lbpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
   --kernel-include-regex lb_step --output-format csv -d gpurun_out/lbpmc -o c2 \
   -- python tools/calib_profile.py --config c2 --driver device > gpurun_out/lbpmc/c2.log 2>&1 || { tail -5 gpurun_out/lbpmc/c2.log; exit 1; }
f=$(find gpurun_out/lbpmc -name "c2_counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    v.sort()
    print(f"{k:20s} n {len(v):5d} median {v[len(v)//2]:12.1f} mean {sum(v)/len(v):12.1f}")
PY
