#!/bin/bash
# Round profile set, run ON THE GPU BOX (gpurun):  TAG=r01 tools/gpu_profile.sh
#   1) rocprofv3 --kernel-trace --stats of the bench (per config, calibration leg off so every
#      COS launch has the bench's request shape);
#   2) PMC passes, one counter group per run, kernel-trace only (never with sys/runtime trace):
#      FETCH_SIZE / WRITE_SIZE (separate passes, MI355X_MICROARCH.md), the fp64 instruction mix, and
#      the L2's read requests by size (32 / 64 / 128 B: the fetched bytes exactly, for access widths
#      the FETCH_SIZE x 2 correction is not calibrated for) and those that reached DRAM.
# Outputs under gpurun_out/prof/; tools/summarize_profiles.py turns them into profiles/<TAG>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r01}
CONFIGS=${CONFIGS:-"c2 c3 c5"}
OUT=gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for c in $CONFIGS; do
  if [ $c = c5 ]; then STEPS="--steps 3 --warmup 1"; PSTEPS="--steps 1 --warmup 1"; else STEPS="--steps 100 --warmup 10"; PSTEPS="--steps 20 --warmup 3"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o ${TAG}_${c}_stats --output-format csv \
      -- python bench.py --config $c $STEPS --no-cpu --no-calib --no-side \
      > $OUT/${TAG}_${c}_stats.log 2>&1 || { echo "stats $c failed rc=$?"; exit 1; }
  echo "stats $c ok"
  i=0
  while IFS= read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT -o ${TAG}_${c}_pmc$i --output-format csv \
        -- python bench.py --config $c $PSTEPS --no-cpu --no-calib --no-side \
        > $OUT/${TAG}_${c}_pmc$i.log 2>&1 || { echo "pmc $c pass $i failed rc=$?"; exit 1; }
    echo "pmc $c pass $i ($grp) ok"
  done <<EOG
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU
TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum
EOG
done
echo done
