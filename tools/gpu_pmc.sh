#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, kernel-trace only, no sys/runtime trace)
# over a short bench run; outputs under gpurun_out/pmc/<tag>_pN.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmc}
ARGS=${ARGS:-"--no-cpu --no-calib --steps 50 --warmup 5"}
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc -o ${TAG}_p$i \
      --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<EOG
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE}
EOG
