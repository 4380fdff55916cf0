#!/bin/bash
# PMC A/B of library variants on C3: VALU instructions and wave stall counters per request kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/pmcab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for v in ${LIBS:-base}; do
  unset DHCOS_MT_TB DHCOS_LIB
  lib=${v%%:*}; opt=""; [ "$lib" != "$v" ] && opt=${v#*:}
  case $lib in base) ;; mt*) opt=$lib ;; *) export DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_$lib.so ;; esac
  case $opt in mt*) export DHCOS_MT_TB=${opt#mt} ;; esac
  tag=${v/:/_}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $OUT -o ${tag} --output-format csv \
      -- python3 bench.py --no-cpu --no-calib --no-side --steps 10 --warmup 2 > $OUT/${tag}.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "$v ok"
done
echo done
