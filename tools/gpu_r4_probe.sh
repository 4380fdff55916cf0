#!/bin/bash
# Round-4 probe: the C3 request with and without the separate prologue kernel
# (libdhcos_pk.so: DH_PROLOGUE_KERNEL_MIN_BLOCKS=1024), kernel-trace stats and VALU counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/probe
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for v in base pk; do
  if [ $v = pk ]; then export DHCOS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_pk.so; else unset DHCOS_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o ${v}_stats --output-format csv \
      -- python3 bench.py --no-cpu --no-calib --no-side --steps 50 --warmup 5 > $OUT/${v}_stats.log 2>&1 || { echo "stats $v failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT -o ${v}_pmc --output-format csv \
      -- python3 bench.py --no-cpu --no-calib --no-side --steps 10 --warmup 2 > $OUT/${v}_pmc.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "$v ok"
done
echo done
