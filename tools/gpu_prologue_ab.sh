#!/bin/bash
# A/B of the prologue-kernel builds on C4 with per-kernel rocprofv3 stats (LIBS: libdhcos_<name>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/pab
D=$PWD/option-pricing-ffn-lbfgs_amd/dhcos
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
for lib in ${LIBS:-base pl1}; do
  L=$D/libdhcos_$lib.so; [ $lib = new ] && L=$D/libdhcos.so
  DHCOS_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pab -o $lib --output-format csv \
    -- python bench.py --config c4 --steps 50 --warmup 5 --no-cpu --no-calib > gpurun_out/pab/$lib.log 2>&1 || { echo "$lib failed"; exit 1; }
  echo "== $lib"; cut -d, -f1-4 gpurun_out/pab/${lib}_kernel_stats.csv | grep -E "prologue|fused" | sed 's/(double const\*.*",/",/'
done
