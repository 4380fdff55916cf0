#!/bin/bash
# Step-kernel phase stamps (tools/lbstep_stamps.py) for the stamps build of HEAD ("old", built into
# dhcos/libdhcos_stampsold.so), of the working tree ("new") and of variants ("x": libdhcos_stamps_x.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for c in ${CONFIGS:-c1 c2}; do for v in ${VERSIONS:-old new}; do
  case $v in
    old) export STAMPS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_stampsold.so ;;
    new) unset STAMPS_LIB ;;
    *) export STAMPS_LIB=$PWD/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_stamps_$v.so ;;
  esac
  timeout -k 10 120 python tools/lbstep_stamps.py --config $c > gpurun_out/lbst_${c}_$v.log 2>&1 || { tail -5 gpurun_out/lbst_${c}_$v.log; exit 1; }
  echo "== $c $v"; grep -v amdgpu.ids gpurun_out/lbst_${c}_$v.log
done; done
