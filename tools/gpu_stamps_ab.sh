#!/bin/bash
# Phase stamps of C3 (fused) for the in-tree stamps build and libdhcos_stamps_prev.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in prev cur; do
  lib=option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_stamps.so; [ $v = prev ] && lib=option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_stamps_prev.so
  echo "== $v"; STAMPS_LIB=$PWD/$lib timeout -k 10 120 python tools/stamps.py --config ${CONFIG:-c3} --path 2 2>&1 | grep -v amdgpu.ids || exit 1
done
