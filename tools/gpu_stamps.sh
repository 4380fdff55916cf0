#!/bin/bash
# Phase stamps (diagnostic build) of the request kernels on c1/c2/c3, fused and split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for c in ${CONFIGS:-c1 c2 c3}; do for p in ${PATHS:-2 1}; do
  timeout -k 10 120 python tools/stamps.py --config $c --path $p ${STAMP_ARGS} > gpurun_out/stamps_${c}_$p.log 2>&1 || exit 1
  cat gpurun_out/stamps_${c}_$p.log
done; done
