#!/bin/bash
# A/B of LLVM scheduler options (libdhcos_<variant>.so builds) on C3, C4, C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
V="base silp smem trk nohrp bias"
LIBS="$V" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c4 STEPS=50 LIBS="$V" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="$V" bash tools/gpu_lib_ab.sh || exit 1
