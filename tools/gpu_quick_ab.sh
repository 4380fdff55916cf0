#!/bin/bash
# Quick A/B of the in-tree library against libdhcos_prev.so on C3 (and C4): two alternations each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1
[ -n "$C4" ] && { CONFIG=c4 STEPS=50 LIBS="prev base" bash tools/gpu_lib_ab.sh || exit 1; }
echo done
