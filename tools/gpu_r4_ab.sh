#!/bin/bash
# Round-4 A/B of the multi-table kernel (tables per block), the big-tile option threads and G
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
LIBS="mt0 mt2 mt4 t128:mt0 t128:mt2 t128:mt4 g5" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c4 STEPS=50 LIBS="mt0 mt2 mt4 pk" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c1 LIBS="mt0 t128:mt0" bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="mt2 mt4" BPATH=mt bash tools/gpu_lib_ab.sh || exit 1
CONFIG=c2 LIBS="base" bash tools/gpu_lib_ab.sh || exit 1
echo done
