#!/bin/bash
# A GPU-box check run: the tests named in $TESTS, then the driver's bench command -> gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-chk}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS \
      > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json \
      2> gpurun_out/${TAG}_bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
  echo bench ok
fi
