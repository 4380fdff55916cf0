#!/bin/bash
# A/B of the generator API's host-side choices: pinning, the dates thread, draw team size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for cfg in "all 1 16" "all 1 14" "all 1 12" "in 1 14" "out 1 14" "none 1 14" "all 0 14" "none 0 16"; do
  set -- $cfg
  DHCOS_GEN_PIN=$1 DHCOS_GEN_DATES_THREAD=$2 DHCOS_GEN_THREADS=$3 timeout -k 10 120 python tools/gen_profile.py --reps 7 > /tmp/g.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('/tmp/g.json')); print('pin=$1 dates_thread=$2 threads=$3', {k: round(d[k]*1e3,1) for k in ('draw','price','assemble','generate_synthetic_calibrations')})"
done
