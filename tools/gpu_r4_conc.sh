#!/bin/bash
# Round-4: concurrent table prologues. Parity tests, then C3 / C4 under $DHCOS_PROLOGUE = 0 (in-block
# prologue), 1 (sequential prologue kernel), 2 (concurrent), two alternations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/conc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "concurrent or fused_equals_split or c3_ or c4_ or handoff" > gpurun_out/conc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/conc_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/conc_tests.log | head -20; exit $rc; }
for cfg in c3 c4; do for rep in 1 2; do for m in 0 1 2; do
  st=200; [ $cfg = c4 ] && st=50
  DHCOS_PROLOGUE=$m timeout -k 10 120 python3 bench.py --config $cfg --no-cpu --no-calib --no-side --steps $st --warmup 20 \
      > gpurun_out/conc/${cfg}_$m_$rep.json 2> gpurun_out/conc/${cfg}_${m}_$rep.err || { echo "$cfg $m failed"; tail -3 gpurun_out/conc/${cfg}_${m}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/conc/${cfg}_$m_$rep.json').read().strip().splitlines()[-1])
print('$cfg mode $m rep $rep', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_ms']*1e3,2), 'us kernel')"
done; done; done
