#!/bin/bash
# Round-4 end check: the full -m gpu suite, smoke(), and the default bench line (as the driver runs them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gputests.log; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_final.json 2> gpurun_out/r04_bench_final.err || { tail -5 gpurun_out/r04_bench_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04_bench_final.json').readline())
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['c5_generator_n128']['generator_end_to_end']['seconds'])"
