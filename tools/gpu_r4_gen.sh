#!/bin/bash
# Round-4 generator: the generator GPU tests, the API timeline, staged and API end-to-end times
# (tools/gen_profile.py), and the c5 bench line with its generator_end_to_end leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "generator or gen_ or price_cols" \
    > gpurun_out/gen_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gen_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/gen_api_timeline.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/gen_profile.py --out gpurun_out/r04_generator_e2e.json > gpurun_out/gen_profile.log 2>&1 \
    || { tail -5 gpurun_out/gen_profile.log; exit 1; }
cat gpurun_out/r04_generator_e2e.json
timeout -k 10 300 python bench.py --config c5 --no-cpu > gpurun_out/r04_c5.json 2> gpurun_out/r04_c5.err || { tail -5 gpurun_out/r04_c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04_c5.json').readline()); print(d['value'], d['ms_per_step'], d.get('generator_end_to_end'))"
