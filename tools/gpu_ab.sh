#!/bin/bash
# GPU tests, then split vs fused request kernels on c1/c2/c3 (bench lines summarised).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for c in c1 c2 c3; do for p in split fused; do
timeout -k 10 200 python bench.py --config $c --path $p --no-cpu --no-calib --steps 200 > gpurun_out/b_${c}_$p.log 2>&1 || exit 1
python - $c $p <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b_{sys.argv[1]}_{sys.argv[2]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "%.3e"%d["value"], "%.4f ms"%d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"])
PY
done; done
