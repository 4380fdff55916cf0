set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/valu_rates > gpurun_out/ub_valu.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1; echo "tests rc=$?" >> gpurun_out/gputests.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r03_c3_stats --output-format csv -- python3 bench.py --no-cpu --no-calib --steps 100 --warmup 10 > gpurun_out/prof_c3.log 2>&1 || exit 1
echo done
