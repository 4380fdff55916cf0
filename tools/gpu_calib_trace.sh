cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ctrace
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ctrace -o c2dev -- python tools/calib_profile.py --config c2 --driver device > gpurun_out/ctrace/c2dev.log 2>&1 || exit 1
f=$(find gpurun_out/ctrace -name "c2dev_kernel_trace.csv" | head -1)
python tools/trace_gaps.py $f
