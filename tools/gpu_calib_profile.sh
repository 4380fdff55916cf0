#!/bin/bash
# Evidence for the device-resident L-BFGS-B: rocprofv3 kernel stats of calibrate(300, 3,
# driver="device") on c1/c2 (tools/calib_profile.py), the kernel-trace timeline summary
# (tools/trace_gaps.py) and the step kernel's phase stamps (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
OUT=gpurun_out/calprof
mkdir -p $OUT
for c in ${CONFIGS:-c1 c2}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o ${TAG:-r01}_calib_${c}_device \
      -- python tools/calib_profile.py --config $c --driver device > $OUT/${c}_device.log 2>&1 || { tail -5 $OUT/${c}_device.log; exit 1; }
  f=$(find $OUT -name "${TAG:-r01}_calib_${c}_device_kernel_trace.csv" | head -1)
  python tools/trace_gaps.py $f > $OUT/${c}_device_timeline.txt
  timeout -k 10 120 python tools/lbstep_stamps.py --config $c > $OUT/${c}_lbstep_stamps.txt 2>&1 || exit 1
  echo "== $c"; cat $OUT/${c}_device_timeline.txt $OUT/${c}_lbstep_stamps.txt
done
