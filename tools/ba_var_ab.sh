#!/bin/bash
# A/B of LocalBA library variants (tools/build_variant.sh) on the GPU box: BA parity tests and the
# solve timing (tools/ba_time.py) per variant, alternating; the in-tree library is restored at the end.
#   tools/ba_var_ab.sh base kt64 ...
set -u
O=gpurun_out/bvab; mkdir -p $O
LIB=orb-slam3_byzyh_amd/lib/liborbgpu.so
cp $LIB $O/base.so
status=0
for v in "$@"; do
  if [ "$v" = base ]; then cp $O/base.so $LIB; else cp build/var/$v/liborbgpu.so $LIB; fi
  if ! timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1; then
    echo "$v: tests failed"; tail -20 $O/t_$v.log; status=1; break
  fi
  echo "$v: $(tail -1 $O/t_$v.log)"
  timeout -k 10 120 python3 tools/ba_time.py --gpu-only > $O/time_$v.txt 2>&1 || { echo "$v: timing failed"; status=1; break; }
  echo "$v: $(grep 'stereo 0.0' $O/time_$v.txt)"
done
cp $O/base.so $LIB
exit $status
