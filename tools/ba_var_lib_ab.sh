#!/bin/bash
# A/B of LocalBA library variants (tools/build_variant.sh -> vars/NAME/liborbgpu.so) on the GPU box:
# for each NAME (or "base", the in-tree build) put it in place, run the BA parity tests, then
# tools/ba_time.py --gpu-only twice, alternating the variants.  The in-tree library is restored.
#   tools/ba_var_lib_ab.sh base NAME [NAME ...]
set -u
O=gpurun_out/bavar; mkdir -p $O
LIB=orb-slam3_byzyh_amd/lib/liborbgpu.so
cp $LIB $O/base.so
status=0
put() { if [ "$1" = base ]; then cp $O/base.so $LIB; else cp vars/$1/liborbgpu.so $LIB; fi; }
for v in "$@"; do
  put $v
  if ! timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1; then
    echo "$v: tests failed"; tail -30 $O/t_$v.log; status=1; break
  fi
  echo "$v: $(tail -1 $O/t_$v.log)"
done
if [ $status = 0 ]; then
  for rep in 1 2; do
    for v in "$@"; do
      put $v
      timeout -k 10 120 python3 tools/ba_time.py --gpu-only > $O/time_${v}_$rep.txt 2>&1 || { cat $O/time_${v}_$rep.txt; status=1; break 2; }
      echo "$v run $rep"; grep stereo $O/time_${v}_$rep.txt
    done
  done
fi
cp $O/base.so $LIB
exit $status
