#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the GPU box: for each NAME (or "base", the
# in-tree build), put it in place, run the extraction parity tests, then a bench pass with the stage
# times.  The in-tree library is restored at the end.
set -u
O=gpurun_out/vab; mkdir -p $O
LIB=orb-slam3_byzyh_amd/lib/liborbgpu.so
cp $LIB $O/base.so
status=0
for v in "$@"; do
  if [ "$v" = base ]; then cp $O/base.so $LIB; else cp build/var/$v/liborbgpu.so $LIB; fi
  if ! timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1; then
    echo "$v: tests failed"; tail -30 $O/t_$v.log; status=1; break
  fi
  echo "$v: $(tail -1 $O/t_$v.log)"
  for rep in 1 2; do
    if ! timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --steps 30 > $O/b_$v.json 2>$O/b_$v.err; then
      echo "$v: bench failed"; tail $O/b_$v.err; status=1; break 2
    fi
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['single_batch_ms'], d['stages_ms'])" $O/b_$v.json $v
  done
done
cp $O/base.so $LIB
exit $status
