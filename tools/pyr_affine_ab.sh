#!/bin/bash
# A/B of the pyramid's frame-affine XCD mapping (ORBGPU_PYR_AFFINE): extraction parity, alternating
# C2 benches, and a FETCH_SIZE pass each.  tools/pyr_affine_ab.sh [pmc]  (pmc: the counter passes only)
set -u
export TMPDIR=/tmp
O=gpurun_out/paff; mkdir -p $O
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
if [ "${1:-}" != pmc ]; then
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_workloads_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for a in 1 0; do
  ORBGPU_PYR_AFFINE=$a timeout -k 10 200 python bench.py $EX > $O/b.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('affine', sys.argv[2], d['value'], d['ms_per_step'], d.get('stages_ms'))" $O/b.json $a
done; done
fi
for a in 1 0; do
  ORBGPU_PYR_AFFINE=$a ORB_BENCH_SETTLE_MS=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc$a -o p -- python3 bench.py --steps 3 --warmup 1 $EX > $O/pmc$a.log 2>&1 || exit 1
done
echo done
