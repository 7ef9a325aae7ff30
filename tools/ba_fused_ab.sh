#!/bin/bash
# LocalBA trial-fusion check on the GPU box: BA parity tests, then tools/ba_time.py --gpu-only with
# the fused trial (default) and ORBGPU_BA_FUSED_TRIAL=0 alternating, then kernel stats of the fused
# solve.  Outputs under gpurun_out/bafuse/.
set -u
export TMPDIR=/tmp
O=gpurun_out/bafuse
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_variants_gpu.py tests/test_ba_dist_gpu.py \
  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "BA tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/ba_time.py --gpu-only > $O/fused$i.txt 2>&1 || { cat $O/fused$i.txt; exit 1; }
  timeout -k 10 120 env ORBGPU_BA_FUSED_TRIAL=0 python3 tools/ba_time.py --gpu-only > $O/base$i.txt 2>&1 || { cat $O/base$i.txt; exit 1; }
done
for f in fused1 base1 fused2 base2; do echo "== $f"; cat $O/$f.txt; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o ba -- python3 tools/ba_time.py --gpu-only > $O/stats.log 2>&1 || { echo "stats failed"; tail -5 $O/stats.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/bafuse/stats/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:20]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
