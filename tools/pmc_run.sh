#!/bin/bash
# Collect rocprofv3 PMC passes (separate runs, --kernel-trace only, no sys/runtime traces) for the
# bench's kernels.  Usage (on the GPU box): tools/pmc_run.sh OUTDIR "bench args"
set -u
OUT=${1:-gpurun_out/pmc}
ARGS=${2:---steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  ORB_BENCH_SETTLE_MS=0 timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d "$OUT" -o "pass$i" -- python3 bench.py $ARGS > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'PASSES'


FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
PASSES
echo "pmc done: $i passes"
