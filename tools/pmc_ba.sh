#!/bin/bash
# MFMA utilisation of the LocalBA (C5) solve: SQ counter passes (separate rocprofv3 runs, kernel trace
# only) over tools/ba_time.py --gpu-only.  Pass 1: the counter list the box offers (for the record).
# Outputs under $1 (default gpurun_out/pmc_ba); summary by tools/pmc_summary.py.
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_ba}; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
i=0
for set in "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS"; do
  i=$((i+1))
  keep=""
  for c in $set; do grep -qw "$c" $O/avail.txt && keep="$keep $c" || echo "pass $i: $c not offered, dropped"; done
  set=$keep
  [ -z "$set" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O -o pass$i -- python3 tools/ba_time.py --gpu-only > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
done
echo "pmc_ba done: $i passes"
