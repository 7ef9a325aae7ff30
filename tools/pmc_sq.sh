#!/bin/bash
# SQ counter passes (separate rocprofv3 runs, kernel trace only) over a short extraction bench.
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/sq}; mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O -o pass$i -- python3 bench.py $ARGS > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O $O/summary.json
