#!/bin/bash
# Round-end measurement on the GPU box: bench (default config), rocprofv3 kernel stats of bench,
# PMC traffic passes.  Outputs under gpurun_out/round/.
set -u
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/stats.log 2>&1 || { echo "stats failed"; exit 1; }
tools/pmc_run.sh $O/pmc "--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4" || { echo "pmc failed"; exit 1; }
echo "round profile done"
