#!/bin/bash
# Round-end measurement on the GPU box: bench (default config), rocprofv3 kernel stats + trace of the
# extraction bench (its timed-region k_pyramid_level average is compared with bench.py's
# roofline.launch_avg_us), PMC traffic passes.  Outputs under gpurun_out/round/.
set -u
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers"
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 bench.py $EX > $O/stats_bench.json 2> $O/stats.log || { echo "stats failed"; exit 1; }
python3 tools/timed_kernel_avg.py $O/stats/bench_kernel_trace.csv 20 > $O/timed_kernel_avg.txt || exit 1
tools/pmc_run.sh $O/pmc "--steps 3 --warmup 1 $EX" || { echo "pmc failed"; exit 1; }
echo "round profile done"
