#!/bin/bash
# Round-end measurement on the GPU box: bench (default config), rocprofv3 kernel stats + trace of the
# extraction bench (the stage kernels' averages over the bench's instrumented pass are compared with
# bench.py's roofline.kernels[*].launch_avg_us), PMC traffic passes.  Outputs under gpurun_out/round/.
set -u
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers"
timeout -k 10 400 python3 bench.py --launch-dump $O/launch_durations.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 bench.py $EX --launch-dump $O/stats_launch_durations.json > $O/stats_bench.json 2> $O/stats.log || { echo "stats failed"; exit 1; }
# the last 20 steps' dispatches = bench.py's instrumented pass (the roofline's per-launch durations)
: > $O/timed_kernel_avg.txt
for kp in "k_pyramid_level 8" "k_fast_cells 2" "k_quadtree_kp 1" "k_describe 1"; do
  python3 tools/timed_kernel_avg.py $O/stats/bench_kernel_trace.csv 20 $kp >> $O/timed_kernel_avg.txt || exit 1
done
tools/pmc_run.sh $O/pmc "--steps 3 --warmup 1 $EX" || { echo "pmc failed"; exit 1; }
echo "round profile done"
