#!/bin/bash
# Batched tracking chain (bench.py's tracking_chain.batch_api) over frames per call (ORB_CHAIN_NB) and
# batch objects taking the calls in turn (ORB_CHAIN_NBUF); args NB:NBUF ...: gpurun_out/chain_sweep/sweep.txt
set -u
O=gpurun_out/chain_sweep; mkdir -p $O
: > $O/sweep.txt
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --steps 10"
for pass in 1 2; do
  for cfg in ${@:-256:1 256:2 512:1 512:2}; do
    nb=${cfg%:*}; nbuf=${cfg#*:}
    ORB_CHAIN_NB=$nb ORB_CHAIN_NBUF=$nbuf timeout -k 10 200 python3 bench.py $EX > $O/r_${nb}_${nbuf}.json 2> $O/r_${nb}_${nbuf}.err || { echo "$cfg failed"; tail -5 $O/r_${nb}_${nbuf}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/r_${nb}_${nbuf}.json').read().strip().splitlines()[-1])
b=d['tracking_chain']['batch_api']; print('nb=$nb nbuf=$nbuf', b['ms_per_call'], b['frames_per_ms'])" | tee -a $O/sweep.txt
  done
done
