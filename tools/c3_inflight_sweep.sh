#!/bin/bash
# C3 chain (bench.py's c3_chain) at several step-buffer counts (ORB_C3_INFLIGHT), alternating, two
# passes: gpurun_out/c3_inflight/sweep.txt
set -u
O=gpurun_out/c3_inflight; mkdir -p $O
: > $O/sweep.txt
EX="--no-cpu-baseline --no-ba --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
for pass in 1 2; do
  for h in ${@:-1 2 3}; do
    ORB_C3_INFLIGHT=$h timeout -k 10 200 python3 bench.py $EX > $O/h$h.json 2> $O/h$h.err || { echo "$h failed"; tail -5 $O/h$h.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1])
c=d['c3_chain']; print('buffers=$h', c.get('keyframes_per_ms'), c.get('ms_per_step'), c.get('matches_per_pair'), c.get('error'))" | tee -a $O/sweep.txt
  done
done
