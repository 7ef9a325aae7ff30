#!/bin/bash
# C3 chain step-buffer sweep (ORB_C3_INFLIGHT 1-5) under the default 4 hardware queues and under
# GPU_MAX_HW_QUEUES=8 / 16: if the non-monotonic curve is which streams share a hardware queue, more
# queues should flatten it.  gpurun_out/c3q/sweep.txt
set -u
O=gpurun_out/c3q; mkdir -p $O
: > $O/sweep.txt
EX="--no-cpu-baseline --no-ba --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
for q in 4 8 16; do
  for h in 1 2 3 4 5; do
    GPU_MAX_HW_QUEUES=$q ORB_C3_INFLIGHT=$h timeout -k 10 200 python3 bench.py $EX > $O/q${q}_h$h.json 2> $O/q${q}_h$h.err || { echo "q$q h$h failed"; tail -5 $O/q${q}_h$h.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/q${q}_h$h.json').read().strip().splitlines()[-1])
c=d['c3_chain']; print('queues=$q buffers=$h', c.get('keyframes_per_ms'), c.get('ms_per_step'))" | tee -a $O/sweep.txt
  done
done
