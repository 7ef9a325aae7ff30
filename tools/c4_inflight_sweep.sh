#!/bin/bash
# C2 / C4 shard / C4 strong at several --in-flight values, alternating, two passes:
# gpurun_out/c4_inflight/sweep.txt
set -u
O=gpurun_out/c4_inflight; mkdir -p $O
: > $O/sweep.txt
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-matchers --no-chain"
for pass in 1 2; do
  for h in ${@:-3 4 6 8}; do
    timeout -k 10 200 python3 bench.py $EX --in-flight $h > $O/h$h.json 2> $O/h$h.err || { echo "in-flight $h failed"; tail -5 $O/h$h.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1])
c4=d.get('c4_shard') or {}; cs=d.get('c4_strong') or {}
print('in_flight=$h', 'C2', d['value'], 'c4_shard', c4.get('features_per_ms'), 'c4_strong', cs.get('features_per_ms'))" | tee -a $O/sweep.txt
  done
done
