#!/bin/bash
# stereo line at several extractor-set counts (ORB_STEREO_SETS), alternating, two
# passes: gpurun_out/stereo_sets/sweep.txt
set -u
O=gpurun_out/stereo_sets; mkdir -p $O
: > $O/sweep.txt
EX="--no-cpu-baseline --no-ba --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
for pass in 1 2; do
  for h in ${@:-1 2 3}; do
    ORB_STEREO_SETS=$h timeout -k 10 200 python3 bench.py $EX > $O/h$h.json 2> $O/h$h.err || { echo "$h failed"; tail -5 $O/h$h.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1])
c=d['stereo']; print('sets=$h', c.get('stereo_frames_per_ms'), c.get('ms_per_step'), c.get('error'))" | tee -a $O/sweep.txt
  done
done
