#!/bin/bash
# C2 knob sweep on the GPU box: alternating bench runs of the main line under environment settings.
#   tools/c2_knob_sweep.sh "ENV=.. ENV2=.." "..."   (each argument one setting; "-" = defaults)
set -u
O=gpurun_out/knobs; mkdir -p $O
EX="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
for r in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then envs=""; else envs="$cfg"; fi
    env $envs timeout -k 10 200 python bench.py $EX > $O/b.json 2>/dev/null || { echo "failed: $cfg"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b.json "$cfg"
  done
done
