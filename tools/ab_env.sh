#!/bin/bash
# A/B of an extraction env switch on the GPU box: bench (extraction only) with and without it.
#   tools/ab_env.sh VAR=value [VAR2=value ...]
set -u
ARGS="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers"
for i in 1 2; do
  timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab_base$i.json 2>/dev/null || exit 1
  timeout -k 10 120 env "$@" python3 bench.py $ARGS > gpurun_out/ab_var$i.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for tag in ("base", "var"):
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/ab_{tag}{i}.json"))
        print(tag, i, d["value"], d["ms_per_step"], d["stages_ms"], d["roofline"]["launch_avg_us"])
PY
