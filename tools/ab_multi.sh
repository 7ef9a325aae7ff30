#!/bin/bash
# A/B of extraction env settings on the GPU box: the default and each variant, twice, interleaved.
#   tools/ab_multi.sh "VAR=1 VAR2=2" "VAR=3" ...
set -u
ARGS="--no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers"
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/abm_base_$rep.json 2>/dev/null || exit 1
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 120 env $v python3 bench.py $ARGS > gpurun_out/abm_v${i}_$rep.json 2>/dev/null || exit 1
  done
done
python3 - "$@" <<'PY'
import json, sys
names = ["base"] + [f"v{i}" for i in range(1, len(sys.argv))]
labels = ["(default)"] + sys.argv[1:]
for n, lab in zip(names, labels):
    vals = [json.load(open(f"gpurun_out/abm_{n}_{r}.json")) for r in (1, 2)]
    print(f"{lab:50s}", [v["value"] for v in vals], [v["ms_per_step"] for v in vals])
PY
