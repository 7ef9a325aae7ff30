set -u
O=gpurun_out/c3ab; mkdir -p $O
EX="--no-cpu-baseline --no-ba --no-pose --no-bow --no-single --no-c4 --no-matchers"
for h in 1 3 1 3; do
  ORB_C3_INFLIGHT=$h timeout -k 10 300 python3 bench.py $EX > $O/h$h.json 2> $O/h$h.err || { echo fail; tail -5 $O/h$h.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1])
print('c3 sets=$h', d['c3_chain']['keyframes_per_ms'], 'chain batch', d['tracking_chain']['batch_api']['frames_per_ms'], d['tracking_chain']['batch_api']['ms_per_call'])"
done
