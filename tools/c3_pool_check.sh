set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pool
timeout -k 10 400 python3 -u -m pytest tests/test_stereo_gpu.py tests/test_bow_gpu.py tests/test_matcher_gpu.py tests/test_chain_gpu.py tests/test_pose_gpu.py tests/test_projection_gpu.py tests/test_tracking_chain_gpu.py tests/test_concurrency_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pool/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pool/tests.log; exit 1; }
tail -1 gpurun_out/pool/tests.log
EX="--no-cpu-baseline --no-ba --no-pose --no-bow --no-single --no-c4 --no-matchers --no-chain"
for pass in 1 2; do for h in 1 2 3 4 5; do
  ORB_C3_INFLIGHT=$h timeout -k 10 200 python3 bench.py $EX > gpurun_out/pool/h$h.json 2> gpurun_out/pool/h$h.err || { echo "h$h failed"; tail -5 gpurun_out/pool/h$h.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/pool/h$h.json').read().strip().splitlines()[-1])
c=d['c3_chain']; s=d['stereo']; print('buffers=$h', c.get('keyframes_per_ms'), c.get('ms_per_step'), 'stereo', s.get('stereo_frames_per_ms'))"
done; done
