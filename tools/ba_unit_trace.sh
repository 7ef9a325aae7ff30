#!/bin/bash
# Per-kernel durations of the LocalBA unit (C5), one rocprofv3 kernel trace per variant, in one GPU call:
#   tools/ba_unit_trace.sh [VAR=value ...]   (each argument: one variant besides the default)
# Prints the median duration of every unit kernel over the live trials (gated no-op launches, under
# 3 us for the Cholesky, excluded) for each variant.  Outputs under gpurun_out/baunit/.
set -u
export TMPDIR=/tmp
O=gpurun_out/baunit
mkdir -p $O
i=0
for v in default "$@"; do
  if [ "$v" = default ]; then
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/v$i -o ba -- python3 tools/ba_time.py --gpu-only > $O/v$i.log 2>&1 || { echo "trace $v failed"; tail -5 $O/v$i.log; exit 1; }
  else
    export "$v"
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/v$i -o ba -- python3 tools/ba_time.py --gpu-only > $O/v$i.log 2>&1 || { echo "trace $v failed"; tail -5 $O/v$i.log; exit 1; }
    unset "${v%%=*}"
  fi
  echo "== $v"; grep stereo $O/v$i.log
  python3 tools/ba_unit_summary.py $O/v$i/ba_kernel_trace.csv
  i=$((i + 1))
done
