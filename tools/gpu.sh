#!/bin/bash
# Build locally (abort on failure), then run the given command on the MI355X box via gpurun.
#   tools/gpu.sh [--timeout S] -- 'command'
set -e
cd "$(dirname "$0")/.."
TO=900
if [ "$1" = "--timeout" ]; then TO=$2; shift 2; fi
[ "$1" = "--" ] && shift
make -s -j8 > /tmp/gpu_build.log 2>&1 || { echo "BUILD FAILED"; grep -E 'error' -A3 /tmp/gpu_build.log | head -30; exit 1; }
mkdir -p gpurun_out
exec /usr/local/graft/bin/gpurun --timeout "$TO" -- "$1"
