#!/bin/bash
# Kernel trace of a short pipelined bench run (which kernels overlap the vote grids).
#   TAG=r04s bash tools/gpu_trace_bench.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o bench -- python3 -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 --profile-steps 1 > "$OUT/trace.log" 2>&1
echo ok > "$OUT/ok"
