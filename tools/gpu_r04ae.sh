#!/bin/bash
# r04ae: pipelined pair A/B: default; fold levels on the per-vote stream (OVH_FOLD_SIDE=0);
# eight hardware queues per process.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04ae}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_default.log" 2>&1
OVH_FOLD_SIDE=0 timeout -k 10 240 $B > "$OUT/bench_foldmain.log" 2>&1
GPU_MAX_HW_QUEUES=8 timeout -k 10 240 $B > "$OUT/bench_q8.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_default2.log" 2>&1
echo ok > "$OUT/ok"
