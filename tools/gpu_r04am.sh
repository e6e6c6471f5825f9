#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04am}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_gate.log" 2>&1
OVH_GATE=0 timeout -k 10 240 $B > "$OUT/bench_nogate.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_gate2.log" 2>&1
OVH_GATE=0 timeout -k 10 240 $B > "$OUT/bench_nogate2.log" 2>&1
echo ok > "$OUT/ok"
