#!/bin/bash
# r04aa: two vs three per-vote streams in turn (the next batch's grid waiting for the tail's slots).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_pair2.log" 2>&1
OVH_VOTE_PAIR=3 timeout -k 10 240 $B > "$OUT/bench_pair3.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_pair2b.log" 2>&1
OVH_VOTE_PAIR=3 timeout -k 10 240 $B > "$OUT/bench_pair3b.log" 2>&1
echo ok > "$OUT/ok"
