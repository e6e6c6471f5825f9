#!/bin/bash
# r04r: pipelined pair A/B of the spilled vote program: one stream (OVH_VOTE_PAIR=0), the pair
# at normal priority, with normal-priority final streams, with a high-priority pair.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04r}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0"
OVH_VOTE_PAIR=0 timeout -k 10 240 $B > "$OUT/bench_single.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_pair.log" 2>&1
OVH_FINAL_LOW=0 timeout -k 10 240 $B > "$OUT/bench_pair_finnorm.log" 2>&1
OVH_PAIR_PRIO=1 timeout -k 10 240 $B > "$OUT/bench_pair_hi.log" 2>&1
echo ok > "$OUT/ok"
