#!/bin/bash
# r04af: the vote kernel on one high-priority per-vote stream (OVH_VOTE_PAIR=1) vs `stream`
# (OVH_VOTE_PAIR=0): the unpipelined profile batches' vote stage time on each.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04af}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 20"
OVH_VOTE_PAIR=1 timeout -k 10 240 $B > "$OUT/bench_one_pstream.log" 2>&1
OVH_VOTE_PAIR=0 timeout -k 10 240 $B > "$OUT/bench_main.log" 2>&1
OVH_VOTE_PAIR=1 OVH_PAIR_PRIO=0 timeout -k 10 240 $B > "$OUT/bench_one_pstream_normal.log" 2>&1
echo ok > "$OUT/ok"
