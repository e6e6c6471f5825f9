#!/bin/bash
# r04aj: final streams on a CU subset (OVH_FIN_CUS), with / without the vote pair excluded from it.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04aj}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_default.log" 2>&1
OVH_FIN_CUS=16 timeout -k 10 240 $B > "$OUT/bench_fin16.log" 2>&1
OVH_FIN_CUS=16 OVH_VOTE_EXCL=1 timeout -k 10 240 $B > "$OUT/bench_fin16_excl.log" 2>&1
OVH_FIN_CUS=32 OVH_VOTE_EXCL=1 timeout -k 10 240 $B > "$OUT/bench_fin32_excl.log" 2>&1
OVH_FIN_CUS=8 OVH_VOTE_EXCL=1 timeout -k 10 240 $B > "$OUT/bench_fin8_excl.log" 2>&1
echo ok > "$OUT/ok"
