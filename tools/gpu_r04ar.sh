#!/bin/bash
# r04ar: OVH_BATCH_SLOTS 8 (libovhip_ab.so) vs 6 with the pipelined pair.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r04ar}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_s6.log" 2>&1
OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 240 $B > "$OUT/bench_s8.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_s6b.log" 2>&1
OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 240 $B > "$OUT/bench_s8b.log" 2>&1
echo ok > "$OUT/ok"
