#!/bin/bash
# r04aq: the vote epilogue's fence at workgroup scope (default build) vs device scope
# (libovhip_ab.so built with -DOVH_VOTE_DEVICE_FENCE=1); parity subset on the default.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r04aq}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "parity or configs or pipelined or config4 or small" > "$OUT/pytest_gpu.log" 2>&1
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_wg.log" 2>&1
OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 240 $B > "$OUT/bench_dev.log" 2>&1
timeout -k 10 240 $B > "$OUT/bench_wg2.log" 2>&1
OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 240 $B > "$OUT/bench_dev2.log" 2>&1
OVH_VOTE_PAIR=0 timeout -k 10 240 $B > "$OUT/bench_wg_single.log" 2>&1
echo ok > "$OUT/ok"
