#!/bin/bash
# r04an: pair-synchronised vote grids (OVH_PAIR_SYNC, default) vs free-running pair; parity subset.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04an}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "parity or configs or pipelined or config4" > "$OUT/pytest_gpu.log" 2>&1
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --steps 30"
timeout -k 10 240 $B > "$OUT/bench_sync.log" 2>&1
OVH_PAIR_SYNC=0 timeout -k 10 240 $B > "$OUT/bench_free.log" 2>&1
timeout -k 10 240 $B --steps 20 > "$OUT/bench_sync20.log" 2>&1
echo ok > "$OUT/ok"
