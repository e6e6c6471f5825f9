#!/bin/bash
# r04t: final streams A/B with the pipelined pair (four vs two), the parity subset.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04t}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0"
timeout -k 10 240 $B > "$OUT/bench_nfin4.log" 2>&1
OVH_NFIN=2 timeout -k 10 240 $B > "$OUT/bench_nfin2.log" 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "parity or configs or pipelined" > "$OUT/pytest_gpu.log" 2>&1
echo ok > "$OUT/ok"
