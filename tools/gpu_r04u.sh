#!/bin/bash
# r04u: the pipelined pair with hash_to_field on the main stream; parity subset.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04u}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0"
timeout -k 10 240 $B > "$OUT/bench_pair.log" 2>&1
timeout -k 10 240 $B --steps 60 > "$OUT/bench_pair60.log" 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "parity or configs or pipelined" > "$OUT/pytest_gpu.log" 2>&1
echo ok > "$OUT/ok"
