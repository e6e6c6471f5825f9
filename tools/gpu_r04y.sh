#!/bin/bash
# r04y: one-wave MSM helper kernels: batch parity subset, bench (30 / 60 steps), shard path.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04y}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "parity or configs or pipelined or config4 or samemsg" > "$OUT/pytest_gpu.log" 2>&1
B="python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0"
timeout -k 10 240 $B --steps 30 > "$OUT/bench30.log" 2>&1
timeout -k 10 240 $B --steps 60 > "$OUT/bench60.log" 2>&1
timeout -k 10 240 $B --steps 30 --shard-path > "$OUT/bench_shard.log" 2>&1
echo ok > "$OUT/ok"
