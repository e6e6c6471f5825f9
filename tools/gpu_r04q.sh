#!/bin/bash
# r04q: spilled vote program (90 LDS slots): occupancy A/B, parity subset, bench with the vote
# kernels of consecutive batches on the two per-vote streams (default) and on one stream.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occupancy_ab.json" 2> "$OUT/occupancy_ab.err"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-latency > "$OUT/bench_pair.log" 2>&1
OVH_VOTE_PAIR=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-latency > "$OUT/bench_single.log" 2>&1
echo ok > "$OUT/ok"
