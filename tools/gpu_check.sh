#!/bin/bash
# One GPU-box pass (round 2): parity tests, smoke, bench. Every GPU step has its own time limit;
# the first failure ends the script (set -e). Output under gpurun_out/$TAG.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
echo ok > "$OUT/ok"
