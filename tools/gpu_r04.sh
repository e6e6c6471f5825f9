#!/bin/bash
# r04 GPU pass: integer-VALU rate ubench (1/2/4/8 waves per SIMD, held clock), the -m gpu
# parity tests, the bench (with the vote kernel's held clock). Each GPU step has its own limit;
# the first failure ends the script.   TAG=r04b bash tools/gpu_r04.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${NO_UBENCH:-}" ]; then
  timeout -k 10 150 tools/ubench/int_rates > "$OUT/int_rates.json" 2> "$OUT/int_rates.err"
fi
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
fi
timeout -k 10 400 python -u bench.py --steps ${STEPS:-30} --warmup 2 ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
echo ok > "$OUT/ok"
