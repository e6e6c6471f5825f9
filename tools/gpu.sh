#!/bin/bash
# One GPU-box pass, parametrised (replaces the round-4 one-off scripts). Every GPU step has its
# own time limit and the first failure ends the script (set -e). Steps run when their variable
# is set (TAG names the output directory gpurun_out/$TAG):
#   POOL=1    tools/pool_probe.py (the vote pool alone)
#   TESTS=1   pytest -m gpu (TESTS_K: a -k expression)
#   SMOKE=1   __graft_entry__.smoke()
#   BENCH=1   bench.py --steps $STEPS (BENCH_ARGS appended)
#   PROF=1    rocprofv3 --kernel-trace --stats over a short bench
#   PMC=1     tools/pmc_pool.sh (the vote pool's counter passes, one run each; then
#             python tools/pmc_pool_summary.py $TAG on the CPU side)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 300 python -c "import torch; print(torch.__version__, torch.cuda.is_available())" > "$OUT/torch.log" 2>&1
if [ -n "${POOL:-}" ]; then
  timeout -k 10 120 python -u tools/pool_probe.py 4096 24 > "$OUT/pool.json" 2> "$OUT/pool.err"
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu ${TESTS_NOX:--x} -v --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > "$OUT/pytest_gpu.log" 2>&1
fi
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup 2 ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_prof.log" 2>&1
  cd "$R"
fi
if [ -n "${PMC:-}" ]; then
  TAG=${TAG:-run} bash tools/pmc_pool.sh > "$OUT/pmc.log" 2>&1
fi
echo done > "$OUT/ok"
