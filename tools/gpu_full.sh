#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats, one SQ PMC pass.
# Every GPU step has its own time limit; the first failure ends the script (set -e).
#   TAG=r02f bash tools/gpu_full.sh      (on the GPU box, from the repo root)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --no-latency > "$OUT/bench_prof.log" 2>&1
if [ -n "${PMC:-}" ]; then
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmc_sq" -o sq --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-latency > "$OUT/pmc_sq.log" 2>&1
fi
if [ -n "${TRACE:-}" ]; then
  cd "$R" && timeout -k 10 200 python -u tools/vm_trace.py "$OUT/trace" > "$OUT/trace.log" 2>&1
fi
echo done > "$OUT/ok"
