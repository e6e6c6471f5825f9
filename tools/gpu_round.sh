#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats. Every GPU step has its
# own time limit; the first failure ends the script (set -e).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -x tools/ubench/fp_mul28 ]; then timeout -k 10 60 tools/ubench/fp_mul28 > "$OUT/fp_mul28.log" 2>&1; fi
timeout -k 10 300 python -c "import torch; print(torch.__version__, torch.cuda.is_available())" > "$OUT/torch.log" 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --steps ${STEPS:-30} --warmup 2 > "$OUT/bench.log" 2>&1
if [ -n "${AB:-}" ]; then
  OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline > "$OUT/bench_ab.log" 2>&1
fi
if [ -n "${Q8:-}" ]; then
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency > "$OUT/bench_q8.log" 2>&1
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency --shard-path > "$OUT/bench_shard_q4.log" 2>&1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency --shard-path > "$OUT/bench_shard_q8.log" 2>&1
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_prof.log" 2>&1
echo done > "$OUT/ok"
