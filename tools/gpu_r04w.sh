#!/bin/bash
# r04 evidence pass: -m gpu tests, smoke, bench (pipelined pair, default), the shard path, the
# one-stream A/B, rocprofv3 kernel stats of the bench. Each GPU step under its own limit.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r04w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py --steps ${STEPS:-30} --warmup 3 > "$OUT/bench.log" 2>&1
timeout -k 10 240 python -u bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 --shard-path > "$OUT/bench_shard.log" 2>&1
OVH_VOTE_PAIR=0 timeout -k 10 240 python -u bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_single.log" 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_prof.log" 2>&1
echo done > "$OUT/ok"
