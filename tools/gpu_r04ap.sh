#!/bin/bash
# r04ap: L2 hit / miss and wait counters of k_vm_vote in the two-grid diagnostic (real votes)
# and in the pipelined bench -- where does the pipeline's 25% go?
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r04ap}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/diag_tcc" -o tcc --output-format csv -- python3 "$R/tools/occupancy_real.py" > "$OUT/diag_tcc.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/bench_tcc" -o tcc --output-format csv -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_tcc.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/diag_sq" -o sq --output-format csv -- python3 "$R/tools/occupancy_real.py" > "$OUT/diag_sq.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/bench_sq" -o sq --output-format csv -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 > "$OUT/bench_sq.log" 2>&1
echo ok > "$OUT/ok"
