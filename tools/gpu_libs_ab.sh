#!/bin/bash
# A/B of library builds on one GPU box: optional parity tests, then bench.py (no CPU baseline;
# latency probes only with LAT=1) with the default library and each LIBS entry (file names under
# consensus_overlord_amd/), ROUNDS times interleaved. Each step has its own limit; the first
# failure ends the script.   TAG=r03g LIBS="libovhip_ab1.so libovhip_ab2.so" TESTS=1
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-libab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in libovhip.so ${LIBS}; do
    OVH_LIBPATH=$R/consensus_overlord_amd/$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 \
      --no-cpu-baseline $([ -n "${LAT:-}" ] && echo --profile-steps 1 || echo --no-latency) > "$OUT/bench_${lib%.so}_$r.log" 2>&1
    echo "$lib $r $(python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['stage_ms'], d.get('latency', ''))" "$OUT/bench_${lib%.so}_$r.log")" >> "$OUT/summary.txt"
  done
done
echo done > "$OUT/ok"
