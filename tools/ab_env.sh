#!/bin/bash
# A/B of environment switches on the bench (no CPU baseline / latency probes), after the GPU
# parity tests: AB="VAR=a VAR=b ..." (each run: one env assignment), TAG names the output dir.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
k=0
for kv in ${AB}; do
  env "$kv" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency --steps ${STEPS:-30} > $OUT/ab$k.log 2>&1
  echo "$kv $(python -c "import json; d=json.loads([l for l in open('$OUT/ab$k.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['stage_ms'])")" >> $OUT/summary.txt
  k=$((k+1))
done
echo ok > $OUT/ok
