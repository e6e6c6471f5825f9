#!/bin/bash
# A/B of the vote-wave start stagger (diagnostic builds under consensus_overlord_amd/exp/).
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency > $OUT/p0.log 2>&1
for p in s2 s4; do
  OVH_LIBPATH=$PWD/consensus_overlord_amd/exp/libovhip_$p.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency > $OUT/p$p.log 2>&1
done
echo ok > $OUT/ok
