#!/bin/bash
# A/B of the final kernel's wave priority (diagnostic builds under consensus_overlord_amd/exp/).
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency > $OUT/p0.log 2>&1
for p in 1 2 3; do
  OVH_LIBPATH=$PWD/consensus_overlord_amd/exp/libovhip_p$p.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency > $OUT/p$p.log 2>&1
done
echo ok > $OUT/ok
