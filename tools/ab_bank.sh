#!/bin/bash
# A/B of the LDS bank-spreading slot allocation (tools/fpvm/sched.py OVH_BANK builds under
# consensus_overlord_amd/exp/): bench + one bank-conflict PMC pass per variant.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-ab_bank}
mkdir -p $OUT
export TMPDIR=/tmp
for v in b8 b1_1 b16_16; do
  if [ $v = b8 ]; then unset OVH_LIBPATH; else export OVH_LIBPATH=$R/consensus_overlord_amd/exp/libovhip_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-latency > $OUT/$v.log 2>&1
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY \
    -d $OUT/pmc_$v -o c --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency > $OUT/pmc_$v.log 2>&1)
done
echo ok > $OUT/ok
