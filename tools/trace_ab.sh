#!/bin/bash
# Kernel traces of the bench under environment switches: AB="VAR=a VAR=b", TAG output dir.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-tr}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
k=0
for kv in ${AB}; do
  export ${kv}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$k -o tr -- python3 $R/bench.py --no-cpu-baseline --no-latency --steps 20 > $OUT/t$k.log 2>&1
  k=$((k+1))
done
echo ok > $OUT/ok
