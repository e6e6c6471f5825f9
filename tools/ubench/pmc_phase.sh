#!/bin/bash
# PMC passes (one counter group per run) over single vm_phase cases: KIND W GRID
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ubpmc
mkdir -p $OUT
for c in "1 16 1024" "2 16 1024" "0 16 1024"; do
  set -- $c
  tag=k$1
  timeout -k 10 60 $R/tools/ubench/vm_phase $1 $2 $3 > $OUT/$tag.json
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/$tag.a -o pmc --output-format csv -- $R/tools/ubench/vm_phase $1 $2 $3 > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/$tag.b -o pmc --output-format csv -- $R/tools/ubench/vm_phase $1 $2 $3 > /dev/null
done
echo done > $OUT/ok
