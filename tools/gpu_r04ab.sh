#!/bin/bash
# r04ab: pipelined same-message batches (tools/samemsg_pipe.py) with and without the vote pair
# streams; kernel trace of the default.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/samemsg_pipe.py 24 4096 > "$OUT/pipe.json" 2> "$OUT/pipe.err"
OVH_VOTE_PAIR=0 timeout -k 10 200 python -u tools/samemsg_pipe.py 24 4096 > "$OUT/pipe_nopair.json" 2> "$OUT/pipe_nopair.err"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o pipe -- python3 -u tools/samemsg_pipe.py 12 4096 > "$OUT/trace.log" 2>&1
echo ok > "$OUT/ok"
