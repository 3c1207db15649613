#!/bin/bash
# c5_refseed leg under a kernel trace: where the mixed-length batch's time goes
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6s
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/c5_ab.py > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 3; }
cat $OUT/c5.json
