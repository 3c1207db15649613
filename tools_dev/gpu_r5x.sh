#!/bin/bash
set -o pipefail
T=${1:-r5x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/c5_ab.py > $OUT/c.json 2> $OUT/c.err || { tail $OUT/c.err; exit 3; }
cat $OUT/c.json
