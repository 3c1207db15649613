#!/bin/bash
set -o pipefail
T=${1:-r5l}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sl in 1 2 4; do
  BWAGPU_STAGE_SLOTS=$sl timeout -k 10 300 python -u tools_dev/e2e_ab.py 1 2 3 4 > $OUT/e$sl.json 2> $OUT/e$sl.err || { tail $OUT/e$sl.err; exit 1; }
  cat $OUT/e$sl.json
done
