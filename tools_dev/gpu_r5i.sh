#!/bin/bash
set -o pipefail
T=${1:-r5i}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rt in 2 4; do
  BWAGPU_REAPER_THREADS=$rt timeout -k 10 300 python -u tools_dev/e2e_ab.py > $OUT/e$rt.json 2> $OUT/e$rt.err || { tail $OUT/e$rt.err; exit 1; }
  cat $OUT/e$rt.json
done
