#!/bin/bash
set -o pipefail
T=${1:-r5w}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ab in 1 0 1 0; do
  if [ $ab = 1 ]; then export BWAGPU_AB_BIN2_FOUR=1; else unset BWAGPU_AB_BIN2_FOUR; fi
  timeout -k 10 300 python -u tools_dev/c5_ab.py > $OUT/c$ab.json 2> $OUT/c$ab.err || { tail $OUT/c$ab.err; exit 5; }
  echo "bin2 four=$ab" $(cat $OUT/c$ab.json)
done
