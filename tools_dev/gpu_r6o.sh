#!/bin/bash
# drop-in stage end to end: host pool threads x stage workers
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6o
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for ht in 8 16 12 8 16; do
  BWAGPU_HOST_THREADS=$ht timeout -k 10 300 python -u tools_dev/e2e_ab.py 3 4 > $OUT/e$ht.json 2> $OUT/e.err || { tail $OUT/e.err; exit 5; }
  sed "s/^/ht=$ht /" $OUT/e$ht.json
done
