#!/bin/bash
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6d
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/host_prof.py > $OUT/host.txt 2> $OUT/host.err || { tail $OUT/host.err; exit 5; }
cat $OUT/host.txt
grep "\[submit\]" $OUT/host.err | tail -40
