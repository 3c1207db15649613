#!/bin/bash
# four-per-wave occupancy diagnostic (lib/alt built with tools_dev/ab/quad_occupancy_diag.patch)
set -o pipefail
T=${1:-qocc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/alt/libbwagpu.so timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste.json 2> $OUT/waste.err || { tail $OUT/waste.err; exit 1; }
cat $OUT/waste.json
EXT_FORM=2 BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/alt/libbwagpu.so timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste2.json 2> $OUT/waste2.err || { tail $OUT/waste2.err; exit 1; }
cat $OUT/waste2.json
