#!/bin/bash
set -o pipefail
T=${1:-r5p}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --steps 10 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
