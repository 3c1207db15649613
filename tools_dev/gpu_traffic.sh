#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes of the stage bench alone (one rocprofv3 --pmc
# run each), for profiles/<tag>_c2_refseed_traffic.json of THIS tree
# (tools_dev/pmc_traffic.py <dir> <tag> c2_refseed 5 afterwards).
set -o pipefail
T=${1:-traffic}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 5 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 $B > $OUT/f.json 2> $OUT/f.err || { tail $OUT/f.err; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 $B > $OUT/w.json 2> $OUT/w.err || { tail $OUT/w.err; exit 4; }
echo done > $OUT/rc.txt
