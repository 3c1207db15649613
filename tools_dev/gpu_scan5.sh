#!/bin/bash
# heavy-scan work: spec-path parity tests, then a kernel trace of the stage bench
set -o pipefail
T=${1:-scan5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 2; }
tail -1 $OUT/t.log
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 20 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s2 -o run --output-format csv -- python3 $B > $OUT/s2.json 2> $OUT/s2.err || { tail $OUT/s2.err; exit 3; }
tail -c 300 $OUT/s2.json
