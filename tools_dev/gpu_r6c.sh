#!/bin/bash
# chaining: one call's latency vs 2 and 3 contexts on host threads (pipeline throughput)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6c; mkdir -p $OUT
export TMPDIR=/tmp
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
for c in 2 3; do
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 6 --fused --concurrent $c > $OUT/cb$c.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 2; }
cat $OUT/cb$c.json
done
