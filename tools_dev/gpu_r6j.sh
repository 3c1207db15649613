#!/bin/bash
# seeding tier-1 budget sweep on seqs2chains
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6j; mkdir -p $OUT
export TMPDIR=/tmp
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
for bg in 2048 4096 1536 1024; do
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 5 --budget $bg > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 2; }
cat $OUT/cb.json
done
