#!/bin/bash
# fused seeding validation + staging: seed/chain/SAM tests, then the chain bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6r; mkdir -p $OUT
export TMPDIR=/tmp
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_seed.py tests/test_gpu_chain.py tests/test_sam_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for k in 1; do
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 6 --fused --concurrent 2 > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 4; }
cat $OUT/cb.json
done
