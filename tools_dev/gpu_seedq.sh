#!/bin/bash
# tier-1 seeding A/B: nested (0) / step (1) / persistent task-queue step (2) kernels; parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/seedq; mkdir -p $OUT
export TMPDIR=/tmp
BWAGPU_SEED_STEP=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_seed.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
for k in 1 2; do for s in 0 1 2; do
BWAGPU_SEED_STEP=$s timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 5 --fused > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 2; }
echo "step=$s $(cat $OUT/cb.json)"
done; done
