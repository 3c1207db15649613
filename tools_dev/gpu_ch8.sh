#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ch8}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_seed.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
BWAGPU_CHAIN_PHASES=1 timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 1 > $OUT/phases.json 2> $OUT/phases.err || { tail $OUT/phases.err; exit 1; }
grep "chain phases" $OUT/phases.err | head -8
for bg in 1024 1024; do
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 5 --fused --budget $bg > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 2; }
cat $OUT/cb.json
done
bash tools_dev/gpu_chain_prof.sh ${1:-ch8}_prof
