#!/bin/bash
# seqs2chains timeline: one call's kernels and gaps (kernel trace of chain_bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6i; mkdir -p $OUT
export TMPDIR=/tmp
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_seed.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 6 --fused > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 4; }
cat $OUT/cb.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 tools_dev/chain_bench.py --reps 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 2; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools_dev/timeline.py $f collect_intv_kernel > $OUT/timeline.txt
tail -60 $OUT/timeline.txt
