#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ch6; mkdir -p $OUT
export TMPDIR=/tmp
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 3; }
BWAGPU_CHAIN_PHASES=1 timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 1 > $OUT/phases.json 2> $OUT/phases.err || { tail $OUT/phases.err; exit 1; }
grep "chain phases" $OUT/phases.err | head -20
bash tools_dev/gpu_chain_prof.sh chprof6
