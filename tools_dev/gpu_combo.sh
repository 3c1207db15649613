#!/bin/bash
# tools_dev/gpu_ab6.sh (every GPU test + stage A/B) then the chaining bench with per-read phases
set -o pipefail
T=${1:-combo}
bash tools_dev/gpu_ab6.sh $T || exit $?
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$T
[ -f bench_data/e2e/ref.fa.sa ] || timeout -k 10 600 python3 -c "import bench; bench.end_to_end_align(2000)" > $OUT/index.log 2>&1 || { tail $OUT/index.log; exit 6; }
BWAGPU_CHAIN_PHASES=1 timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 1 > $OUT/phases.json 2> $OUT/phases.err || { tail $OUT/phases.err; exit 7; }
grep "chain phases" $OUT/phases.err | head -8
for k in 1 2; do
timeout -k 10 300 python3 tools_dev/chain_bench.py --reps 5 --fused --budget 1024 > $OUT/cb.json 2> $OUT/cb.err || { tail $OUT/cb.err; exit 8; }
cat $OUT/cb.json
done
