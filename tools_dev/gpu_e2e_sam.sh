# whole-pipeline end to end on a chr21-sized genome: bwa mem's own pipeline vs
# the SAM harness with seeding / chain2aln / rescue / CIGAR on the GPU
# usage: bash tools_dev/gpu_e2e_sam.sh <tag> [pairs] [threads] [modes]
set -o pipefail
TAG=${1:-e2esam}; P=${2:-100000}; T=${3:-16}; MODES=${4:-"ref gpuseed"}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT bench_data/e2e
for M in $MODES; do
  timeout -k 10 500 oracle/_ref/sam_harness $M bench_data/e2e /tmp/$M.sam 7 $P 150 10000000 $T 46709983 > $OUT/$M.log 2>&1 || { echo "$M failed: $?"; tail -5 $OUT/$M.log; exit 1; }
  tail -1 $OUT/$M.log
done
for M in $MODES; do [ $M = ref ] || { cmp /tmp/ref.sam /tmp/$M.sam && echo "$M SAM_IDENTICAL"; }; done
rm -f /tmp/*.sam
