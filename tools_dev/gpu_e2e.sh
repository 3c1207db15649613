# End-to-end numbers on the GPU box: the SAM harness (bwa mem's pipeline: CPU
# seeding + [CPU | GPU] mem_chain2aln + CPU SAM stage, 16 threads) at 100k
# pairs, and bench.py with the host-path / end_to_end legs.
# usage: bash tools_dev/gpu_e2e.sh <tag>
set -o pipefail
TAG=${1:-e2e}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/h_ref $OUT/h_gpu
timeout -k 10 300 oracle/_ref/sam_harness ref $OUT/h_ref $OUT/h_ref/out.sam 21 100000 150 10000000 16 2> $OUT/h_ref.err || { tail $OUT/h_ref.err; exit 1; }
timeout -k 10 300 oracle/_ref/sam_harness gpu $OUT/h_gpu $OUT/h_gpu/out.sam 21 100000 150 10000000 16 2> $OUT/h_gpu.err || { tail $OUT/h_gpu.err; exit 2; }
cmp $OUT/h_ref/out.sam $OUT/h_gpu/out.sam && echo "SAM identical" | tee $OUT/sam_cmp.txt
grep mode $OUT/h_ref.err $OUT/h_gpu.err | tee $OUT/harness_times.txt
rm -f $OUT/h_ref/out.sam $OUT/h_gpu/out.sam $OUT/h_ref/ref.fa* $OUT/h_gpu/ref.fa*
timeout -k 10 300 python bench.py --no-cpu --no-cigar > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
cat $OUT/bench.json
