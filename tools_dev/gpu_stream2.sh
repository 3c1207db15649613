# sw_stream timing on the C2 batch, then SQ counters of the small spec kernels
set -o pipefail
TAG=${1:-stream2}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools_dev/stream_bench.py > $OUT/stream_bench.json 2> $OUT/stream_bench.err || { tail -20 $OUT/stream_bench.err; exit 1; }
cat $OUT/stream_bench.json
bash tools_dev/gpu_pmc_k.sh $TAG/pmc spec_order > $OUT/pmc_order.txt 2>&1 || { tail -20 $OUT/pmc_order.txt; exit 2; }
cat $OUT/pmc_order.txt
python3 tools_dev/pmc_summary.py $OUT/pmc spec_chain_kernel
