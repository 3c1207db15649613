# the FPGA wire-format path after the claim-size change: its GPU parity tests,
# then its C2 timing (tools_dev/stream_bench.py)
set -o pipefail
TAG=${1:-streamclaim}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpga_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u tools_dev/stream_bench.py > $OUT/stream_bench.json 2> $OUT/stream_bench.err || { tail -20 $OUT/stream_bench.err; exit 2; }
cat $OUT/stream_bench.json
