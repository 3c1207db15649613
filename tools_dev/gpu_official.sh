# Official round measurement: GPU parity tests, default bench line, rocprofv3
# kernel-trace summary of the same command, and HBM-traffic PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM).
# usage (on the GPU box): bash tools_dev/gpu_official.sh <tag>
set -o pipefail
TAG=${1:-r01}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?" >> $OUT/gpu_tests.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 2
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof.log 2>&1 || exit 3
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --steps 8 --warmup 1"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o f --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o w --output-format csv -- $B > $OUT/pmc_write.log 2>&1 || exit 5
echo done > $OUT/rc.txt
