# Official round measurement on the GPU box: every -m gpu test, the default
# bench line, the rocprofv3 kernel-trace summary of the same command, the
# dominant kernel's SQ instruction mix (two counter passes), and the HBM
# traffic PMC passes (FETCH_SIZE and WRITE_SIZE separately, MI355X_MICROARCH.md §HBM).
# usage (on the GPU box): bash tools_dev/gpu_round.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r02}; SKIPT=${2:-0}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$SKIPT" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?" >> $OUT/gpu_tests.log; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
cat $OUT/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 8 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1 || { tail $OUT/pmc_fetch.log; exit 6; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- $B > $OUT/pmc_write.log 2>&1 || { tail $OUT/pmc_write.log; exit 7; }
python3 $GRAFT_REPO_ROOT/tools_dev/pmc_summary.py $OUT "spec_ext2_kernel<5>" > $OUT/pmc_summary.txt
echo done > $OUT/rc.txt
