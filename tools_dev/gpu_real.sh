# Reference-seeded workload on the GPU box: C2-batch parity test, realbench
# (150 bp and mixed lengths), rocprofv3 kernel stats and two SQ PMC passes of
# the dominant kernel.
# usage (on the GPU box): bash tools_dev/gpu_real.sh <tag> [kernel-substring] [skip-tests]
set -o pipefail
TAG=${1:-real}; KN=${2:-chain2aln_fast_kernel<3>}; SKIPT=${3:-0}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ "$SKIPT" != "1" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
fi
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/real150.json 2> $OUT/real150.err || { tail $OUT/real150.err; exit 2; }
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 --length mix --pairs 24000 > $OUT/realmix.json 2> $OUT/realmix.err || { tail $OUT/realmix.err; exit 3; }
cat $OUT/real150.json $OUT/realmix.json
cd /tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 1 --reps 4"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- $B > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 4; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 5; }
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 6; }
python3 $GRAFT_REPO_ROOT/tools_dev/pmc_summary.py $OUT "$KN" | tee $OUT/pmc_summary.txt
grep -h "chain2aln\|chain_prep\|read_" $OUT/prof/*kernel_stats.csv | cut -d, -f1-8 | head -20
