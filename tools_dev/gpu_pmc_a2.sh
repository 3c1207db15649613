# SQ counters of the align2 kernels (two --pmc passes, kernel-trace only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmca2}
mkdir -p $OUT
cd /tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/align2_bench.py --reps 2 --check 0 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1
rc=$?
echo "pmc rc=$rc" > $OUT/rc.txt
for k in "align2_kernel<2, true>" "align2_kernel<3, true>" "align2_kernel<4, false>"; do echo "== $k"; python3 $GRAFT_REPO_ROOT/tools_dev/pmc_summary.py $OUT "$k"; done
exit $rc
