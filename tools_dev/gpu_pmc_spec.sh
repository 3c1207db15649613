# SQ counters of the spec path's kernels on realbench (one batch, 4 reps)
set -o pipefail
TAG=${1:-pmcspec}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 1 --reps 3"
timeout -k 10 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -k 10 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 2; }
for k in "spec_select_light<0>" "spec_select_light<1>" "spec_ext_kernel<3>" "spec_scan_kernel<1>" "spec_pairs_kernel"; do echo "== $k"; python3 $GRAFT_REPO_ROOT/tools_dev/pmc_summary.py $OUT "$k"; done | tee $OUT/summary.txt
