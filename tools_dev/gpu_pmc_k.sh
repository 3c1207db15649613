# two SQ PMC passes on a short bench run, summarised for one kernel
# usage: bash tools_dev/gpu_pmc_k.sh <tag> <kernel-substring> [bench args]
set -o pipefail
TAG=${1:-pk}; KN=$2; shift; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --pairs 100000 --steps 4 --warmup 1 --no-cpu --no-host-path $@"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 2; }
python3 $GRAFT_REPO_ROOT/tools_dev/pmc_summary.py $OUT "$KN"
