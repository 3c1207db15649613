# align2 (mate rescue) on the GPU: parity tests, throughput, kernel-trace stats
# usage: bash tools_dev/gpu_align2.sh <tag> [align2_bench args]
set -o pipefail
TAG=${1:-a2}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 420 python -m pytest tests/test_gpu_align2.py -x -q > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python tools_dev/align2_bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/align2_bench.py --reps 3 --check 0 --cpu-sample 0 "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 3; }
python3 - "$OUT" <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/prof/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {float(r['Percentage']):5.1f}%  {r['Name'][:110]}")
PY
