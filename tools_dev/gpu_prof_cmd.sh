# kernel-trace summary of any python tool; usage: bash tools_dev/gpu_prof_cmd.sh <tag> <script.py> [args]
set -o pipefail
TAG=${1:-p}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SCRIPT=$GRAFT_REPO_ROOT/$1; shift
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $SCRIPT "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 3; }
python3 - "$OUT" <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/prof/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {float(r['Percentage']):5.1f}%  {r['Name'][:110]}")
PY
grep -v amdgpu.ids $OUT/prof.log | tail -3
