# FPGA wire-format tests, then the whole -m gpu suite + smoke, then a kernel
# profile of realbench (spec_order_kernel et al.)
set -o pipefail
TAG=${1:-stream}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpga_stream.py -x -v --timeout 200 --timeout-method thread > $OUT/stream_tests.log 2>&1 || { tail -40 $OUT/stream_tests.log; exit 1; }
tail -1 $OUT/stream_tests.log
bash tools_dev/gpu_all.sh $TAG || exit 2
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 2 --reps 10 > $OUT/rb.json 2> $OUT/rb.err || { tail $OUT/rb.err; exit 3; }
python3 - $OUT/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("%-60s calls %6s avg_us %9.1f tot_ms %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
cat $OUT/rb.json
