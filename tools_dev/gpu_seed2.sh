# seeding: parity tests, then the bench at several tier budgets + kernel profile
set -o pipefail
TAG=${1:-seedt}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seed.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for B in 1024 512 2048; do
  timeout -k 10 300 python -u tools_dev/seed_bench.py --reps 5 --check 1000 --cpu-reads 10 --budget $B > $OUT/seed_$B.json 2> $OUT/seed_$B.err || { tail $OUT/seed_$B.err; exit 2; }
  python3 -c "import json; d=json.load(open('$OUT/seed_$B.json')); print('budget $B', d['ms_per_batch'], d['gpu_reads_per_s'], d['parity'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/seed_bench.py --reps 5 --check 10 --cpu-reads 10 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
python3 - $OUT/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print("%-50s calls %5s avg_us %10.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
