# seeding bench + kernel profile on the GPU box
# usage: bash tools_dev/gpu_seed.sh <tag>
set -o pipefail
TAG=${1:-seed}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/seed_bench.py > $OUT/seed.json 2> $OUT/seed.err || { tail $OUT/seed.err; exit 1; }
cat $OUT/seed.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/seed_bench.py --reps 5 --check 10 --cpu-reads 10 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 2; }
python3 - $OUT/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print("%-50s calls %5s avg_us %10.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
