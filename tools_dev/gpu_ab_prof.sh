# per-kernel A/B of two libbwagpu.so builds: rocprofv3 kernel stats of
# realbench (reference-seeded C2 batches) with lib/ and with $2
# usage (on the GPU box): bash tools_dev/gpu_ab_prof.sh <tag> <alt-lib-path>
set -o pipefail
TAG=${1:-abprof}; ALT=${2}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for V in a b; do
  if [ "$V" = b ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/$ALT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 2 --reps 10 > $OUT/rb_$V.json 2> $OUT/rb_$V.err || { tail $OUT/rb_$V.err; exit 2; }
  python3 - $OUT/prof_$V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print("%-60s calls %6s avg_us %9.1f tot_ms %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done
cat $OUT/rb_a.json $OUT/rb_b.json
