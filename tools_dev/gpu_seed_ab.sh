#!/bin/bash
# tier-1 A/B on one box: the nested kernel vs the one-extension-per-step kernel
# (kernel times by rocprofv3, the batch's host wall by seed_bench)
set -o pipefail
T=${1:-seedab}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in 1 0 1 0; do
  export BWAGPU_SEED_STEP=$((1 - V))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/seed_bench.py --reps 5 --check 200 --cpu-reads 10 > $OUT/b$V.json 2> $OUT/b$V.err || { tail $OUT/b$V.err; exit 1; }
  python3 - $OUT/p$V $OUT/b$V.json $V <<'PY'
import csv, glob, sys, json
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
d = json.load(open(sys.argv[2]))
import re
ks = {re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)", "anon")).split("::")[-1]: float(r["AverageNs"]) / 1e3
      for r in csv.DictReader(open(f))}
print("nested" if sys.argv[3] == "1" else "step  ", "wall %.2f ms parity %s" % (d["ms_per_batch"], d["parity"]),
      {k: round(v, 1) for k, v in ks.items() if "intv" in k or "merge" in k})
PY
done
