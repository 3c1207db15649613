#!/bin/bash
# memory-side PMC of the seeding kernels (L2 hits/misses, fabric requests,
# L1 requests); flat (default) and nested tier 1; outputs in gpurun_out/$1
set -o pipefail
T=${1:-seedmem}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/seed_bench.py --reps 1 --check 10 --cpu-reads 10"
for V in 0 1; do
  export BWAGPU_SEED_NESTED=$V
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d $OUT/a$V -o a --output-format csv -- $B > $OUT/a$V.log 2>&1 || { tail $OUT/a$V.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU -d $OUT/b$V -o b --output-format csv -- $B > $OUT/b$V.log 2>&1 || { tail $OUT/b$V.log; exit 2; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for V in "01":
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(sys.argv[1] + "/[ab]%s/**/*counter_collection.csv" % V, recursive=True):
        for r in csv.DictReader(open(f)):
            if "collect_intv" in r["Kernel_Name"]:
                tot[r["Kernel_Name"][:50]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("nested" if V == "1" else "flat")
    for k, v in tot.items():
        print(" ", k, {a: "%.4g" % b for a, b in sorted(v.items())})
PY
