#!/bin/bash
# PMC counters of the seeding kernels; outputs in gpurun_out/$1
set -o pipefail
T=${1:-seedpmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/seed_bench.py --reps 1 --check 10 --cpu-reads 10"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 2; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "collect_intv" in r["Kernel_Name"]:
            tot[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in tot.items():
    print(k, {a: "%.3g" % b for a, b in sorted(v.items())})
PY
