#!/bin/bash
# kernel stats of the chaining path; outputs in gpurun_out/$1
set -o pipefail
T=${1:-chainprof}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null


timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 tools_dev/chain_bench.py --reps 3 > gpurun_out/$T/prof.log 2>&1 || { tail -20 gpurun_out/$T/prof.log; exit 2; }
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1); python3 -c "import csv,sys; r=list(csv.DictReader(open(sys.argv[1]))); [print(x[\"Name\"][:60], x[\"Calls\"], x[\"TotalDurationNs\"], x[\"AverageNs\"], x[\"MaxNs\"]) for x in r[:25]]" "$f"
