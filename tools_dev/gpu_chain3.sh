#!/bin/bash
# chaining tests + kernel stats of the chaining path; outputs in gpurun_out/$1
set -o pipefail
T=${1:-chain3}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_sam_parity.py -k "chain or seqs2regions" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python -u tools_dev/chain_bench.py --reps 5 --fused > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 2; }
cat gpurun_out/$T/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 tools_dev/chain_bench.py --reps 3 > gpurun_out/$T/prof.log 2>&1 || { tail -20 gpurun_out/$T/prof.log; exit 3; }
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1); python3 -c "import csv,sys; r=list(csv.DictReader(open(sys.argv[1]))); [print(x['Name'][:70], x['Calls'], x['AverageNs'], x['MaxNs']) for x in r[:16]]" "$f"
