#!/bin/bash
# chaining GPU tests + SAM parity (gpuchain) + the bench's seeding/chaining legs; outputs in gpurun_out/$1
set -o pipefail
T=${1:-chain2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_sam_parity.py -k "chain or seqs2regions" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -3 gpurun_out/$T/tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-host-path --no-cigar --no-regime --no-e2e > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); print(json.dumps({k: d.get(k) for k in ('value','seeding_stage','chaining_stage')}))"
