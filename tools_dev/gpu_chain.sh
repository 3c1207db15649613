#!/bin/bash
# the chaining + seeding GPU tests; outputs in gpurun_out/$1
set -o pipefail
T=${1:-chain}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_seed.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -3 gpurun_out/$T/tests.log
