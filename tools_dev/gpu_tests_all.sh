#!/bin/bash
# every -m gpu test in one process, then smoke(); outputs in gpurun_out/$1
set -o pipefail
T=${1:-tests}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { cat gpurun_out/$T/smoke.log; exit 2; }
cat gpurun_out/$T/smoke.log
