#!/bin/bash
# the driver's round-end sequence on this tree: every -m gpu test, smoke(), the default bench line
set -o pipefail
T=${1:-final}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail gpurun_out/$T/smoke.log; exit 2; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail gpurun_out/$T/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/$T/bench.json'));print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:(v.get('value') if isinstance(v,dict) else None) for k,v in d.items() if isinstance(v,dict) and 'value' in v})"
