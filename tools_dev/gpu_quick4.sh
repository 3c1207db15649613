#!/bin/bash
# quick check of this round's host/ABI changes on the GPU box + the counter list
set -o pipefail
T=${1:-q4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_error_conditions tests/test_gpu_chain.py tests/test_host_stage.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms','traffic_source')})"
