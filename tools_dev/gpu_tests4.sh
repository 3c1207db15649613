#!/bin/bash
# every -m gpu test + a bench line on this tree (GPU box)
set -o pipefail
T=${1:-t4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp

timeout -k 10 1200 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms','traffic_source')})"
