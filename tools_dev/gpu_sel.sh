#!/bin/bash
# selection-pass work: spec counters, parity of the spec path, the stage bench, the per-read trace
set -o pipefail
T=${1:-sel}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste.json 2> $OUT/waste.err || { tail $OUT/waste.err; exit 1; }
cat $OUT/waste.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 2; }
tail -1 $OUT/t.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','frac','frac_isolated','isolated_launch_ms')})"
timeout -k 10 300 python -u tools_dev/spec_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 4; }
