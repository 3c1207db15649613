#!/bin/bash
# quad-kernel bring-up: the extension-kernel parity tests first, then the C2 bench (quad and pair forms)
set -o pipefail
T=${1:-quad}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ksw_extend2_tasks or chain_sets or cell_and_call" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -1 $OUT/t1.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/t2.log 2>&1 || { tail -40 $OUT/t2.log; exit 2; }
tail -1 $OUT/t2.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms')})"
timeout -k 10 300 python -u bench.py --ext-form 1 --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench_pair.json 2> $OUT/bench_pair.err || { tail $OUT/bench_pair.err; exit 4; }
python3 -c "import json;d=json.load(open('$OUT/bench_pair.json'));r=d['roofline'];print('pair',d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms')})"
