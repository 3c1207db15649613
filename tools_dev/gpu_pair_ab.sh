#!/bin/bash
# A/B of the two-seeds-per-wave extension kernel (BWAGPU_EXT_PAIR): parity
# first (every spec-path GPU test with the pair kernel), then the stage bench
# with each setting.  Run under gpurun; outputs in gpurun_out/$1.
set -o pipefail
T=${1:-pairab}
mkdir -p gpurun_out/$T
export BWAGPU_EXT_PAIR=${PAIRMODE:-2}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/$T/tests_pair.log 2>&1 || { echo "pair tests failed"; exit 1; }
for p in 0 1 2 0 2; do
  BWAGPU_EXT_PAIR=$p timeout -k 10 200 python -u bench.py --no-cpu --no-host-path --no-cigar --no-seeding --steps 30 \
    > gpurun_out/$T/bench_p$p.json 2>> gpurun_out/$T/bench.err || exit 1
  python -c "import json,sys;d=json.load(open('gpurun_out/$T/bench_p$p.json'));r=d['roofline'];g=d.get('regime_grch38',{});print('pair=$p',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],r['frac'],g.get('c3',{}).get('ms_per_batch'),g.get('c5',{}).get('ms_per_batch'),g.get('c3',{}).get('parity_all_steps'),g.get('c5',{}).get('parity_all_steps'))" | tee -a gpurun_out/$T/summary.txt
done
