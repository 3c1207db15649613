#!/bin/bash
# the pair kernel at 2 workgroups per CU (default) vs capacity, by caller-stream count
set -o pipefail
T=${1:-gridab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_host_stage.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for c in ${CASES:-2:0 3:0 4:0 2:100 3:100 4:100 3:3}; do
  S=${c%%:*}; P=${c##*:}
  if [ "$P" = "3" ]; then export BWAGPU_EXT2_BLOCKS_PER_CU=3; unset BWAGPU_EXT2_GRID_PCT; else unset BWAGPU_EXT2_BLOCKS_PER_CU; export BWAGPU_EXT2_GRID_PCT=$P; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-cigar --no-seeding --no-e2e --steps 30 --streams $S > gpurun_out/$T/b_${S}_$P.json 2>> gpurun_out/$T/bench.err || exit 2
  python -c "import json;d=json.load(open('gpurun_out/$T/b_${S}_$P.json'));r=d['roofline'];g=d['regime_grch38'];e=d['end_to_end'];print('streams=$S grid=$P',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],r['frac'],g['c3']['ms_per_batch'],g['c5']['ms_per_batch'],'e2e',e['value'],'hostbuf',d['host_buffer_path']['value'])" | tee -a gpurun_out/$T/summary.txt
done
