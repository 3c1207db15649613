#!/bin/bash
# A/B of extend_pair's band trim: the in-tree build (ballot + readlane) vs
# alt_lib/libbwagpu_trimdpp.so (-DBWAGPU_TRIM_DPP=1, the r03c DPP reductions).
# Parity on the spec-path tests first; then the stage bench interleaved.
set -o pipefail
T=${1:-trimab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for L in new dpp new dpp; do
  if [ $L = dpp ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/alt_lib/libbwagpu_trimdpp.so; else unset BWAGPU_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-host-path --no-cigar --no-seeding --no-e2e --steps 30 > gpurun_out/$T/b_$L.json 2>> gpurun_out/$T/bench.err || exit 2
  python -c "import json;d=json.load(open('gpurun_out/$T/b_$L.json'));r=d['roofline'];g=d['regime_grch38'];print('$L',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],r['frac'],g['c3']['ms_per_batch'],g['c5']['ms_per_batch'],g['c3']['parity_all_steps'],g['c5']['parity_all_steps'])" | tee -a gpurun_out/$T/summary.txt
done
