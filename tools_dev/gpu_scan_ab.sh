#!/bin/bash
# A/B of spec_scan_kernel's grid (BWAGPU_SCAN_GRID), stage bench + C3/C5
set -o pipefail
T=${1:-scanab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
for P in ${PS:-1024 256 512 2048 1024 256 512 2048}; do
  BWAGPU_SCAN_GRID=$P timeout -k 10 200 python -u bench.py --no-cpu --no-host-path --no-cigar --no-seeding --no-e2e --steps 30 > gpurun_out/$T/b_$P.json 2>> gpurun_out/$T/bench.err || exit 2
  python -c "import json;d=json.load(open('gpurun_out/$T/b_$P.json'));r=d['roofline'];g=d['regime_grch38'];print('scan_grid=$P',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],g['c3']['ms_per_batch'],g['c5']['ms_per_batch'],g['c3']['parity_all_steps'],g['c5']['parity_all_steps'])" | tee -a gpurun_out/$T/summary.txt
done
