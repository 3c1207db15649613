#!/bin/bash
# the final pass without the inline extension (alt_lib/libbwagpu_noinline.so,
# -DBWAGPU_LIGHT_INLINE=0) at capped spec_select_light grids vs the default build
set -o pipefail
T=${1:-inl}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
for c in def:0 noinl:0 noinl:1 noinl:2 def:0 noinl:1 noinl:2; do
  L=${c%%:*}; P=${c##*:}
  if [ $L = noinl ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/alt_lib/libbwagpu_noinline.so; else unset BWAGPU_LIB; fi
  BWAGPU_LIGHT_BLOCKS_PER_CU=$P timeout -k 10 200 python -u bench.py --no-cpu --no-host-path --no-cigar --no-seeding --no-e2e --steps 30 > gpurun_out/$T/b.json 2>> gpurun_out/$T/bench.err || exit 2
  python -c "import json;d=json.load(open('gpurun_out/$T/b.json'));r=d['roofline'];g=d['regime_grch38'];print('$L light_per_cu=$P',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],g['c3']['ms_per_batch'],g['c5']['ms_per_batch'],g['c3']['parity_all_steps'],g['c5']['parity_all_steps'])" | tee -a gpurun_out/$T/summary.txt
done
