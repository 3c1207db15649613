#!/bin/bash
# round 6: round C unlaunched under the strict emulation — the stage's GPU
# tests, c5_refseed with the second bin phased or not (BWAGPU_EXT_PHASED 1 / 3),
# the regime legs and the fixture line
set -o pipefail
T=${1:-r06s}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py tests/test_sam_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for M in 1 3 1 3; do
  BWAGPU_EXT_PHASED=$M timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$M.json 2> $OUT/c5_$M.err || exit 7
  python3 -c "import json;a=json.load(open('$OUT/c5_$M.json'));print('c5 mask $M', a['ms_per_batch'], a['parity_all_steps'])"
done
timeout -k 10 600 python -u bench.py --workload c2_refseed --no-cpu --no-host-path --no-cigar --no-e2e --no-seeding --no-hwq4 > $OUT/reg.json 2> $OUT/reg.err || exit 3
python3 -c "
import json;d=json.load(open('$OUT/reg.json'));rg=d['regime_grch38']
print('fix', d['value'], d['ms_per_step'], d['parity_all_steps'])
print('regime', {k:(rg[k]['ms_per_batch'], rg[k]['parity_all_steps']) for k in ('c3','c5','c3_refseed')}, 'c5_refseed', d['c5_refseed']['ms_per_batch'], d['c5_refseed']['parity_all_steps'])"
echo done > $OUT/rc.txt
