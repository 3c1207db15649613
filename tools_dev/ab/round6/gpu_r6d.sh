#!/bin/bash
# round 6: the claim-ahead as a knob (BWAGPU_EXT_PREFETCH) — parity, A/B against
# lib/ab0 and across prefetch settings, the cycle split of the diag build
set -o pipefail
T=${1:-r06d}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BWAGPU_EXT_PREFETCH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_pf.log 2>&1 || { echo "pytest (prefetch) failed"; tail -30 $OUT/gpu_tests_pf.log; exit 1; }
tail -1 $OUT/gpu_tests_pf.log
for rep in 1 2; do
for V in ab0 pf0 pf1 pf3; do
  unset BWAGPU_LIB BWAGPU_EXT_PREFETCH
  case $V in ab0) export BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab0/libbwagpu.so;; pf*) export BWAGPU_EXT_PREFETCH=${V#pf};; esac
  timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));print('$V', d['value'], d['parity_all_steps'], d['roofline']['isolated_launch_ms'])"
done
done
unset BWAGPU_LIB BWAGPU_EXT_PREFETCH
for pf in 0 1 3; do
BWAGPU_EXT_PREFETCH=$pf BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_pf$pf.json 2> $OUT/occ_pf$pf.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ_pf$pf.json'));b=d['batch0'];print($pf, b['split'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
done
echo done > $OUT/rc.txt
