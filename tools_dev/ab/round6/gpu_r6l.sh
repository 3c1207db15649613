#!/bin/bash
# round 6: spec_sidep_kernel with the producer at a raised priority and the
# queue's tail left to the DP waves' own claims (BWAGPU_SIDEP_RETIRE) —
# the stage's GPU tests, C2 fixture A/B over RETIRE and against
# BWAGPU_EXT_PRODUCER=0, the occupancy / clock split of the producer form
set -o pipefail
T=${1:-r06l}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for V in p1r1024 p1r0 p1r4096 p0r0; do
  P=${V:1:1}; R=${V#*r}
  BWAGPU_EXT_PRODUCER=$P BWAGPU_SIDEP_RETIRE=$R timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));r=d['roofline'];print('fix $V', d['value'], d['parity_all_steps'], r['isolated_launch_ms'][:2], r['kernel_ms_per_step'], r['frac'])"
done
done
for V in p1r1024 p1r0; do
P=${V:1:1}; R=${V#*r}
BWAGPU_EXT_PRODUCER=$P BWAGPU_SIDEP_RETIRE=$R BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_$V.json 2> $OUT/occ_$V.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ_$V.json'));b=d['batch0'];print('occ $V', d['kernel'], b['split'], b['row_occupancy'], b['generations'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
done
echo done > $OUT/rc.txt
