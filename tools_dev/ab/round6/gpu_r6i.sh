#!/bin/bash
# round 6: the phased extension per length bin (BWAGPU_EXT_PHASED mask) —
# the stage's GPU tests at the default, c5_refseed at masks 0-3, C2 at 0 / 1
set -o pipefail
T=${1:-r06i}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py tests/test_host_stage.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for M in 0 1 2 3; do
  BWAGPU_EXT_PHASED=$M timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$M.json 2> $OUT/c5_$M.err || exit 7
  python3 -c "import json;a=json.load(open('$OUT/c5_$M.json'));print('c5 mask $M', a['ms_per_batch'], a['parity_all_steps'])"
done
for M in 1 0; do
  BWAGPU_EXT_PHASED=$M timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_$M.json 2> $OUT/fix_$M.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_$M.json'));print('fix mask $M', d['value'], d['parity_all_steps'], d['roofline']['isolated_launch_ms'])"
done
echo done > $OUT/rc.txt
