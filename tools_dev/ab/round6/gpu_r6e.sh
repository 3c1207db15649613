#!/bin/bash
# round 6: task state parked in non-volatile LDS — parity, A/B against lib/ab1
# (the previous commit), the cycle split of the diag build
set -o pipefail
T=${1:-r06e}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2 3; do
for V in ab1 new; do
  unset BWAGPU_LIB
  [ $V = ab1 ] && export BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab1/libbwagpu.so
  timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));print('$V', d['value'], d['parity_all_steps'], d['roofline']['isolated_launch_ms'])"
done
done
unset BWAGPU_LIB
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ.json 2> $OUT/occ.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ.json'));b=d['batch0'];print(b['split'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
timeout -k 10 300 python -u bench.py --headline-only > $OUT/str.json 2> $OUT/str.err || exit 6
python3 -c "import json;d=json.load(open('$OUT/str.json'));print('stream', d['value'], d['parity_all_steps'], d['roofline']['frac'])"
echo done > $OUT/rc.txt
