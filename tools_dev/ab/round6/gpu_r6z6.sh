#!/bin/bash
# round 6 (second session): the lane F of pass 1 as a tree (BWAGPU_QUAD_TTREE, lib = default) against
# the serial recursion (lib/t0): extension parity, C2 fixture (isolated round A / B), c5_refseed
set -o pipefail
T=${1:-r06z6}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/bwa-flow_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/par.log 2>&1 || { echo "parity failed"; tail -20 $OUT/par.log; exit 1; }
echo "parity $(tail -1 $OUT/par.log)"
for rep in 1 2 3; do
for V in t0 cur; do
  P=$L/$V/libbwagpu.so; [ $V = cur ] && P=$L/libbwagpu.so
  BWAGPU_LIB=$P timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));r=d['roofline'];print('fix ${V} $rep', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'][:2])"
done
done
for V in t0 cur; do
  P=$L/$V/libbwagpu.so; [ $V = cur ] && P=$L/libbwagpu.so
  BWAGPU_LIB=$P timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$V.json 2> $OUT/c5_$V.err || exit 5
  python3 -c "import json;a=json.load(open('$OUT/c5_$V.json'));print('c5 $V', a['ms_per_batch'], a['parity_all_steps'])"
done
echo done > $OUT/rc.txt
