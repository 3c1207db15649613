#!/bin/bash
# round 6 (second session): extend_quad variants — the band trim (TRIM_BITS
# 0: per-column selects without the lower-bound mask, 1: one bit per column,
# serial, 2: two interleaved bit chains) x the shared gap-open subtraction
# (SYM) — against ab0 (ea27e67): extension parity per variant, then the C2
# fixture headline (isolated round A / B launches), interleaved, two reps
set -o pipefail
T=${1:-r06z2}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/bwa-flow_amd/lib
for V in v1 v2 v3 v4; do
  BWAGPU_LIB=$L/$V/libbwagpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/par_$V.log 2>&1 || { echo "parity $V failed"; tail -20 $OUT/par_$V.log; exit 1; }
  echo "parity $V $(tail -1 $OUT/par_$V.log)"
done
for rep in 1 2; do
for V in ab0 v1 v2 v3 v4 cur; do
  P=$L/$V/libbwagpu.so; [ $V = cur ] && P=$L/libbwagpu.so
  BWAGPU_LIB=$P timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));r=d['roofline'];print('fix ${V} $rep', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'][:2])"
done
done
echo done > $OUT/rc.txt
