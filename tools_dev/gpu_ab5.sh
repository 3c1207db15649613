#!/bin/bash
# parity of the default build, then stage-bench A/B against lib/alt/libbwagpu.so (alternating)
set -o pipefail
T=${1:-ab5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $OUT/gpu_tests.log
for k in 1 2; do
for L in "" bwa-flow_amd/lib/alt/libbwagpu.so; do
  if [ -n "$L" ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/$L; else unset BWAGPU_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding $BARGS > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('lib=${L:-default}',d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','frac','frac_isolated')})"
done
done
unset BWAGPU_LIB
timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste.json 2> $OUT/waste.err && cat $OUT/waste.json
