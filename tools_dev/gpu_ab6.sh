#!/bin/bash
# every -m gpu test on the default build, then the stage bench + GRCh38-regime legs A/B
# against lib/alt/libbwagpu.so (alternating), then the per-read selection trace
set -o pipefail
T=${1:-ab6}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $OUT/gpu_tests.log
for k in 1 2; do
for L in "" bwa-flow_amd/lib/alt/libbwagpu.so; do
  if [ -n "$L" ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/$L; else unset BWAGPU_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding $BARGS > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];g=d.get('regime_grch38',{})
print('lib=${L:-default}',d['value'],d['ms_per_step'],d['parity_all_steps'],r['kernel_ms_per_step'],{k:(v['ms_per_batch'],v['parity_all_steps']) for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
done
unset BWAGPU_LIB
timeout -k 10 300 python -u tools_dev/spec_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 4; }
timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste.json 2> $OUT/waste.err || { tail $OUT/waste.err; exit 5; }
