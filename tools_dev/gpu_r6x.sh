#!/bin/bash
# row bound in extend_quad: parity on the spec tests, then the bench
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6x
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_c3_regime.py > $OUT/tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|FAILED" $OUT/tests.log | tail -15
for k in 1; do
  timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b$k.json 2> $OUT/b$k.err || { tail $OUT/b$k.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b$k.json'));c=d.get('c5_refseed',{})
print('$k', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline'].get('frac'), c.get('ms_per_batch'), c.get('parity_all_steps'), {k:(v['ms_per_batch'], v['parity_all_steps']) for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
