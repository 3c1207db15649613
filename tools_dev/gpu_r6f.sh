#!/bin/bash
# parity of the extension kernels after a row-loop change, then the headline
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6f}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];c=d.get('c5_refseed',{})
print(d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), r['isolated_launch_ms'], c.get('ms_per_batch'), c.get('parity_all_steps'), {k:(v['ms_per_batch'], v['parity_all_steps']) for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
