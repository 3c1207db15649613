#!/bin/bash
# round C over a long read's remaining seeds: parity, C5 counters/trace, the c5 legs
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6u
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_sam_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools_dev/c5_counters.py > $OUT/cnt.json 2> $OUT/cnt.err || { tail $OUT/cnt.err; exit 5; }
cat $OUT/cnt.json
timeout -k 10 300 python -u tools_dev/c5_redo_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 5; }
timeout -k 10 300 python -u tools_dev/c5_ab.py > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 5; }
cat $OUT/c5.json
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 4; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));c=d.get('c5_refseed',{})
print(d['value'], d['ms_per_step'], d['parity_all_steps'], c.get('ms_per_batch'), c.get('parity_all_steps'), {k:(v['ms_per_batch'], v['parity_all_steps']) for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
