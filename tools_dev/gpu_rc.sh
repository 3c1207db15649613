#!/bin/bash
# spec-path parity tests, then the C2 stage bench and the GRCh38-regime legs (C3, C5, c3_refseed)
set -o pipefail
T=${1:-rc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 2; }
tail -1 $OUT/t.log
timeout -k 10 600 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));print(d['value'],d['ms_per_step'],d['parity_all_steps'])
g=d.get('regime_grch38',{})
for k,v in g.items():
  if isinstance(v,dict): print(k, {x:v[x] for x in v if x in ('ms_per_batch','value','parity_all_steps','ext_busy_ms_per_batch')})"
timeout -k 10 300 python -u tools_dev/spec_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 4; }
timeout -k 10 300 python -u tools_dev/spec_waste.py > $OUT/waste.json 2> $OUT/waste.err || { tail $OUT/waste.err; exit 5; }
