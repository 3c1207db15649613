#!/bin/bash
# second length bin kernel capped at 256 VGPRs (lib_cap) vs uncapped (default)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6w
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_cap/libbwagpu.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for v in def cap def cap; do
  L=""; [ $v = cap ] && L="BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_cap/libbwagpu.so"
  env $L timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));c=d.get('c5_refseed',{})
print('$v', d['value'], d['ms_per_step'], d['parity_all_steps'], c.get('ms_per_batch'), {k:(v['ms_per_batch'], v['parity_all_steps']) for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
