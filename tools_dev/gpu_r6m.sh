#!/bin/bash
# oct kernel at <= 168 VGPRs (BWAGPU_EXT_W3=1) vs default: parity, then A/B
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6m
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_EXT_W3=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for w in 0 1 0 1; do
  BWAGPU_EXT_W3=$w timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('w3=$w', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), r['isolated_launch_ms'])"
done
