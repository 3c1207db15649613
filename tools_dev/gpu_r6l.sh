#!/bin/bash
# next-call refill (BWAGPU_EXT_REFILL=1): parity, then A/B against the default at three triggers
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6l
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_EXT_REFILL=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
run() {
  env $1 timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('$1', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), r['isolated_launch_ms'])"
}
run BWAGPU_EXT_REFILL=0
for t in 1 2 4; do run "BWAGPU_EXT_REFILL=1 BWAGPU_RF_TRIG=$t"; done
run BWAGPU_EXT_REFILL=0
