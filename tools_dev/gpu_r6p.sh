#!/bin/bash
# library pass pool: submit/seeding tests, then host path + end-to-end twice
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6p
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_host_stage.py tests/test_gpu_seed.py tests/test_gpu_chain.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));h=d['host_buffer_path'];e=d.get('end_to_end',{})
print(d['value'], h['value'], h['ms_per_batch'], h['parity_last_batches'], e.get('value'), e.get('parity_last_rep'), e.get('ms_per_record'), e.get('chains_forwarded',{}).get('value'))"
done
