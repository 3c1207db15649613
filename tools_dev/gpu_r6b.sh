#!/bin/bash
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6b
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_host_stage.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools_dev/host_prof.py > $OUT/host.txt 2> $OUT/host.err || { tail $OUT/host.err; exit 5; }
cat $OUT/host.txt
for hs in 4 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime --host-slots $hs > $OUT/b$hs.json 2> $OUT/b.err || { tail $OUT/b.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$OUT/b$hs.json'));h=d['host_buffer_path'];e=d.get('end_to_end',{})
print('slots $hs', d['value'], h['value'], h['ms_per_batch'], h['parity_last_batches'], e.get('value'), e.get('ms_per_record'), e.get('chains_forwarded',{}).get('value'))"
done
