#!/bin/bash
# headline at 2 vs 4 caller streams; host-buffer path at 3 vs 4 slots
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6h
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for cfg in "--streams 2 --host-slots 4" "--streams 4 --host-slots 3" "--streams 2 --host-slots 3" "--streams 4 --host-slots 4"; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime --no-e2e $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));h=d['host_buffer_path']
print('$cfg', d['value'], d['ms_per_step'], h['value'], h['ms_per_batch'], h['parity_last_batches'])"
done
