#!/bin/bash
# wave-time breakdown of the packed extension kernel (diag build in lib_diag/); host-buffer path at 2/3/4 slots
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6a
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/time_diag.py > $OUT/time.json 2> $OUT/time.err || { tail $OUT/time.err; exit 5; }
cat $OUT/time.json
for hs in 2 3 4 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-regime --host-slots $hs > $OUT/b$hs.json 2> $OUT/b.err || { tail $OUT/b.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$OUT/b$hs.json'));h=d['host_buffer_path'];e=d.get('end_to_end',{})
print('slots $hs', d['value'], h['value'], h['ms_per_batch'], h['parity_last_batches'], e.get('value'))"
done
