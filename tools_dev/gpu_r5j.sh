#!/bin/bash
# probed side streams: regime-state tool, bench with regime, stream counts, trace
set -o pipefail
T=${1:-r5j}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/regime_state_ab.py > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 4; }
echo "probed sides" $(cat $OUT/st.json)
timeout -k 10 300 python -u tools_dev/regime_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail $OUT/ab.err; exit 2; }
cat $OUT/ab.json
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
for ns in 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime --streams $ns > $OUT/bs$ns.json 2> $OUT/bs$ns.err || { tail $OUT/bs$ns.err; exit 7; }
  python3 -c "
import json;d=json.load(open('$OUT/bs$ns.json'));r=d['roofline']
print('streams $ns', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
