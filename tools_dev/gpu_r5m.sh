#!/bin/bash
set -o pipefail
T=${1:-r5m}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/regime_ab.py --modes c2alt > $OUT/tr.json 2> $OUT/tr.err || { tail $OUT/tr.err; exit 3; }
bash tools_dev/gpu_strace.sh r5m_strace || exit 8
