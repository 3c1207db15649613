#!/bin/bash
set -o pipefail
T=${1:-r5i}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rt in 2 4; do
  BWAGPU_REAPER_THREADS=$rt timeout -k 10 300 python -u tools_dev/e2e_ab.py > $OUT/e$rt.json 2> $OUT/e$rt.err || { tail $OUT/e$rt.err; exit 1; }
  cat $OUT/e$rt.json
done
timeout -k 10 300 python -u tools_dev/regime_state_ab.py > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 4; }
echo "lazy slot streams" $(cat $OUT/st.json)
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_host_stage.py tests/test_gpu_parity.py tests/test_gpu_align2.py tests/test_gpu_cigar.py tests/test_gpu_seed.py tests/test_gpu_chain.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
