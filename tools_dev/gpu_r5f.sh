#!/bin/bash
# round-5 change check: issue microbenchmark, the touched tests, the bench
set -o pipefail
T=${1:-r5f}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 ./tools_dev/micro/issue > $OUT/issue.json || { echo issue failed; exit 1; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_host_stage.py tests/test_gpu_parity.py tests/test_abi.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel'], r.get('kernel_ms_per_step'), r['frac'], r['frac_pk16'], r['alg_bytes_per_launch'], r['traffic_over_alg'])
print('host_buffer_path', d.get('host_buffer_path'))
print('end_to_end', json.dumps(d.get('end_to_end')))"
