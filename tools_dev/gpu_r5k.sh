#!/bin/bash
set -o pipefail
T=${1:-r5k}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/e2e_ab.py > $OUT/e.json 2> $OUT/e.err || { tail $OUT/e.err; exit 1; }
cat $OUT/e.json
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime --no-e2e --steps 4 > $OUT/h.json 2> $OUT/h.err || { tail $OUT/h.err; exit 3; }
python3 -c "
import json;d=json.load(open('$OUT/h.json'))
print('host_buffer_path', d.get('host_buffer_path'))"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_host_stage.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
