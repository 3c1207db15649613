#!/bin/bash
# round 6: the new stream bench (default line) + the GPU tests it adds + the
# end_to_end host-settings sweep
set -o pipefail
T=${1:-r06b}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_c2_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
[ $rc -ge 124 ] && { tail $OUT/bench.err; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['parity_all_steps'])" || tail -20 $OUT/bench.err
timeout -k 10 600 python -u tools_dev/e2e_sweep.py 20 > $OUT/e2e_sweep.jsonl 2> $OUT/e2e_sweep.err; rc=$?
[ $rc -ge 124 ] && exit $rc
echo done > $OUT/rc.txt
