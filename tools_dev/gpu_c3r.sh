#!/bin/bash
# the reference-seeded GRCh38-regime test + the regime bench leg
set -o pipefail
T=${1:-c3r}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py -k refseed -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 600 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step']); r=d['regime_grch38']; [print(k, {x: r[k][x] for x in ('ms_per_batch','value','parity_all_steps','ext_busy_ms_per_batch')}) for k in ('c3','c5','c3_refseed')]"
