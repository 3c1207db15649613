#!/bin/bash
# the end-to-end align leg alone (bench.end_to_end_align) at a few input sizes
set -o pipefail
T=${1:-e2e5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for p in ${PAIRS:-100000 300000}; do
  timeout -k 10 600 python -u -c "import bench, json; print(json.dumps(bench.end_to_end_align($p)))" > $OUT/e2e_$p.json 2> $OUT/e2e_$p.err || { tail $OUT/e2e_$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/e2e_$p.json')); print($p, d['value'], d['bwa_mem_cpu'], d['speedup_vs_bwa_mem'], d['sam_identical'], d['phases_s'])"
done
