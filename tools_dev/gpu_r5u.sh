#!/bin/bash
set -o pipefail
T=${1:-r5u}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for L in "" gpurun_ab/fill2/libbwagpu.so "" gpurun_ab/fill2/libbwagpu.so; do
  if [ -n "$L" ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/$L; else unset BWAGPU_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 7; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('lib [$L]', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'])"
done
