#!/bin/bash
# refill policy matrix: (slack, trigger, drain) -> headline bench (parity per step in the line)
set -o pipefail
T=${1:-r5z}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {
  env $1 timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('$1', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), r['isolated_launch_ms'])"
}
run BWAGPU_EXT_REFILL=0
for cfg in "1 1 0" "16 4 1" "1 4 1" "2 2 1" "1 2 1"; do
  set -- $cfg
  run "BWAGPU_EXT_REFILL=1 BWAGPU_RF_SLACK=$1 BWAGPU_RF_TRIG=$2 BWAGPU_RF_DRAIN=$3"
done
run BWAGPU_EXT_REFILL=0
