#!/bin/bash
# round 6: C5's second bin at four calls per wave (BWAGPU_BIN1_G32=1), task
# state machine and phased (mask 3), against the default — c5_refseed and the
# regime legs, parity on every step
set -o pipefail
T=${1:-r06y}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for V in base g32 g32ph; do
  E="X=1"; [ $V = g32 ] && E="BWAGPU_BIN1_G32=1"; [ $V = g32ph ] && E="BWAGPU_BIN1_G32=1 BWAGPU_EXT_PHASED=3"
  env $E timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_${V}_$rep.json 2> $OUT/c5_${V}_$rep.err || exit 7
  python3 -c "import json;a=json.load(open('$OUT/c5_${V}_$rep.json'));print('c5 $V', a['ms_per_batch'], a['parity_all_steps'])"
done
done
echo done > $OUT/rc.txt
