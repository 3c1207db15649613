#!/bin/bash
# the PMC passes alone (SQ + FETCH/WRITE: roofline.traffic of this source
# digest), plus the headline at 2 / 4 caller streams beside the default 3
set -o pipefail
T=${1:-r06x}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
bash tools_dev/gpu_pmc4.sh $T/pmc all --headline-only --stream-batches 8 > /dev/null || exit 5
cd $GRAFT_REPO_ROOT
for S in 2 4 3; do
  timeout -k 10 300 python -u bench.py --headline-only --streams $S > $OUT/str_$S.json 2> $OUT/str_$S.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$S.json'));print('streams $S', d['value'], d['ms_per_step'], d['parity_all_steps'], d['host_enqueue_ms_per_step'])"
done
echo done > $OUT/rc.txt
