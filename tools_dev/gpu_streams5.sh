#!/bin/bash
# stage bench by caller-stream count, alternating
set -o pipefail
T=${1:-st5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2; do for ns in ${NSTREAMS:-2 3 4}; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --streams $ns > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('streams',$ns,d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','frac','frac_isolated')})"
done; done
