#!/bin/bash
# C2 stage bench, quad vs pair forms (+ the whole-pipeline leg when asked)
set -o pipefail
T=${1:-b2}; E2E=${2:-0}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
X="--no-e2e"; [ "$E2E" = "1" ] && X=""
timeout -k 10 600 python -u bench.py --no-cpu --no-cigar --no-host-path --no-regime --no-seeding $X > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel','kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms')}, d.get('end_to_end_align'))"
timeout -k 10 300 python -u bench.py --ext-form 1 --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/bench_pair.json 2> $OUT/bench_pair.err || { tail $OUT/bench_pair.err; exit 4; }
python3 -c "import json;d=json.load(open('$OUT/bench_pair.json'));r=d['roofline'];print('pair',d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel','kernel_ms_per_step','kernel_sum_ms_per_step','frac','frac_step','frac_isolated','isolated_launch_ms')})"
