#!/bin/bash
# round 6: the phased kernel with each call's query staged in LDS, against the
# tree before it (lib/ab1 = a0a106a) — C2 fixture and stream, occupancy split
set -o pipefail
T=${1:-r06t}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
AB1=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab1/libbwagpu.so
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_$tag.json 2> $OUT/fix_$tag.err || return 1
  python3 -c "import json;d=json.load(open('$OUT/fix_$tag.json'));r=d['roofline'];print('fix $tag', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'][:2])"
}
for rep in 1 2; do
  run new_$rep X=1 || exit 3
  run old_$rep BWAGPU_LIB=$AB1 || exit 3
done
for V in new old; do
  L="X=1"; [ $V = old ] && L="BWAGPU_LIB=$AB1"
  env $L timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));print('stream $V', d['value'], d['ms_per_step'], d['parity_all_steps'])"
done
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ.json 2> $OUT/occ.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ.json'));b=d['batch0'];print('occ', d['kernel'], b['split'], b['row_occupancy'], b['generations'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
echo done > $OUT/rc.txt
