#!/bin/bash
# round 6 (second session): extend_quad's band trim from one bit per column
# and the shared gap-open subtraction (o_del == o_ins), against the tree
# before them (lib/ab0 = ea27e67): the extension parity tests, then the C2
# fixture / stream headline and c5_refseed, new and old alternating
set -o pipefail
T=${1:-r06z}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
AB0=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab0/libbwagpu.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_variants.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_$tag.json 2> $OUT/fix_$tag.err || return 1
  python3 -c "import json;d=json.load(open('$OUT/fix_$tag.json'));r=d['roofline'];print('fix $tag', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'][:2])"
}
for rep in 1 2; do
  run new_$rep X=1 || exit 3
  run old_$rep BWAGPU_LIB=$AB0 || exit 3
done
for V in new old; do
  L="X=1"; [ $V = old ] && L="BWAGPU_LIB=$AB0"
  env $L timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));r=d['roofline'];print('stream $V', d['value'], d['ms_per_step'], d['parity_all_steps'], r['frac'], r['kernel_ms_per_step'])"
done
for V in new old; do
  L="X=1"; [ $V = old ] && L="BWAGPU_LIB=$AB0"
  env $L timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$V.json 2> $OUT/c5_$V.err || exit 5
  python3 -c "import json;a=json.load(open('$OUT/c5_$V.json'));print('c5 $V', a['ms_per_batch'], a['parity_all_steps'])"
done
echo done > $OUT/rc.txt
