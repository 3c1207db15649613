#!/bin/bash
# round 6: the final light pass without its inline extension (84 VGPRs; a miss
# goes to the redo pass) against -DBWAGPU_LIGHT_INLINE=1 (lib/ab1); the
# phased kernel at 2 workgroups per CU; parity of the redo fallback with the
# strict emulation off
set -o pipefail
T=${1:-r06p}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
AB1=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab1/libbwagpu.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BWAGPU_EMU_STRICT=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_nostrict.log 2>&1 || { echo "pytest (strict 0) failed"; tail -40 $OUT/gpu_tests_nostrict.log; exit 1; }
tail -1 $OUT/gpu_tests_nostrict.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_$tag.json 2> $OUT/fix_$tag.err || return 1
  python3 -c "import json;d=json.load(open('$OUT/fix_$tag.json'));r=d['roofline'];print('fix $tag', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['inline_extensions'][:2], r['isolated_launch_ms'][:1])"
}
for rep in 1 2; do
  run new_$rep X=1 || exit 3
  run inl_$rep BWAGPU_LIB=$AB1 || exit 3
  run bpc2_$rep BWAGPU_EXT2_BLOCKS_PER_CU=2 || exit 3
done
for V in new inl; do
  L=""; [ $V = inl ] && L="BWAGPU_LIB=$AB1"
  env $L X=1 timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));print('stream $V', d['value'], d['ms_per_step'], d['parity_all_steps'])"
done
timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5.json 2> $OUT/c5.err || exit 7
python3 -c "import json;a=json.load(open('$OUT/c5.json'));print('c5', a['ms_per_batch'], a['parity_all_steps'])"
echo done > $OUT/rc.txt
