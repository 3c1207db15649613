#!/bin/bash
# round 6: the strict emulation's uncertain set narrowed (pending, extended
# after a pending one, uncertain skips) against round 6's first form (every
# seed from the first pending one; lib/ab1 = commit e577363) — stage tests,
# C2 fixture / stream / c5 A/B, round-B task counts
set -o pipefail
T=${1:-r06q}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
AB1=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab1/libbwagpu.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_$tag.json 2> $OUT/fix_$tag.err || return 1
  python3 -c "import json;d=json.load(open('$OUT/fix_$tag.json'));r=d['roofline'];print('fix $tag', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['tasks_round_a_b'][:2], r['inline_extensions'][:2], r['isolated_launch_ms'][:1])"
}
for rep in 1 2; do
  run new_$rep X=1 || exit 3
  run old_$rep BWAGPU_LIB=$AB1 || exit 3
done
for V in new old; do
  L="X=1"; [ $V = old ] && L="BWAGPU_LIB=$AB1"
  env $L timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));print('stream $V', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline']['inline_extensions'][:3])"
  env $L timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$V.json 2> $OUT/c5_$V.err || exit 7
  python3 -c "import json;a=json.load(open('$OUT/c5_$V.json'));print('c5 $V', a['ms_per_batch'], a['parity_all_steps'])"
done
echo done > $OUT/rc.txt
