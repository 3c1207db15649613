#!/bin/bash
# round 6: FatTask prefetch in spec_ext4_kernel — parity, A/B against the
# previous library (lib/ab0), the occupancy split (lib/diag), one PMC pass
set -o pipefail
T=${1:-r06c}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for L in new ab0; do
  if [ $L = new ]; then unset BWAGPU_LIB; else export BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/ab0/libbwagpu.so; fi
  timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${L}_$rep.json 2> $OUT/fix_${L}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_${L}_$rep.json 2> $OUT/str_${L}_$rep.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/fix_${L}_$rep.json'));e=json.load(open('$OUT/str_${L}_$rep.json'));print('$L', d['value'], d['parity_all_steps'], d['roofline']['isolated_launch_ms'][0], e['value'], e['parity_all_steps'])"
done
done
unset BWAGPU_LIB
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_new.json 2> $OUT/occ.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ_new.json'));print(d['batch0']['split'], d['batch0']['row_occupancy'], d['batch0']['parity'])"
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --headline-only --workload c2_refseed --steps 5 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_a -o a --output-format csv -- python3 $B > $OUT/pmc_a.json 2> $OUT/pmc_a.err || exit 6
cd $GRAFT_REPO_ROOT
echo done > $OUT/rc.txt
timeout -k 10 900 python -u tools_dev/e2e_sweep.py 20 1 2 > $OUT/e2e_sweep.jsonl 2> $OUT/e2e_sweep.err; rc=$?
[ $rc -ge 124 ] && exit $rc
echo done2 > $OUT/rc2.txt
