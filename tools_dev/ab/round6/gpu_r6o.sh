#!/bin/bash
# round 6: the emulate pass gives uncertain skips round-B tasks too
# (BWAGPU_EMU_STRICT=1), so the final light pass has no inline extension —
# the stage's GPU tests with it on, C2 fixture / stream / c5 A/B, traces
set -o pipefail
T=${1:-r06o}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
BWAGPU_EMU_STRICT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for V in 1 0; do
  BWAGPU_EMU_STRICT=$V timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));r=d['roofline'];print('fix strict $V', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['tasks_round_a_b'][:2], r['inline_extensions'][:2], r['isolated_launch_ms'][:2])"
done
done
for V in 1 0; do
  BWAGPU_EMU_STRICT=$V timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));print('stream strict $V', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline']['inline_extensions'][:4])"
  BWAGPU_EMU_STRICT=$V timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_$V.json 2> $OUT/c5_$V.err || exit 7
  python3 -c "import json;a=json.load(open('$OUT/c5_$V.json'));print('c5 strict $V', a['ms_per_batch'], a['parity_all_steps'])"
done
cd /tmp
BWAGPU_EMU_STRICT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --headline-only --workload c2_refseed --steps 20 > $OUT/tr1.json 2> $OUT/tr1.err || exit 5
cd $GRAFT_REPO_ROOT
python3 tools_dev/trace_busy.py $OUT/tr1/run_kernel_trace.csv 3 20 "spec_side4_kernel<16, 10, true>" > $OUT/busy1.json
python3 -c "
import json,csv
d=json.load(open('$OUT/busy1.json'));print('busy strict', d['window_ms_per_step'], d['gpu_busy_ms_per_step'], d['kernel_busy_ms_per_step'])
for r in csv.DictReader(open('$OUT/tr1/run_kernel_stats.csv')):
    if 'select_light' in r['Name'] or 'scan_kernel' in r['Name']: print('  ', r['Name'][:40], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
echo done > $OUT/rc.txt
