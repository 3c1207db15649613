#!/bin/bash
# round 6: the final light pass takes the reads with a round-B task first and
# claims the rest (BWAGPU_LIGHT_RISKY_FIRST) — the stage's GPU tests, C2
# fixture + stream A/B, a kernel trace of each (select_light<1>'s spread)
set -o pipefail
T=${1:-r06n}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for V in 1 0; do
  BWAGPU_LIGHT_RISKY_FIRST=$V timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));r=d['roofline'];print('fix risky $V', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
done
for V in 1 0; do
  BWAGPU_LIGHT_RISKY_FIRST=$V timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$V.json 2> $OUT/str_$V.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$V.json'));print('stream risky $V', d['value'], d['ms_per_step'], d['parity_all_steps'])"
done
cd /tmp
for V in 1 0; do
BWAGPU_LIGHT_RISKY_FIRST=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr$V -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --headline-only --workload c2_refseed --steps 20 > $OUT/tr$V.json 2> $OUT/tr$V.err || exit 5
done
cd $GRAFT_REPO_ROOT
for V in 1 0; do
python3 tools_dev/trace_busy.py $OUT/tr$V/run_kernel_trace.csv 3 20 "spec_side4_kernel<16, 10, true>" > $OUT/busy$V.json
python3 -c "
import json,csv
d=json.load(open('$OUT/busy$V.json'));print('busy $V', d['window_ms_per_step'], d['gpu_busy_ms_per_step'], d['kernel_busy_ms_per_step'])
for r in csv.DictReader(open('$OUT/tr$V/run_kernel_stats.csv')):
    if 'select_light<1>' in r['Name'] or 'scan_kernel<1>' in r['Name']: print('  ', r['Name'][:40], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
done
echo done > $OUT/rc.txt
