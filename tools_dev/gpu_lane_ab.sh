#!/bin/bash
# A/B of the lane-per-seed extension kernel (BWAGPU_EXT_LANE 0/1/2): parity
# first (every spec-path GPU test with the default), then the stage bench
# (+ C3/C5 legs) with each setting and a rocprofv3 kernel summary of the
# default.  Run under gpurun; outputs in gpurun_out/$1.
set -o pipefail
T=${1:-laneab}
mkdir -p gpurun_out/$T
BWAGPU_EXT_LANE=${TESTLANE:-2} timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for sp in ${MODES:-0:2 2:2 0:4 2:4 1:4}; do
  p=${sp%%:*}; S=${sp##*:}
  BWAGPU_EXT_LANE=$p timeout -k 10 200 python -u bench.py --no-cpu --no-host-path --no-cigar --no-seeding --no-e2e --steps 30 --streams $S \
    > gpurun_out/$T/bench_l${p}_s$S.json 2>> gpurun_out/$T/bench.err || exit 1
  python -c "import json,sys;d=json.load(open('gpurun_out/$T/bench_l${p}_s$S.json'));r=d['roofline'];g=d.get('regime_grch38',{});print('lane=$p streams=$S',d['value'],d['ms_per_step'],d['parity_all_steps'],r['avg_launch_ms'],r['frac'],g.get('c3',{}).get('ms_per_batch'),g.get('c5',{}).get('ms_per_batch'),g.get('c3',{}).get('parity_all_steps'),g.get('c5',{}).get('parity_all_steps'))" | tee -a gpurun_out/$T/summary.txt
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/$T/prof.log 2>&1 || exit 3
head -12 $GRAFT_REPO_ROOT/gpurun_out/$T/prof/run_kernel_stats.csv | cut -c1-160
# the drop-in stage end to end: stage workers 2/3/4 with submit's phase timing
cd $GRAFT_REPO_ROOT
[ "$E2EW" = "0" ] && exit 0
for wk in ${E2EW:-2 3 4}; do
  BWAGPU_SUBMIT_PROF=1 BWAGPU_E2E_WORKERS=$wk timeout -k 10 200 python -u bench.py --no-cpu --no-cigar --no-seeding --no-e2e --no-regime --steps 5 \
    > gpurun_out/$T/e2e_w$wk.json 2> gpurun_out/$T/e2e_w$wk.err || exit 4
  python -c "import json;d=json.load(open('gpurun_out/$T/e2e_w$wk.json'));e=d['end_to_end'];print('workers=$wk',e['value'],e['phases'],e['parity_last_rep'],d['host_buffer_path']['value'])" | tee -a gpurun_out/$T/summary.txt
  grep -i "submit" gpurun_out/$T/e2e_w$wk.err | tail -4
done
