#!/bin/bash
# round 6: the phased extension (spec_side4_kernel) — parity on every GPU test
# file of the stage, A/B against BWAGPU_EXT_PHASED=0 (the task-state kernel),
# occupancy + clock split of both
set -o pipefail
T=${1:-r06h}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py tests/test_host_stage.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2 3; do
for V in ph0 ph1; do
  export BWAGPU_EXT_PHASED=${V#ph}
  timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${V}_$rep.json 2> $OUT/fix_${V}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${V}_$rep.json'));print('$V', d['value'], d['parity_all_steps'], d['roofline']['isolated_launch_ms'], d['roofline']['kernel_ms_per_step'])"
done
done
for V in ph0 ph1; do
BWAGPU_EXT_PHASED=${V#ph} BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_$V.json 2> $OUT/occ_$V.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ_$V.json'));b=d['batch0'];print('$V', b['split'], b['row_occupancy'], b['generations'], b['cycle_split'], b['parity'])"
done
unset BWAGPU_EXT_PHASED
timeout -k 10 300 python -u bench.py --headline-only > $OUT/str.json 2> $OUT/str.err || exit 6
python3 -c "import json;d=json.load(open('$OUT/str.json'));print('stream', d['value'], d['parity_all_steps'], d['roofline']['frac'])"
BWAGPU_EXT_PHASED=0 timeout -k 10 300 python -u bench.py --headline-only > $OUT/str0.json 2> $OUT/str0.err || exit 6
python3 -c "import json;d=json.load(open('$OUT/str0.json'));print('stream ph0', d['value'], d['parity_all_steps'], d['roofline']['frac'])"
timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_ph1.json 2> $OUT/c5_ph1.err || exit 7
BWAGPU_EXT_PHASED=0 timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5_ph0.json 2> $OUT/c5_ph0.err || exit 7
python3 -c "import json;a=json.load(open('$OUT/c5_ph1.json'));b=json.load(open('$OUT/c5_ph0.json'));print('c5', a['ms_per_batch'], a['parity_all_steps'], b['ms_per_batch'], b['parity_all_steps'])"
echo done > $OUT/rc.txt
