#!/bin/bash
# round 6: the side kernel with a producer wave (spec_sidep_kernel) — the
# stage's GPU tests, C2 fixture A/B against BWAGPU_EXT_PRODUCER=0
# (spec_side4_kernel), occupancy + clock split of both, c5_refseed, stream
set -o pipefail
T=${1:-r06k}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py tests/test_gpu_chain.py tests/test_host_stage.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for P in 1 0; do
  BWAGPU_EXT_PRODUCER=$P timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${P}_$rep.json 2> $OUT/fix_${P}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${P}_$rep.json'));r=d['roofline'];print('fix prod $P', d['value'], d['parity_all_steps'], r['kernel'], r['isolated_launch_ms'][:2], r['kernel_ms_per_step'], r['frac'])"
done
done
for P in 1 0; do
BWAGPU_EXT_PRODUCER=$P BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_$P.json 2> $OUT/occ_$P.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ_$P.json'));b=d['batch0'];print('occ prod $P', b['split'], b['row_occupancy'], b['generations'], b['cycle_split'], b['parity'])"
done
timeout -k 10 300 python -u tools_dev/c5_prof.py > $OUT/c5.json 2> $OUT/c5.err || exit 7
python3 -c "import json;a=json.load(open('$OUT/c5.json'));print('c5', a['ms_per_batch'], a['parity_all_steps'])"
timeout -k 10 300 python -u bench.py --headline-only > $OUT/str.json 2> $OUT/str.err || exit 6
python3 -c "import json;d=json.load(open('$OUT/str.json'));print('stream', d['value'], d['parity_all_steps'], d['roofline']['frac'], d['roofline']['kernel'])"
echo done > $OUT/rc.txt
