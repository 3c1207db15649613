#!/bin/bash
# round 6: claim-ahead in the phased kernel (BWAGPU_EXT_PREFETCH: eight
# entries claimed during a generation, their records loaded at the next,
# while more than PREFETCH x 1024 entries of the shard are left) — the stage's
# GPU tests at 1, C2 fixture / stream A/B over 0 / 1 / 2, occupancy split
set -o pipefail
T=${1:-r06u}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
BWAGPU_EXT_PREFETCH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for P in 1 0 2; do
  BWAGPU_EXT_PREFETCH=$P timeout -k 10 300 python -u bench.py --headline-only --workload c2_refseed > $OUT/fix_${P}_$rep.json 2> $OUT/fix_${P}_$rep.err || exit 3
  python3 -c "import json;d=json.load(open('$OUT/fix_${P}_$rep.json'));r=d['roofline'];print('fix pf $P', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'][:2])"
done
done
for P in 1 0; do
  BWAGPU_EXT_PREFETCH=$P timeout -k 10 300 python -u bench.py --headline-only > $OUT/str_$P.json 2> $OUT/str_$P.err || exit 4
  python3 -c "import json;d=json.load(open('$OUT/str_$P.json'));print('stream pf $P', d['value'], d['ms_per_step'], d['parity_all_steps'])"
  BWAGPU_EXT_PREFETCH=$P BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ_$P.json 2> $OUT/occ_$P.err || exit 5
  python3 -c "import json;d=json.load(open('$OUT/occ_$P.json'));b=d['batch0'];print('occ pf $P', b['split'], b['generations'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
done
echo done > $OUT/rc.txt
