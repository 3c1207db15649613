# GPU check + A/B of the packed extension bodies (extend_wave_pk<1|2>): their
# own tests first (a four-column failure turns that body off for the rest and
# is reported), the parity suites, smoke, then the bench with packing on / off
# usage (on the GPU box): bash tools_dev/gpu_packed.sh <tag>
set -o pipefail
TAG=${1:-packed}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_parity.py -k two_segment > $OUT/p2_tests.log 2>&1 || { echo "two-segment tests failed"; tail -30 $OUT/p2_tests.log; exit 1; }
tail -1 $OUT/p2_tests.log
timeout -k 10 300 $PT tests/test_gpu_parity.py -k four_column > $OUT/p4_tests.log 2>&1
rc=$?
tail -1 $OUT/p4_tests.log
if [ $rc -eq 1 ]; then echo "four-column tests failed: BWAGPU_EXT_P4=0 from here"; tail -30 $OUT/p4_tests.log; export BWAGPU_EXT_P4=0
elif [ $rc -ne 0 ]; then echo "four-column tests rc=$rc"; exit 1; fi
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_cigar.py -k "not packed" > $OUT/gpu_tests.log 2>&1 || { echo "parity tests failed"; tail -40 $OUT/gpu_tests.log; exit 2; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
for k in 1 2; do for v in 1 0; do
  BWAGPU_EXT_P2=$v timeout -k 10 200 python bench.py --pairs 300000 --steps 18 --warmup 2 --no-cpu --no-host-path --no-cigar > $OUT/c2_$v$k.json 2> $OUT/c2_$v$k.err || { tail -20 $OUT/c2_$v$k.err; exit 4; }
  python -c "import json;d=json.load(open('$OUT/c2_$v$k.json'));print('C2 p2=$v', d['value'], d['ms_per_step'], d['gcups'])"
done; done
if [ -z "$BWAGPU_EXT_P4" ]; then for v in 1 0; do
  BWAGPU_EXT_P4=$v timeout -k 10 200 python bench.py --pairs 300000 --read-len 0 --steps 12 --warmup 2 --no-cpu --no-host-path --no-cigar > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -20 $OUT/c5_$v.err; exit 5; }
  python -c "import json;d=json.load(open('$OUT/c5_$v.json'));print('C5 p4=$v', d['value'], d['ms_per_step'], d['gcups'])"
done; fi
timeout -k 10 300 python bench.py --pairs 300000 --steps 10 --warmup 2 --no-host-path --cpu-budget 5 > $OUT/bench_cigar.json 2> $OUT/bench_cigar.err || { tail -20 $OUT/bench_cigar.err; exit 6; }
python -c "import json;d=json.load(open('$OUT/bench_cigar.json'));print(d['value'], d.get('parity_batch0_vs_cpu'), d.get('cigar_stage'))"
