# A/B of two builds of libbwagpu.so (default lib/ vs $2) on realbench + bench
set -o pipefail
TAG=${1:-ablib}; ALT=${2}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_sam_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for L in "" "$ALT"; do
  if [ -n "$L" ]; then export BWAGPU_LIB=$GRAFT_REPO_ROOT/$L; fi
  timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/rb.json 2> $OUT/rb.err || { tail $OUT/rb.err; exit 2; }
  timeout -k 10 200 python bench.py --no-cpu --no-cigar --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "import json; r=json.load(open('$OUT/rb.json')); d=json.load(open('$OUT/b.json')); print('lib=$L', 'realbench', r['ms_per_batch'], 'redo', r['redo_reads'], r['redo_inline'], 'bench', d['value'], d['ms_per_step'], d['parity_all_steps'])"
  BWAGPU_LIB= python3 -c "pass"
done
timeout -k 10 200 python bench.py --no-cpu --no-cigar --no-host-path --streams 1 > $OUT/b1.json 2> $OUT/b1.err && python3 -c "import json; d=json.load(open('$OUT/b1.json')); print('1 stream (alt lib)', d['value'], d['ms_per_step'])"
