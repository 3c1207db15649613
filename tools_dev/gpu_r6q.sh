#!/bin/bash
# select_light capped at 6 waves per SIMD (lib_sl6, 80 VGPRs: fits beside two extension waves) vs default
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6q
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_sl6/libbwagpu.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c2_batch.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 6; }
tail -1 $OUT/tests.log
for v in def sl6 def sl6; do
  L=""; [ $v = sl6 ] && L="BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_sl6/libbwagpu.so"
  env $L timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('$v', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
