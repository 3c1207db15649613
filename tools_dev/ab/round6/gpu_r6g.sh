#!/bin/bash
# round 6: the diag build's start split (claim / task record / fill), and the
# C5 second-bin kernel's trace + PMC (spec_ext4_kernel<16,16,false>)
set -o pipefail
T=${1:-r06g}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib/diag/libbwagpu.so timeout -k 10 300 python -u tools_dev/occ_diag.py 1 > $OUT/occ.json 2> $OUT/occ.err || exit 5
python3 -c "import json;d=json.load(open('$OUT/occ.json'));b=d['batch0'];print(b['split'], b['cycle_split'], b['cycles_per_generation'], b['parity'])"
cd /tmp
C="$GRAFT_REPO_ROOT/tools_dev/c5_prof.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5trace -o run --output-format csv -- python3 $C > $OUT/c5trace.json 2> $OUT/c5trace.err || exit 6
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/c5pmc_a -o a --output-format csv -- python3 $C > $OUT/c5pmc_a.json 2> $OUT/c5pmc_a.err || exit 7
cd $GRAFT_REPO_ROOT
echo done > $OUT/rc.txt
