#!/bin/bash
# Knock-out budget of the C2 solver kernel: interleaved timing of the variant
# libraries lib/v_* (tools/build_variant.sh) in one process, then their SQ
# instruction / wait counters (one --pmc pass).
set -e
export TMPDIR=/tmp
O=gpurun_out/ko
mkdir -p $O
LIBS="$*"
timeout -k 10 300 python3 tools/ab_multi.py C2 7 $LIBS > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq -o sq -- python3 tools/ab_multi.py C2 1 $LIBS > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
python3 tools/sq_variants.py $O/sq $((65536*8)) $LIBS
