#!/bin/bash
# Interleaved C2 timing of variant libraries lib/v_* in one process (tuning).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python3 tools/ab_multi.py C2 ${REPS:-9} "$@" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.log
