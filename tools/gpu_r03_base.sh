#!/bin/bash
# Round-3 lease: the two-wave overlap probe, the rank-update tests, then every GPU test, smoke(), the default bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 120 ./tools/probe_overlap2 > $O/probe_overlap2.log 2>&1 || { cat $O/probe_overlap2.log; exit 1; }
cat $O/probe_overlap2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sqr.py -x -q --timeout 120 --timeout-method thread > $O/pytest_sqr.log 2>&1 || { tail -40 $O/pytest_sqr.log; exit 1; }
tail -2 $O/pytest_sqr.log
bash tools/gpu_final.sh
