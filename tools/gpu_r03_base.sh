#!/bin/bash
# Round-3 first lease: the two-wave overlap probe, then every GPU test, smoke(), the default bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 120 ./tools/probe_overlap2 > $O/probe_overlap2.log 2>&1 || { cat $O/probe_overlap2.log; exit 1; }
cat $O/probe_overlap2.log
bash tools/gpu_final.sh
