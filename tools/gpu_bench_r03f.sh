#!/bin/bash
# Round-3 final tree, phase 2: the C4 and C2 bench lines (traffic from the
# committed profiles/r03_pmc_traffic*.json).
set -e
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 400 python3 bench.py --config C4 --steps 3 --warmup 1 --no-ingest > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
timeout -k 10 500 python3 bench.py > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-300
