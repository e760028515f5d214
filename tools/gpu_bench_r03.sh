#!/bin/bash
# Round-3 measurement session, phase 2: the bench lines (traffic from the
# committed profiles/r03_pmc_traffic*.json), one GPU step each.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-300
timeout -k 10 400 python3 bench.py --config C4 --steps 3 --warmup 1 --no-ingest > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
timeout -k 10 300 python3 bench.py --config C1 --no-ingest > $O/bench_c1.log 2>&1 || { tail -30 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | cut -c1-300
timeout -k 10 400 python3 bench.py --mode reference --no-ingest > $O/bench_refrule.log 2>&1 || { tail -30 $O/bench_refrule.log; exit 1; }
tail -1 $O/bench_refrule.log | cut -c1-300
timeout -k 10 400 python3 bench.py --mode sqr --steps 10 --warmup 2 --traffic-json profiles/r03_pmc_traffic_sqr.json > $O/bench_sqr.log 2>&1 || { tail -30 $O/bench_sqr.log; exit 1; }
tail -1 $O/bench_sqr.log | cut -c1-300
