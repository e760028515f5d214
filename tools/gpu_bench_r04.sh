#!/bin/bash
# Round-4 bench lines (traffic from the committed profiles/r04_pmc_traffic*.json),
# one GPU step each; then the default bench command under rocprofv3 --stats.
set -e
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
grep '^{' $O/bench_c2.log | cut -c1-200
timeout -k 10 400 python3 bench.py --config C4 --steps 3 --warmup 1 --no-ingest > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | cut -c1-200
timeout -k 10 300 python3 bench.py --config C1 --no-ingest > $O/bench_c1.log 2>&1 || { tail -30 $O/bench_c1.log; exit 1; }
grep '^{' $O/bench_c1.log | cut -c1-200
timeout -k 10 400 python3 bench.py --mode reference --no-ingest > $O/bench_refrule.log 2>&1 || { tail -30 $O/bench_refrule.log; exit 1; }
grep '^{' $O/bench_refrule.log | cut -c1-200
timeout -k 10 400 python3 bench.py --mode sqr --steps 10 --warmup 2 > $O/bench_sqr.log 2>&1 || { tail -30 $O/bench_sqr.log; exit 1; }
grep '^{' $O/bench_sqr.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --no-cpu --no-ingest > $O/prof_c2.log 2>&1 || { tail -30 $O/prof_c2.log; exit 1; }
grep socp_small $O/prof_c2/c2_kernel_stats.csv | cut -c1-150
