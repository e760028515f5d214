#!/bin/bash
# Rank-update plugin (socp_sqr_*): its GPU tests, PMC traffic of the setup
# kernel (FETCH_SIZE / WRITE_SIZE, one counter per pass), the --mode sqr bench
# line and a rocprofv3 kernel-stats pass of the same command.
set -e
export TMPDIR=/tmp
O=gpurun_out/sqr
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sqr.py -x -q --tb=line --timeout 120 --timeout-method thread > $O/pytest_sqr.log 2>&1 || { tail -60 $O/pytest_sqr.log; exit 1; }
tail -3 $O/pytest_sqr.log
if [ -z "$NO_PMC" ]; then
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- python3 bench.py --mode sqr --steps 1 --warmup 0 --no-cpu > $O/pmc_f.log 2>&1 || { tail -20 $O/pmc_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- python3 bench.py --mode sqr --steps 1 --warmup 0 --no-cpu > $O/pmc_w.log 2>&1 || { tail -20 $O/pmc_w.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_f $O/pmc_w C2 65536 1 $O/pmc_traffic_sqr.json socp_sqr_setup_kernel
fi
timeout -k 10 300 python bench.py --mode sqr --steps 10 --warmup 2 --traffic-json $O/pmc_traffic_sqr.json > $O/bench_sqr.log 2>&1 || { tail -30 $O/bench_sqr.log; exit 1; }
tail -1 $O/bench_sqr.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sqr -o sqr -- python3 bench.py --mode sqr --steps 10 --warmup 2 --no-cpu > $O/prof_sqr.log 2>&1 || { tail -30 $O/prof_sqr.log; exit 1; }
find $O/prof_sqr -name "*kernel_stats.csv"
