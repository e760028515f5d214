#!/bin/bash
# Round-3 final tree (in-place tile updates): every GPU test, smoke(), the
# tile probe, rocprofv3 kernel stats of the C2 bench command, then the C2, C4
# and C1 bench lines.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 60 ./tools/probe_tile > $O/probe_tile.log 2>&1 || { cat $O/probe_tile.log; exit 1; }
cat $O/probe_tile.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ingest > $O/prof_c2.log 2>&1 || { tail -30 $O/prof_c2.log; exit 1; }
grep socp_small $O/prof_c2/c2_kernel_stats.csv | cut -c1-150
timeout -k 10 500 python3 bench.py > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-300
timeout -k 10 400 python3 bench.py --config C4 --steps 3 --warmup 1 --no-ingest > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
timeout -k 10 300 python3 bench.py --config C1 --no-ingest > $O/bench_c1.log 2>&1 || { tail -30 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/prof_c4.log 2>&1 || { tail -30 $O/prof_c4.log; exit 1; }
grep socp_large $O/prof_c4/c4_kernel_stats.csv | cut -c1-150
