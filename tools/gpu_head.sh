#!/bin/bash
# Head check: every GPU test, smoke(), the C2 and C4 bench lines (no CPU legs).
set -e
export TMPDIR=/tmp
O=gpurun_out/head
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --tb=short --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -40; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --no-cpu --no-ingest > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-400
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-400
timeout -k 10 200 python bench.py --config C1 --no-cpu --no-ingest > $O/bench_c1.log 2>&1 || { tail -30 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | cut -c1-400
