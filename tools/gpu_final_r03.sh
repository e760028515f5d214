#!/bin/bash
# Round-3 final tree, phase 1: every GPU test, smoke(), then the C4 PMC traffic
# (FETCH_SIZE, WRITE_SIZE; one counter per pass) and rocprofv3 kernel stats of
# the C4 bench command (the blocked kernel changed last).  Phase 2 runs the
# bench lines against the committed profiles/r03_pmc_traffic*.json.
set -e
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f_c4 -o f -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_f_c4.log 2>&1 || { tail -20 $O/pmc_f_c4.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w_c4 -o w -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_w_c4.log 2>&1 || { tail -20 $O/pmc_w_c4.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_f_c4 $O/pmc_w_c4 C4 1024 5 $O/pmc_traffic_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/prof_c4.log 2>&1 || { tail -30 $O/prof_c4.log; exit 1; }
grep socp_large $O/prof_c4/c4_kernel_stats.csv | cut -c1-150
