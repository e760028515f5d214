#!/bin/bash
# Round measurement session: GPU tests, smoke, bench lines (C2 headline, C4),
# rocprofv3 kernel stats, PMC HBM traffic passes (one counter per pass),
# phase stamps.  Each GPU step has its own limit; the first failure ends it.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json.log 2>&1 || { tail -30 gpurun_out/bench_c2.json.log; exit 1; }
timeout -k 10 400 python bench.py --config C4 --steps 3 --warmup 1 --traffic-json profiles/r01_pmc_traffic_c4.json > gpurun_out/bench_c4.json.log 2>&1 || { tail -30 gpurun_out/bench_c4.json.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c2.log 2>&1 || { tail -30 gpurun_out/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c4.log 2>&1 || { tail -30 gpurun_out/prof_c4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write C2 65536 8 gpurun_out/pmc_traffic.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch4 -o f -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_fetch4.log 2>&1 || { tail -30 gpurun_out/pmc_fetch4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write4 -o w -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_write4.log 2>&1 || { tail -30 gpurun_out/pmc_write4.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch4 gpurun_out/pmc_write4 C4 1024 5 gpurun_out/pmc_traffic_c4.json
timeout -k 10 300 python tools/stamps.py C2,C1,C4 > gpurun_out/stamps.log 2>&1 || { tail -30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_c4.json
