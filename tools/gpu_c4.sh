#!/bin/bash
# C4 round profile: blocked-kernel parity tests, PMC traffic (two passes),
# rocprofv3 kernel stats, bench line with the CPU leg.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/c4/c4_pytest.log 2>&1 || { tail -30 gpurun_out/c4/c4_pytest.log; exit 1; }
tail -1 gpurun_out/c4/c4_pytest.log
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c4/pmc4_fetch -o f -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu > gpurun_out/c4/pmc4_fetch.log 2>&1 || { tail -30 gpurun_out/c4/pmc4_fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c4/pmc4_write -o w -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu > gpurun_out/c4/pmc4_write.log 2>&1 || { tail -30 gpurun_out/c4/pmc4_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/c4/pmc4_fetch gpurun_out/c4/pmc4_write C4 1024 5 gpurun_out/c4/pmc_traffic_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4/prof_c4 -o c4 -- python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > gpurun_out/c4/prof_c4.log 2>&1 || { tail -20 gpurun_out/c4/prof_c4.log; exit 1; }
timeout -k 10 400 python bench.py --config C4 > gpurun_out/c4/bench_c4.log 2>&1 || { tail -20 gpurun_out/c4/bench_c4.log; exit 1; }
tail -1 gpurun_out/c4/bench_c4.log
