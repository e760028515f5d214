#!/bin/bash
# C1 round profile: PMC traffic (two passes), rocprofv3 kernel stats, bench line with the CPU leg.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1_fetch -o f -- python bench.py --config C1 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc1_fetch.log 2>&1 || { tail -30 gpurun_out/pmc1_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc1_write -o w -- python bench.py --config C1 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc1_write.log 2>&1 || { tail -30 gpurun_out/pmc1_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc1_fetch gpurun_out/pmc1_write C1 4096 3 gpurun_out/pmc_traffic_c1.json
cp gpurun_out/pmc_traffic_c1.json profiles/r01_pmc_traffic_c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o c1 -- python bench.py --config C1 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c1.log 2>&1 || { tail -20 gpurun_out/prof_c1.log; exit 1; }
timeout -k 10 300 python bench.py --config C1 > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
