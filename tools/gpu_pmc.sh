set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { tail -30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write C2 65536 8 gpurun_out/pmc_traffic.json
