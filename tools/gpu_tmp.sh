set -e
export TMPDIR=/tmp
O=gpurun_out/sqfin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sqr.py tests/test_gpu_dense.py -m gpu -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "FAILED|ERROR" $O/pt.log | head; tail -5 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sqr -o sqr -- python3 bench.py --mode sqr --steps 3 --warmup 1 --no-cpu > $O/prof_sqr.log 2>&1 || { tail -30 $O/prof_sqr.log; exit 1; }
timeout -k 10 400 python3 bench.py --mode sqr --steps 10 --warmup 2 > $O/bench_sqr.log 2>&1 || { tail -30 $O/bench_sqr.log; exit 1; }
grep '^{' $O/bench_sqr.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["kernels"], d["solve_socp"]["value"], d["solve_socp"]["ms_per_solve"])'
