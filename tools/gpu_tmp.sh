set -e
export TMPDIR=/tmp
O=gpurun_out/tmp
mkdir -p $O
for v in new old new old; do
  if [ $v = old ]; then L=socp.jl_amd/lib/v_sqr0/libsocp.so; else L=socp.jl_amd/lib/libsocp.so; fi
  SOCP_AMD_LIB=$L timeout -k 10 300 python3 bench.py --mode sqr --steps 10 --warmup 2 --no-cpu > $O/sqr_$v.log 2>&1 || { tail -30 $O/sqr_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/sqr_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], json.dumps(d.get("solve_socp", d.get("rank_update_plugin", {})))[:300])')"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sqr.py -m gpu -q --timeout 300 --timeout-method thread > $O/pt_sqr.log 2>&1 || { grep -E "FAILED|ERROR" $O/pt_sqr.log | head; tail -5 $O/pt_sqr.log; exit 1; }
tail -2 $O/pt_sqr.log
