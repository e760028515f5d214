set -e
export TMPDIR=/tmp
O=gpurun_out/lrep5
mkdir -p $O
V="0 1 2 4 8 16 32 64"
L=""; for v in $V; do L="$L socp.jl_amd/lib/v_lrep$v/libsocp.so"; done
timeout -k 10 400 python3 tools/ab_multi.py C4 3 $L > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep "^C4" $O/ab.log
for v in $V; do
  export SOCP_AMD_LIB=socp.jl_amd/lib/v_lrep$v/libsocp.so
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o f -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/f_$v.log 2>&1 || { tail -20 $O/f_$v.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o w -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/w_$v.log 2>&1 || { tail -20 $O/w_$v.log; exit 1; }
  python3 tools/pmc_traffic.py $O/f_$v $O/w_$v C4 1024 5 $O/traffic_$v.json > /dev/null
  echo "$v $(python3 -c "import json; d=json.load(open('$O/traffic_$v.json')); print(d['hbm_read_bytes']/1e9, d['hbm_write_bytes']/1e9)")"
done
