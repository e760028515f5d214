set -e
export TMPDIR=/tmp
O=gpurun_out/cg
mkdir -p $O
L="socp.jl_amd/lib/libsocp.so socp.jl_amd/lib/v_lrep0cg2/libsocp.so socp.jl_amd/lib/v_lrep0cg8/libsocp.so"
timeout -k 10 400 python3 tools/ab_multi.py C4 3 $L $L > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep "^C4" $O/ab.log
