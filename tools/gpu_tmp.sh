set -e
export TMPDIR=/tmp
O=gpurun_out/bidir
mkdir -p $O
L="socp.jl_amd/lib/v_cur/libsocp.so socp.jl_amd/lib/v_bidir/libsocp.so socp.jl_amd/lib/v_postra/libsocp.so"
timeout -k 10 500 python3 tools/ab_multi.py C2 9 $L $L $L > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep "^C2" $O/ab.log
AB_BATCH=65536 AB_K=8 timeout -k 10 300 python3 tools/ab_multi.py C1 5 $L $L > $O/ab_c1.log 2>&1 || { tail -30 $O/ab_c1.log; exit 1; }
grep "^C1" $O/ab_c1.log
