set -e
export TMPDIR=/tmp
O=gpurun_out/tmp
mkdir -p $O
AB_SHAPE=64,16,32 timeout -k 10 300 python3 tools/ab_multi.py C2 7 socp.jl_amd/lib/v_w1/libsocp.so socp.jl_amd/lib/v_w2/libsocp.so > $O/ab_w.log 2>&1 || { tail -30 $O/ab_w.log; exit 1; }
tail -3 $O/ab_w.log
