set -e
export TMPDIR=/tmp
O=gpurun_out/lrep4
mkdir -p $O
L="socp.jl_amd/lib/v_old/libsocp.so socp.jl_amd/lib/v_lrep0ns/libsocp.so socp.jl_amd/lib/libsocp.so socp.jl_amd/lib/v_lrep0su2/libsocp.so"
timeout -k 10 400 python3 tools/ab_multi.py C4 3 $L $L > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep "^C4" $O/ab.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -m gpu -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "FAILED|ERROR" $O/pt.log | head; tail -5 $O/pt.log; exit 1; }
tail -1 $O/pt.log
