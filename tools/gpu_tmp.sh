set -e
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -q -k "wide_n" --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { grep -E "FAILED|ERROR|Error" $O/pt.log | head; tail -15 $O/pt.log; exit 1; }
tail -2 $O/pt.log
L="socp.jl_amd/lib/libsocp.so socp.jl_amd/lib/v_lrep0gu2/libsocp.so socp.jl_amd/lib/v_lrep0sk1/libsocp.so"
timeout -k 10 400 python3 tools/ab_multi.py C4 3 $L $L > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep "^C4" $O/ab.log
