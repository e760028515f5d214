set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/w
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k "wide_n or beyond" -v --timeout 300 --timeout-method thread > gpurun_out/w/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/w/pytest.log | head -30; tail -15 gpurun_out/w/pytest.log; exit 1; }
tail -8 gpurun_out/w/pytest.log
bash tools/gpu_ab2.sh socp.jl_amd/lib/v_base/libsocp.so socp.jl_amd/lib/v_cur/libsocp.so socp.jl_amd/lib/v_ubt/libsocp.so
