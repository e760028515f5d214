set -e
export TMPDIR=/tmp
bash tools/gpu_ab2.sh socp.jl_amd/lib/v_cur/libsocp.so socp.jl_amd/lib/v_ubt/libsocp.so socp.jl_amd/lib/v_u1/libsocp.so
timeout -k 10 200 python3 tools/ab_multi.py C1 15 socp.jl_amd/lib/v_cur/libsocp.so socp.jl_amd/lib/v_ubt/libsocp.so socp.jl_amd/lib/v_u1/libsocp.so 2>&1 | grep -v amdgpu.ids
