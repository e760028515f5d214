#!/bin/bash
# Tuning builds (never the product): the rank-update kernels (socp_sqr.hip)
# with extra flags, linked with the product build's other objects into
# socp.jl_amd/lib/v_<name>/libsocp.so.
#   tools/build_sqr_variant.sh <name> "<extra hipcc flags>"
set -e
name=$1; extra=$2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/socp.jl_amd/csrc
M=$R/socp.jl_amd/build/obj
O=$R/socp.jl_amd/build/obj_v_$name
mkdir -p $O $R/socp.jl_amd/lib/v_$name
/opt/rocm/bin/hipcc -I$C -O3 -std=c++17 -ffp-contract=fast-honor-pragmas -mllvm -amdgpu-mfma-vgpr-form=1 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $extra -c $C/socp_sqr.hip -o $O/socp_sqr.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/socp.jl_amd/lib/v_$name/libsocp.so $(ls $M/*.o | grep -v "socp_sqr.o\|asan") $O/socp_sqr.o
echo "built socp.jl_amd/lib/v_$name/libsocp.so"
