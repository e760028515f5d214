#!/bin/bash
# Tuning builds (never the product): the C1/C2 register-kernel instantiations
# (gen_inst.py SOCP_DEV_VARIANTS) compiled with extra flags, linked with the
# product build's other objects into socp.jl_amd/lib/v_<name>/libsocp.so.
#   tools/build_variant.sh <name> "<extra hipcc flags>"
set -e
name=$1; extra=$2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/socp.jl_amd/csrc
GEN=$R/socp.jl_amd/build/gen_v_$name
OBJ=$R/socp.jl_amd/build/obj_v_$name
LIB=$R/socp.jl_amd/lib/v_$name
mkdir -p $GEN $OBJ $LIB
SOCP_DEV_VARIANTS=${DEV_VARIANTS:-1} python3 $C/gen_inst.py $GEN > /dev/null
FLAGS="-I$C -O3 -std=c++17 -ffp-contract=fast-honor-pragmas -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-use-amdgpu-trackers=1 -mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1 --offload-arch=gfx950 -fPIC -Wno-unused-function -Wno-unused-variable $extra"
pids=()
for f in $GEN/inst_*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc $FLAGS -c $f -o $OBJ/$b.o > $OBJ/$b.log 2>&1 &
  pids+=($!)
done
# the C ABI too (host-side layout helpers such as small_lds_bytes see the flags)
/opt/rocm/bin/hipcc $FLAGS -c $C/socp_api.hip -o $OBJ/socp_api.o > $OBJ/socp_api.log 2>&1 &
pids+=($!)
for p in "${pids[@]}"; do wait $p || { echo "compile failed"; cat $OBJ/*.log | tail -20; exit 1; }; done
M=$R/socp.jl_amd/build/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $LIB/libsocp.so $OBJ/socp_api.o $M/socp_large.o $M/socp_large_gv.o $M/socp_sqr.o $M/socp_sqr_ipm.o $OBJ/inst_*.o
echo "built $LIB/libsocp.so"
