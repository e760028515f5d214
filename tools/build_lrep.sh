#!/bin/bash
# Tuning builds (never the product): the blocked kernel (socp_large.hip) with
# SOCP_LREP=<bits> (phases run twice), linked with the product
# build's other objects into socp.jl_amd/lib/v_lrep<bits>/libsocp.so.
#   tools/build_lrep.sh <bits> ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/socp.jl_amd/csrc
M=$R/socp.jl_amd/build/obj
FLAGS="-I$C -O3 -std=c++17 -ffp-contract=fast-honor-pragmas -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-use-amdgpu-trackers=1 -mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1 --offload-arch=gfx950 -fPIC -Wno-unused-function -Wno-unused-variable"
pids=()
for b in "$@"; do
  O=$R/socp.jl_amd/build/obj_v_lrep$b$TAG; mkdir -p $O $R/socp.jl_amd/lib/v_lrep$b$TAG
  ( /opt/rocm/bin/hipcc $FLAGS $EXTRA -DSOCP_LREP=$b -c $C/socp_large.hip -o $O/socp_large.o > $O/build.log 2>&1 &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/socp.jl_amd/lib/v_lrep$b$TAG/libsocp.so \
      $(ls $M/*.o | grep -v "socp_large.o\|asan") $O/socp_large.o >> $O/build.log 2>&1 ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build failed"; exit 1; }; done
echo "built: $*"
