set -e
export TMPDIR=/tmp
O=gpurun_out/stamps5
mkdir -p $O
timeout -k 10 300 python3 tools/stamps.py C4 > $O/c4.log 2>&1 || { tail -30 $O/c4.log; exit 1; }
cat $O/c4.log | grep -v amdgpu.ids
