set -e
export TMPDIR=/tmp
O=gpurun_out/benchfin
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
