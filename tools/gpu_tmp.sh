set -e
export TMPDIR=/tmp
O=gpurun_out/tmp
mkdir -p $O
V="cur cl0 postra memcl bidir ilp"
L=""; for v in $V; do L="$L socp.jl_amd/lib/v_$v/libsocp.so"; done
timeout -k 10 400 python3 tools/ab_multi.py C2 9 $L $L > $O/ab_flags.log 2>&1 || { tail -30 $O/ab_flags.log; exit 1; }
grep "^C2" $O/ab_flags.log
timeout -k 10 300 python3 tools/ab_multi.py C1 15 $L > $O/ab_flags_c1.log 2>&1 || { tail -30 $O/ab_flags_c1.log; exit 1; }
grep "^C1" $O/ab_flags_c1.log
timeout -k 10 300 python3 bench.py --config C1 --no-ingest --no-cpu > $O/b_c1.log 2>&1 || { tail -30 $O/b_c1.log; exit 1; }
grep '^{' $O/b_c1.log | cut -c1-330
timeout -k 10 300 python3 bench.py --no-ingest --no-cpu > $O/b_c2.log 2>&1 || { tail -30 $O/b_c2.log; exit 1; }
grep '^{' $O/b_c2.log | cut -c1-330
