# Does the per-source LDS wait of the two-wave code cost time?  C5 and C3
# (the probe hook was removed after this measurement: it lived in jit_prog.cpp build_matrix_code_wide as lds_probe, rsgpu_internal_set_lds_probe, bench.py --lds-probe)
# generated encodes normal vs the timing-only probe (next source's loads
# issued after the composites): bash tools/r03_ldsprobe.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for rep in 1 2; do
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5_norm_$rep.log 2>&1 || exit 1
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline --lds-probe 1 > $O/c5_probe_$rep.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c3_norm_$rep.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated --lds-probe 1 > $O/c3_probe_$rep.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items() if 'prepare' not in k and 'emit' not in k})"; done
