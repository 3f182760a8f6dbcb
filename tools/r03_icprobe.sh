# Is the generated kernels' lower VALU rate the instruction fetch?  Shared
# two-wave programs (C5 AUTO encode, C3 generated encode) normal vs every
# chunk running chunk 0's code (timing only, wrong parity; the hook was
# removed after): bash tools/r03_icprobe.sh TAG
# (the probe hook -- rsgpu_internal_set_icache_probe, bench.py --icache-probe, chunk_stride 0 allowed in launch_rs_jitw -- was removed after this measurement)
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for rep in 1 2; do
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5_norm_$rep.log 2>&1 || exit 1
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline --icache-probe 1 > $O/c5_probe_$rep.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c3_norm_$rep.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated --icache-probe 1 > $O/c3_probe_$rep.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items() if 'prepare' not in k and 'emit' not in k})"; done
