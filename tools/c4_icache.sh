# C4-shaped (L 32000, 4096 blocks = one decode slice) instruction-cache price:
# the diagnostic build, variant 8 (chunk-0 code for every full chunk), variant 7
# (block 0 code for every block) and the product, each in its own process
# (tools/bound_probe.py).  Build: make -C storage-benchmarks_amd diag DIAG_VARIANT={,7,8}
#   bash tools/c4_icache.sh   -> gpurun_out/c4ic/
set -o pipefail
O=gpurun_out/c4ic; mkdir -p $O
D=tools/diag
run() { echo "== $1"; RSGPU_LIB=$2 timeout -k 10 120 python3 -u tools/bound_probe.py --symbol-size 32000 --blocks 4096 --seconds 1.5 --order enc:rand,dec:rand,enc:rand,dec:rand --out $O/$1.json > $O/$1.log 2>&1 && python3 -c "
import json; d=json.load(open('$O/$1.json'))
print('$1', [(p['phase'], p['median_ms'], p.get('clock_MHz_median')) for p in d['phases']])"; }
run p $D/librsgpu_diag.so && run v8 $D/librsgpu_diag_v8.so && run v7 $D/librsgpu_diag_v7.so && run product storage-benchmarks_amd/rsgpu/librsgpu.so && run p2 $D/librsgpu_diag.so
