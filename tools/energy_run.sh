# Which switching energy bounds the C3 kernels: the
# timing-only energy variants of the diagnostic build (diag_clock.h,
# DIAG_VARIANT 1..5) and the diagnostic product build, each in its own
# process, one after another on one box, through tools/bound_probe.py (the
# encode k_rs_bs and the decode k_rs_jit16 back to back for SEC seconds per
# phase, the in-kernel clock per phase).  Build first, on the CPU:
#   for v in "" 1 2 3 4 5; do make -C storage-benchmarks_amd diag DIAG_VARIANT=$v; done
# then on the GPU box, from the repo root:
#   bash tools/energy_run.sh TAG   -> gpurun_out/energy_TAG/
set -o pipefail
TAG=${1:-r05}
O=$(pwd)/gpurun_out/energy_$TAG
mkdir -p $O
export TMPDIR=/tmp
SEC=${SEC:-2.5}
ORDER=${ORDER:-enc:rand,dec:rand,enc:rand,dec:rand}
D=$(pwd)/tools/diag
run() {  # name lib order
    echo "== $1 $(date +%T)"
    RSGPU_LIB=$2 timeout -k 10 180 python3 -u tools/bound_probe.py --seconds $SEC --order $3 \
        --out $O/$1.json > $O/$1.log 2>&1
}
run p1 $D/librsgpu_diag.so enc:rand,dec:rand,enc:zero,dec:zero,enc:rand,dec:rand && \
run v1_hbmq $D/librsgpu_diag_v1.so $ORDER && \
run v2_zplane $D/librsgpu_diag_v2.so $ORDER && \
run v3_valuq $D/librsgpu_diag_v3.so $ORDER && \
run v4_nowait $D/librsgpu_diag_v4.so $ORDER && \
run v5_notr $D/librsgpu_diag_v5.so $ORDER && \
run p2 $D/librsgpu_diag.so $ORDER && \
run product $(pwd)/storage-benchmarks_amd/rsgpu/librsgpu.so $ORDER && \
python3 tools/energy_summary.py $O > $O/summary.md
