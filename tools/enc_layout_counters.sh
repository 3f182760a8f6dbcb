# C3 encode layouts side by side, one SQ counter pass each (same box):
# the compiled 4 waves x 8 rows k_rs_bs vs the generated 2 waves x 16 rows
# shared program (k_rs_jitw, I-cache-streamed code).  Per launch: VALU and
# LDS instructions, cycles.  bash tools/enc_layout_counters.sh TAG
set -o pipefail
TAG=$1
O=$(pwd)/gpurun_out/enc_layout_$TAG; mkdir -p $O
export TMPDIR=/tmp
for ek in compiled generated; do
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/$ek/pass1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --encode-kernel $ek > $O/$ek.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/$ek > $O/$ek.summary 2>&1 || exit 1
done
for ek in compiled generated; do
  timeout -k 10 200 python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel $ek > $O/${ek}_time.log 2>&1 || exit 1
done
