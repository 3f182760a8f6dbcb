# SQ/SQC counter passes over a short bench run (run on the GPU box from the
# repo root):  bash tools/pmc_sq.sh TAG
# -> gpurun_out/sq_<TAG>/pass*/run_counter_collection.csv ; summarise with
#    python3 tools/pmc_summary.py gpurun_out/sq_<TAG>
set -o pipefail
TAG=${1:-x}
O=$(pwd)/gpurun_out/sq_$TAG
mkdir -p $O
export TMPDIR=/tmp
B=${SQ_BENCH:-"python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify"}  # SQ_BENCH: another run
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pass1 -o run --output-format csv -- $B > $O/pass1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES -d $O/pass2 -o run --output-format csv -- $B > $O/pass2.log 2>&1
