# SQ/SQC counters of A/B tool binaries (run on the GPU box from the repo root):
#   bash tools/pmc_variants.sh TAG "name:cmd args" ...
# -> gpurun_out/pmcv_TAG/<name>/pass{1,2}/ ; summarise each with
#    python3 tools/pmc_summary.py gpurun_out/pmcv_TAG/<name>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  n=${v%%:*}; c=${v#*:}
  O=$(pwd)/gpurun_out/pmcv_$TAG/$n
  mkdir -p $O
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/pass1 -o run --output-format csv -- $c > $O/pass1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY -d $O/pass2 -o run --output-format csv -- $c > $O/pass2.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1 || exit 1
done
