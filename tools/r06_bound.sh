# What bounds the C3 kernels (tools/bound_probe.py): zero vs random inputs
# with the product library, the in-kernel clock with the diagnostic build,
# one SQ counter pass.  Run on the GPU box from the repo root:
#   bash tools/r06_bound.sh TAG  -> gpurun_out/bound_TAG/ (round 6: the diagnostic
# library from tools/diag_r06/, which the push carries)
set -o pipefail
TAG=${1:-r06}
O=$(pwd)/gpurun_out/bound_$TAG
mkdir -p $O
export TMPDIR=/tmp
SEC=${SEC:-2.5}
N=${N:-100}
timeout -k 10 240 python3 -u tools/bound_probe.py --seconds $SEC --out $O/time_product.json > $O/time_product.log 2>&1 && \
RSGPU_LIB=$(pwd)/tools/diag_r06/librsgpu_diag.so timeout -k 10 240 python3 -u tools/bound_probe.py --seconds $SEC --out $O/clock_diag.json > $O/clock_diag.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc1 -o run --output-format csv -- python3 tools/bound_probe.py --launches $N --out $O/pmc1/probe.json > $O/pmc1.log 2>&1 && \
python3 tools/bound_summary.py $O/summary.json $O/pmc1 > $O/summary.log 2>&1
