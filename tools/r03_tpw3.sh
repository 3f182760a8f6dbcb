# Why are 6-wave workgroups (three column tiles) of the two-wave decode slow?
# One SQ counter pass each, C4 geometry resident, tiles per workgroup 2 vs 3:
# bash tools/r03_tpw3.sh TAG
set -o pipefail
O=$(pwd)/gpurun_out/r03_$1; mkdir -p $O
export TMPDIR=/tmp
for t in 2 3; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/t$t -o run --output-format csv -- python3 bench.py --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-verify --jitw-tiles $t > $O/t$t.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/t$t > $O/t${t}_summary.txt 2>&1 || exit 1
done
grep -A9 "jit16" $O/t2_summary.txt $O/t3_summary.txt
