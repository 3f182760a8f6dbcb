set -o pipefail
mkdir -p gpurun_out/prof2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/bench_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD -d gpurun_out/prof2/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --blocks 256 --no-cpu-baseline --no-verify > gpurun_out/prof2/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof2/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --blocks 256 --no-cpu-baseline --no-verify > gpurun_out/prof2/pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof2/pmc3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --blocks 256 --no-cpu-baseline --no-verify > gpurun_out/prof2/pmc3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/prof2/pmc4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --blocks 256 --no-cpu-baseline --no-verify > gpurun_out/prof2/pmc4.log 2>&1
