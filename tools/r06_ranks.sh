# Round 6: the N-rank path on one GPU (every rank on device 0, the default
# gloo backend): 4 and 8 self-spawned ranks and 4 ranks under
# torch.distributed.run, C3 geometry with few blocks per rank, and C4.
#   gpurun -- bash tools/r06_ranks.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_ranks}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 4 --same-device --blocks 64 --steps 2 --warmup 1 --no-cpu-baseline > $O/spawn4.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 8 --same-device --blocks 16 --steps 2 --warmup 1 --no-cpu-baseline > $O/spawn8.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --same-device --blocks 64 --steps 2 --warmup 1 --no-cpu-baseline > $O/torchrun4.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 4 --same-device --config c4 --blocks 8192 --batch 2048 --no-cpu-baseline > $O/spawn4_c4.log 2>&1
for f in spawn4 spawn8 torchrun4 spawn4_c4; do grep -h '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['n_gpus'], d['value'], d['verified'], d['config'].get('dist_backend'), [(r['rank'], r.get('block0'), r.get('blocks')) for r in d.get('ranks', [])])"; done
