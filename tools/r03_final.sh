# Round-3 closing evidence at HEAD: GPU suite, smoke(), C2 / C3 / C4 / C5
# lines, the geometry sweep: bash tools/r03_final.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
$T python3 bench.py --config c2 --steps 300 --no-cpu-baseline > $O/c2.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
$T python3 bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 || exit 1
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5.log 2>&1 || exit 1
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
bash tools/geom_sweep.sh $1 || true
