# C4 batch-size / decode-kernel sweep: bash tools/r03_c4sweep.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for b in 16384 4096 1024; do
  for d in auto generated; do
    $T python3 bench.py --config c4 --batch $b --decode-kernel $d --warmup 1 --no-cpu-baseline > $O/c4_b${b}_$d.log 2>&1 || exit 1
  done
done
for f in $O/c4_*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:(v['avg_ms'],v['launches']) for k,v in d['kernels'].items()})"; done
export TMPDIR=/tmp
B="python3 bench.py --config c4 --blocks 32768 --warmup 1 --no-cpu-baseline --no-verify"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/c4_fetch -o run --output-format csv -- $B > $O/c4_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/c4_write -o run --output-format csv -- $B > $O/c4_write.log 2>&1 && \
python3 tools/pmc_traffic.py $O/c4_fetch/run_counter_collection.csv $O/c4_write/run_counter_collection.csv $O/c4_traffic.json > $O/c4_traffic.log 2>&1
cat $O/c4_traffic.json
