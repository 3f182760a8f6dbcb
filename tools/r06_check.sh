# Round 6 check of a build: the GPU suite, smoke, the driver's default bench
# line and C4.  (Round 6's first run also took the diagnostic build's phase
# stamps at C4 after the hooks refactor: profiles/r06_check1/.)
#   gpurun -- bash tools/r06_check.sh NAME  -> gpurun_out/NAME/
set -o pipefail
O=gpurun_out/${1:-r06_check}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 &&
tail -1 $O/pytest_gpu.log && tail -c 600 $O/bench_default.log && python3 -c "
import json
for f in ('bench_default', 'c4'):
    d = json.loads([l for l in open('$O/%s.log' % f) if l.startswith('{')][-1])
    print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_ms'], d['verified'])
"
