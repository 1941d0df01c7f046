# Round 2, call AZ: re-entry check on the restored final build (XCD dispatch) — the full GPU suite, smoke(), and
# the driver's bench command under a rocprofv3 kernel trace (per-kernel stats for profiles/).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02az
O=$R/gpurun_out/r02az
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 $R/bench.py > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_trace.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], d['exact']['kernel'])"
echo all-done
