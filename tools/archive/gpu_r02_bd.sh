# Round 2, call BD: the column-panel exact dispatch — full GPU suite, the probe on the product
# entry points (relayout timed first in each round), and the driver's bench under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02bd
O=$R/gpurun_out/r02bd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; }
S=cfg2_16384sq,mid_8192x16384,ref_10200sq,ref_7800sq,mid_6144x4096,cfg3_g8_strip_65536x8192,cfg4_block_65536x32768,tall_262144x4096,odd_16384x16383
timeout -k 10 600 python -u tools/panel_probe.py 7 $S 256 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 $R/bench.py > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_trace.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], d['exact']['kernel'], d['exact']['roofline_frac'], [(c['config'], c['value'], c['exact']['value'], c['exact']['kernel']) for c in d['configs']])"
echo all-done
