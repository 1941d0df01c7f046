# Round 2, call BC: the product's column-panel exact path — the exact GPU tests (panel kernels,
# relayout, engine), then tools/panel_probe.py on the product entry points over the config and
# edge shapes (P = 128 / 256 / 512), then the default bench's exact section.
set -o pipefail
mkdir -p gpurun_out/r02bc
O=gpurun_out/r02bc
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -2 $O/pytest_exact.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_exact.log | head -20; exit $rc; }
S=cfg2_16384sq,mid_8192x16384,cfg3_g8_strip_65536x8192,cfg3_g4_strip_65536x16384,cfg4_block_65536x32768,tall_131072x16384,odd_16384x16383,even_16384x16386,ref_10200sq,ref_7800sq,mid_6144x2048,mid_6144x4096,tall_262144x4096,tall_1048576x2048,cfg3_g1_65536sq
timeout -k 10 600 python -u tools/panel_probe.py 5 $S 128,256,512 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-configs --no-e2e > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact'])"
echo all-done
