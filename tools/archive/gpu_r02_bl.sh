# Round 2, call BL: 16-B panel relayout — the exact GPU tests, then the probe's relayout timing
# on config 2 and config 4's block.
set -o pipefail
mkdir -p gpurun_out/r02bl
O=gpurun_out/r02bl
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -2 $O/pytest_exact.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_exact.log | head -20; exit $rc; }
timeout -k 10 600 python -u tools/panel_probe.py 5 cfg2_16384sq,cfg4_block_65536x32768,odd_16384x16383 256 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
grep relayout $O/probe.jsonl
echo all-done
