# Round 2, call L: chunked distribution overlap — parity test, then end-to-end times over chunk
# counts at config 2 and at two of the reference's test.sh sizes.
set -o pipefail
mkdir -p gpurun_out/r02l
O=gpurun_out/r02l
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k overlapped > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head; exit $rc; }
for shape in "16384 16384 5" "10200 10200 10" "4200 4200 20"; do
  timeout -k 10 300 python -u tools/overlap_probe.py $shape >> $O/overlap.jsonl 2>> $O/overlap.err || { tail $O/overlap.err; exit 1; }
done
cat $O/overlap.jsonl
