# Cache-policy sweep of the buffer-load row-block kernel against the production kernel (the record
# of how profiles/r01/variant_sweep19_cachepolicy.jsonl was made; the rowblkbuf_* experiment
# variants were dropped afterwards, so today it times only rowblk_w4_r2_u8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "all_variants" -x -q --timeout 120 --timeout-method thread > gpurun_out/cpol_test.log 2>&1 || { tail -30 gpurun_out/cpol_test.log; exit 1; }
tail -1 gpurun_out/cpol_test.log
timeout -k 10 600 python -u tools/sweep_variants.py 7 cfg2_16384sq,cfg3_g4_strip_65536x16384,cfg4_block_65536x32768,cfg3_g1_65536sq 'rowblkbuf,rowblk_w4_r2_u8$' > gpurun_out/cpol_sweep.jsonl 2> gpurun_out/cpol_sweep.err || { tail gpurun_out/cpol_sweep.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/cpol_sweep.jsonl'):
    d=json.loads(l); print(d['shape'], d['variant'], d['median_us'], d['GBps_median'], d['max_rel_vs_rocblas'])
"
