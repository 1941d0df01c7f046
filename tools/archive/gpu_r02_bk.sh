# Round 2, call BK: deeper chain-hopping pipelines for few rows (hop8_l16_w4_u16, l16_w8_u8,
# l32_w8_u8, l32_w4_u16: 256 VGPRs, one wave per SIMD, twice the bytes in flight) against every
# exact variant on the few-row shapes.
set -o pipefail
mkdir -p gpurun_out/r02bk
O=gpurun_out/r02bk
S=ref_4200sq,ref_1800sq,ref_600sq,mid_4096x16384,mid_4096x32768,mid_2048x65536,asym_1200x60000,asym_120x60000,mid_8192x16384,odd_4096x16383,odd_1200x60001,mid_8192x8192
timeout -k 10 600 python -u tools/sweep_exact.py 7 $S > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
