# Round 2, call BA: the exact variants beside a plain streaming read of the same bytes
# (mvg_stream_read, 4096 contiguous streams, no chain) on config shapes, same box, 7 rounds.
set -o pipefail
mkdir -p gpurun_out/r02ba
O=gpurun_out/r02ba
S=cfg2_16384sq,even_16384x16400,mid_8192x16384,ref_10200sq,cfg3_g8_strip_65536x8192,cfg5_shard_524288x512,cfg4_block_65536x32768
timeout -k 10 600 python -u tools/sweep_exact.py 7 $S > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
