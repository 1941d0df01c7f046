# Round 2, call AI: is it the rows' 128-B alignment? The exact and tree forms on even widths
# whose rows are 16-B aligned but start at varying offsets within a 128-B line.
set -o pipefail
mkdir -p gpurun_out/r02ai
O=gpurun_out/r02ai
timeout -k 10 600 python -u tools/sweep_exact.py 3 cfg2_16384sq,even_16384x16386,even_16384x16388,even_16384x16400,odd_16384x16383 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
