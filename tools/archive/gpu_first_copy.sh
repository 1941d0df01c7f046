set -o pipefail
mkdir -p gpurun_out
for args in "2880000" "2880000 --no-scratch" "25920000" "2147483648"; do
timeout -k 10 60 python -u tools/first_copy.py $args >> gpurun_out/first_copy.jsonl 2>> gpurun_out/first_copy.err || { tail gpurun_out/first_copy.err; exit 1; }
done
cat gpurun_out/first_copy.jsonl
