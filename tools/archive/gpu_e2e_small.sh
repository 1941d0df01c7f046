# Small-size end-to-end phase breakdown (tools/e2e_small.py) with and without pinned x/y and
# spin-wait, plus the NUMA placement of H2D sources (tools/numa_h2d.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/e2e_small.py > gpurun_out/e2e_small.jsonl 2> gpurun_out/e2e_small.err || { tail gpurun_out/e2e_small.err; exit 1; }
timeout -k 10 120 python -u tools/e2e_small.py --pin-xy >> gpurun_out/e2e_small.jsonl 2>> gpurun_out/e2e_small.err || { tail gpurun_out/e2e_small.err; exit 1; }
timeout -k 10 120 python -u tools/e2e_small.py --pin-xy --spin >> gpurun_out/e2e_small.jsonl 2>> gpurun_out/e2e_small.err || { tail gpurun_out/e2e_small.err; exit 1; }
timeout -k 10 120 python -u tools/e2e_small.py --alg colwise --pin-xy >> gpurun_out/e2e_small.jsonl 2>> gpurun_out/e2e_small.err || { tail gpurun_out/e2e_small.err; exit 1; }
cat gpurun_out/e2e_small.jsonl
timeout -k 10 180 python -u tools/numa_h2d.py > gpurun_out/numa_h2d.jsonl 2> gpurun_out/numa_h2d.err || { tail gpurun_out/numa_h2d.err; exit 1; }
cat gpurun_out/numa_h2d.jsonl
