# Round 2, call BF: PMC passes (separate runs) over the panel-layout exact kernel
# (gemv_seq_hop_panel, via tools/exact_probe.py ... panels) at config 2 and config 3's G = 8
# strip: HBM bytes, and L1->L2 read requests / L2 hits; summaries by tools/pmc_traffic.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02bf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "16384 16384" "65536 8192"; do
  tag=$(echo $shape | tr ' ' x)
  dirs=""
  for pass in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    ptag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/${tag}_$ptag -o run -- python3 $R/tools/exact_probe.py $shape 8 panels > $O/${tag}_$ptag.log 2>&1 || { tail -5 $O/${tag}_$ptag.log; exit 1; }
    dirs="$dirs $O/${tag}_$ptag"
  done
  set -- $shape
  python3 $R/tools/pmc_traffic.py --out $O/pmc_exact_gemv_seq_hop_panel_${tag}.json --alg rowwise-probe-gemv_seq_hop_panel --R $1 --C $2 --kernel gemv_seq_hop_panel $dirs > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/pmc_exact_gemv_seq_hop_panel_${tag}.json')); print('$tag', d['traffic_over_algorithmic'], d['median_counters'])"
done
echo all-done
