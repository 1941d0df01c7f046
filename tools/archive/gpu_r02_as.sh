# Round 2, call AS: PMC passes (separate runs) over the final exact kernel at 16384^2 and at
# 16384 x 16386 (rows off the 128-B lines): HBM bytes, and L1->L2 read requests / L2 hits.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02as
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "16384 16384" "16384 16386"; do
  tag=$(echo $shape | tr ' ' x)
  for pass in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    ptag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/${tag}_$ptag -o run -- python3 $R/tools/exact_probe.py $shape 8 > $O/${tag}_$ptag.log 2>&1 || { tail -5 $O/${tag}_$ptag.log; exit 1; }
  done
done
echo all-done
