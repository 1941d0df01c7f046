# Round 2, call S: PMC passes over the dispatch's exact kernel (gemv_seq_x) at 16384^2 and
# 65536 x 32768: HBM bytes and LDS bank conflicts.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "16384 16384" "65536 32768"; do
  tag=$(echo $shape | tr ' ' x)
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
    ptag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $O/${tag}_$ptag -o run -- python3 $R/tools/exact_probe.py $shape 8 > $O/${tag}_$ptag.log 2>&1 || { tail -5 $O/${tag}_$ptag.log; exit 1; }
  done
done
echo all-done
