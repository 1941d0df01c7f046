# Round 2, call E: PMC passes over the bit-exact kernel (HBM bytes; LDS bank conflicts of the
# swizzled transposed reads; VALU/LDS activity), one counter group per run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "16384 16384" "65536 32768"; do
  tag=$(echo $shape | tr ' ' x)
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES"; do
    ptag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    echo "== $tag $pass"
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $O/${tag}_$ptag -o run -- python3 $R/tools/exact_probe.py $shape 8 > $O/${tag}_$ptag.log 2>&1 || { tail -5 $O/${tag}_$ptag.log; exit 1; }
  done
done
echo all-done
