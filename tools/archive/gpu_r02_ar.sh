# Round 2, call AR: the reference's test.sh sizes through the executables in bit-exact mode on
# the final build (chain-hopping exact kernels), then the comparison table.
set -o pipefail
mkdir -p gpurun_out/r02ar
O=gpurun_out/r02ar
rm -rf $O/ref_sweep_exact
MVG_EXACT=1 timeout -k 10 900 python tools/ref_sweep.py --out $O/ref_sweep_exact > $O/ref_sweep.log 2>&1 || { tail $O/ref_sweep.log; exit 1; }
tail -2 $O/ref_sweep.log
echo all-done
