#!/bin/bash
# The reference's benchmark sweep (its test.sh) with the drop-in executables:
#   tools/test.sh <rowwise|colwise|blockwise> [P ...]
# Runs `mpiexec -n P bin/multiplier_<alg> n n` for the reference's nine square sizes, from the
# current directory (which must hold ./data/matrix_n_n.txt, ./data/vector_n.txt and
# ./data/out/, as for the reference — `python -m matvec_mpi_multiplier_amd.gendata --test-sh` writes
# them; MVG_SYNTH=1 generates the inputs in memory instead). Rows go to
# ./data/out/<alg>.csv in the reference's format. P defaults to 1 2 4 8 (one MI355X per rank;
# the reference's 1 2 6 12 24 counted CPU processes). Set MPIEXEC to use another launcher.
set -e
ALG=${1:?usage: tools/test.sh <rowwise|colwise|blockwise> [P ...]}
shift
PROCS=${*:-1 2 4 8}
HERE=$(cd "$(dirname "$0")/.." && pwd)
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
make -s -C "$HERE" -j8 >/dev/null
for p in $PROCS; do
    echo "$p"
    for n in 600 1800 3000 4200 5400 6600 7800 9000 10200; do
        "$MPIEXEC" -n "$p" "$HERE/bin/multiplier_$ALG" "$n" "$n"
    done
done
