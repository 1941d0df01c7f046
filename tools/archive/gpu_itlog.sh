set -o pipefail
mkdir -p gpurun_out/itlog && cd gpurun_out/itlog && mkdir -p data/out
for n in 600 1800; do
MVG_SYNTH=1 MVG_ITERS=300 MVG_ITER_LOG=it_$n.txt timeout -k 10 60 ../../bin/multiplier_rowwise $n $n > out_$n.txt 2>&1 || { cat out_$n.txt; exit 1; }
done
python - <<'PY'
import numpy as np
for n in (600,1800):
    t=np.loadtxt(f'it_{n}.txt')*1e6
    print(n, 'first5', np.round(t[:5],1), 'mean100', round(t[:100].mean(),1), 'median', round(np.median(t),1), 'mean_all', round(t.mean(),1), 'p90', round(np.percentile(t,90),1))
PY
