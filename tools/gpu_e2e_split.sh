# Small-size end-to-end with the distribution's H2D on one stream, x on the copy stream, or A
# split over both streams (MVG_H2D_SPLIT = 0 / 1 / 2).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/e2e_split.jsonl
for sp in 0 1 2 0 1 2; do
MVG_H2D_SPLIT=$sp timeout -k 10 120 python -u tools/e2e_small.py --pin-xy >> gpurun_out/e2e_split.jsonl 2>> gpurun_out/e2e_split.err || { tail gpurun_out/e2e_split.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/e2e_split.jsonl'):
    d=json.loads(l); print(d['h2d_split'], d['n'], 'whole', d['whole_us_median'], 'dist', d['distribute_us_median'])
PY
