"""Scaling table from bench.py JSON lines at several N (development tool).

    python tools/scaling_report.py SCALE_r01.json [more files or lines ...]

Accepts files holding one bench.py JSON line each, a JSON list of them, or JSON-lines. Prints,
per N: config 2's weak-scaled `value` and its efficiency against N x value(N=1) (aggregate GB/s),
and for each entry of `configs` (BASELINE configs 3-5, strong-scaled: fixed total work) the
aggregate GB/s, the time per step, speed-up T1/TN and efficiency speed-up / N, plus the
end-to-end times.
"""
import json
import sys


def lines(paths):
    for p in paths:
        text = open(p).read().strip()
        try:
            d = json.loads(text)
            items = d if isinstance(d, list) else [d]
        except json.JSONDecodeError:
            items = [json.loads(l) for l in text.splitlines() if l.strip().startswith("{")]
        for it in items:
            if isinstance(it, dict) and "n_gpus" in it:
                yield it
            elif isinstance(it, dict):  # a driver wrapper {"1": {...}, "2": {...}} or similar
                for v in it.values():
                    if isinstance(v, dict) and "n_gpus" in v:
                        yield v


def main():
    runs = sorted(lines(sys.argv[1:]), key=lambda d: d["n_gpus"])
    if not runs:
        raise SystemExit("no bench lines found")
    base = runs[0]
    n0 = base["n_gpus"]
    print("| N | config 2 value (GB/s) | weak eff. | ms/step | e2e shared (s) | e2e root_send (s) |")
    print("|---|---|---|---|---|---|")
    for d in runs:
        eff = d["value"] / (base["value"] * d["n_gpus"] / n0)
        e2e = d.get("end_to_end") or {}
        sh = e2e.get("shared") if isinstance(e2e.get("shared"), dict) else {}
        rs = e2e.get("root_send") if isinstance(e2e.get("root_send"), dict) else {}
        print(f"| {d['n_gpus']} | {d['value']:.0f} | {eff:.3f} | {d['ms_per_step']:.4f} | "
              f"{sh.get('mean_s', float('nan')):.4f} | {rs.get('mean_s', float('nan')):.4f} |")
    names = [c["config"] for c in (base.get("configs") or []) if "value" in c]
    for name in names:
        t1 = next(c for c in base["configs"] if c["config"] == name)
        print(f"\n{name} ({t1['alg']} {t1['R']} x {t1['C']}, strong scaling)\n")
        print("| N | grid | shard | GB/s | ms/step | speed-up | eff. | kernel frac |")
        print("|---|---|---|---|---|---|---|---|")
        for d in runs:
            c = next((c for c in d.get("configs") or [] if c["config"] == name and "value" in c), None)
            if c is None:
                print(f"| {d['n_gpus']} | skipped | | | | | | |")
                continue
            sp = t1["ms_per_step"] / c["ms_per_step"]
            print(f"| {d['n_gpus']} | {c.get('grid') or ''} | {c['shard']} | {c['value']:.0f} | {c['ms_per_step']:.4f} | "
                  f"{sp:.2f} | {sp / (d['n_gpus'] / n0):.3f} | {c.get('kernel_frac')} |")


if __name__ == "__main__":
    main()
