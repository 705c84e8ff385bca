"""rocprofv3 --pmc CSVs (separate FETCH_SIZE / WRITE_SIZE / SQ_* passes of `bench.py --sync --steps 1`)
-> profiles/traffic.json (per-kernel HBM-side bytes per launch, read by bench.py) and a per-kernel counter
summary CSV.  Tooling only.

    python tools/traffic.py gpurun_out/prof profiles/r1_pmc_summary.csv

FETCH_SIZE and WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE counts half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section), so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(prof):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(prof, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not name.startswith("k_"):
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main(prof, out_csv):
    m = load(prof)
    kernels = {}
    for k, c in sorted(m.items()):
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            kernels[k] = {"fetch_kb": c["FETCH_SIZE"], "write_kb": c["WRITE_SIZE"],
                          "bytes_per_launch": 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate runs of bench.py --sync --steps 1 "
                         "--warmup 1 (tools/gpu/profile.sh); bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950)",
               "kernels": kernels}, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    cols = sorted({c for cs in m.values() for c in cs})
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel"] + cols)
        for k, cs in sorted(m.items()):
            w.writerow([k] + ["%.6g" % cs[c] if c in cs else "" for c in cols])
    print(open(out_csv).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
