"""rocprofv3 --pmc CSVs -> profiles/traffic.json (per-kernel HBM-side bytes per launch, read by bench.py's
roofline objects) and a per-kernel counter summary CSV.  Tooling only.

    python tools/traffic.py gpurun_out/r2prof profiles/r2_pmc_summary.csv

The profile directory holds one rocprofv3 output directory per counter pass, named pmc_<config>_<counter>
(tools/gpu/profile_r2.sh, profile_r3.sh): config "head" = bench.py --sync --steps 1 (the headline batches), "c3" = the
Recover run at BASELINE configs[2], "c5" = the adversarial Recover run at configs[4].  Values are averaged
over every dispatch of a kernel in the run, the same launch mix as bench.py's per-launch kernel averages.

FETCH_SIZE and WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE counts half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section), so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLAUSIBLE_BYTES_S = 10e12  # above MI355X HBM (8 TB/s) plus on-die cache hits counted at the memory side


acc_raw = {}


def load(prof, raw=False):
    """{config: {kernel: {counter: mean value per dispatch}}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for f in glob.glob(os.path.join(prof, "pmc_*", "*counter_collection.csv")):
        m = re.match(r"pmc_([a-z0-9]+)_", os.path.basename(os.path.dirname(f)))
        cfg = m.group(1) if m else "head"
        per = collections.defaultdict(float)
        names, dur = {}, {}
        for r in csv.DictReader(open(f)):
            if not r["Kernel_Name"].startswith("k_"):
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        for (d, c), v in per.items():
            acc[cfg][names[d]][c].append(v)
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                acc[cfg][names[d]]["_dur_" + c].append(dur[d])
    out = {cfg: {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in ks.items()} for cfg, ks in acc.items()}
    for cfg, ks in acc.items():  # dispatch counts, for the per-call sums of a multi-kernel pipeline
        for k, cs in ks.items():
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in cs:
                    out[cfg][k]["_n_" + c] = len(cs[c])
    return (out, acc) if raw else out


def main(prof, out_csv, out_json=None):
    global acc_raw
    m, acc_raw = load(prof, raw=True)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate runs per counter (tools/gpu/profile_r2.sh, profile_r3.sh); "
                     "bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950); head = bench.py --sync --steps 1, c3 = Recover "
                     "configs[2], c5 = adversarial Recover configs[4]", "configs": {}}
    # configs of earlier runs that this one did not profile are kept (one call per config group fits the box limits)
    dst = out_json or os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(dst):
        try:
            out["configs"].update(json.load(open(dst)).get("configs", {}))
        except ValueError:
            pass
    for cfg, ks in sorted(m.items()):
        sec = {}
        for k, c in sorted(ks.items()):
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                b = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
                t = max(1e-9, min(c["_dur_FETCH_SIZE"], c["_dur_WRITE_SIZE"]))
                sec[k] = {"fetch_kb": c["FETCH_SIZE"], "write_kb": c["WRITE_SIZE"], "bytes_per_launch": b,
                          "implied_tb_s": b / t / 1e12}
                if b / t > PLAUSIBLE_BYTES_S:  # beyond the memory system: the counter, not traffic
                    sec[k]["bytes_per_launch"] = None
                    sec[k]["note"] = ("FETCH/WRITE_SIZE imply %.0f TB/s over the launch, beyond the memory "
                                      "system: counter not usable for this (long, scratch-heavy) kernel" % (b / t / 1e12))
        # Recover's pairing-check pipeline (checks.h k_ck_*) as one unit, as bench.py prices it: the bytes of every
        # k_ck_* dispatch of the run over the number of per-item passes (one k_ck_round_lines per dg_recover call)
        # (the real calls only: dg_init's prewarm dispatches of k_ck_round_lines read nothing)
        calls = sum(1 for v in acc_raw.get(cfg, {}).get("k_ck_round_lines", {}).get("FETCH_SIZE", []) if v > 1024)
        if calls:
            tot = 0.0
            for k, c in ks.items():
                if k.startswith("k_ck_") and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    tot += (2 * c["FETCH_SIZE"] * c["_n_FETCH_SIZE"] + c["WRITE_SIZE"] * c["_n_WRITE_SIZE"]) * 1024
            sec["k_ck_* pipeline"] = {"bytes_per_launch": tot / calls, "calls": calls,
                                      "note": "sum over every k_ck_* dispatch / dg_recover calls of the run"}
        # the cross-round isolation of failed single-key batches (xr.h) as one unit, as bench.py's c2_negative line
        # prices it: the bytes of every k_xq_* / k_xg_* / k_ck_* dispatch of the run over the failed batches (the
        # k_xq_sum dispatches that read their candidates' points: FETCH_SIZE above 1 MB; a passed batch's is empty)
        xq = acc_raw.get(cfg, {}).get("k_xq_sum", {}).get("FETCH_SIZE", [])
        failed = sum(1 for v in xq if v > 1024)
        if failed:
            tot = 0.0
            for k, c in ks.items():
                if k.startswith(("k_xq_", "k_xg_", "k_ck_")) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    tot += (2 * c["FETCH_SIZE"] * c["_n_FETCH_SIZE"] + c["WRITE_SIZE"] * c["_n_WRITE_SIZE"]) * 1024
            sec["xr pipeline"] = {"bytes_per_launch": tot / failed, "calls": failed,
                                  "note": "sum over every k_xq_* / k_xg_* / k_ck_* dispatch / failed batches of the run"}
        out["configs"][cfg] = sec
    json.dump(out, open(dst, "w"), indent=1)
    cols = sorted({c for ks in m.values() for cs in ks.values() for c in cs if not c.startswith("_")})
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["config", "kernel"] + cols)
        for cfg, ks in sorted(m.items()):
            for k, cs in sorted(ks.items()):
                w.writerow([cfg, k] + ["%.6g" % cs[c] if c in cs else "" for c in cols])
    print(open(out_csv).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
