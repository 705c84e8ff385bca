"""Overlap analysis of a rocprofv3 kernel trace (tooling): per-queue busy time, concurrency, and an estimate of the
chip's wave-slot fill over the timed region, with the kernels that run while the chip is under-filled.

    python tools/trace/timeline.py gpurun_out/lat_trace/run_kernel_trace.csv [--first-kernel k_beacon_msgs --skip 1]

Wave slots: 256 CUs x 4 SIMDs x floor(512 / VGPRs(+AGPRs)) (the kernel's register budget bounds waves per SIMD);
a kernel's resident waves = min(its waves, that slot count) -- an upper bound (LDS and scratch ignored).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first-kernel", default="k_beacon_msgs")
    ap.add_argument("--skip", type=int, default=2, help="batches (first-kernel dispatches) to skip as warmup")
    ap.add_argument("--last-kernel", default="k_final_coop", help="the window ends with this kernel after the last "
                    "first-kernel dispatch")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        n = r["Kernel_Name"]
        if not n.startswith("k_"):
            continue
        vg = int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"] or 0)
        waves = (int(r["Grid_Size_X"]) + 63) // 64
        slots = 1024 * max(1, min(8, 512 // max(vg, 1)))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0], int(r["Queue_Id"]),
                     min(waves, slots) / slots if slots else 1.0, waves))
    rows.sort()
    starts = [x[0] for x in rows if x[2] == a.first_kernel]
    t0 = starts[a.skip] if len(starts) > a.skip else rows[0][0]
    last_start = starts[-1]
    t1 = min(x[1] for x in rows if x[0] >= last_start and x[2] == a.last_kernel) if a.last_kernel else \
        max(x[1] for x in rows)
    rows = [x for x in rows if x[1] > t0 and x[0] < t1]
    span = t1 - t0
    nb = sum(1 for s in starts if s >= t0)
    print(f"window {span / 1e6:.2f} ms, {nb} batches -> {span / 1e6 / max(nb, 1):.3f} ms per batch")
    ev = []
    for i, x in enumerate(rows):
        ev.append((max(x[0], t0), 1, i))
        ev.append((x[1], -1, i))
    ev = [(min(t, t1), d, i) for t, d, i in ev]
    ev.sort()
    live = set()
    last = t0
    conc = collections.Counter()
    fillw = 0.0
    under = collections.Counter()   # kernel -> time (ns) it ran while the summed fill < 0.5
    under_t = 0
    qbusy = collections.Counter()
    for t, d, i in ev:
        if t > last and live:
            dt = t - last
            conc[len(live)] += dt
            fill = min(1.0, sum(rows[j][4] for j in live))
            fillw += fill * dt
            if fill < 0.5:
                under_t += dt
                for j in live:
                    under[rows[j][2]] += dt
            for q in {rows[j][3] for j in live}:
                qbusy[q] += dt
        elif t > last:
            conc[0] += t - last
            under_t += t - last
            under["<idle>"] += t - last
        last = t
        if d > 0:
            live.add(i)
        else:
            live.discard(i)
    print("concurrency (kernels running): " + ", ".join(f"{k}: {v / span:.1%}" for k, v in sorted(conc.items())))
    print(f"estimated wave-slot fill {fillw / span:.1%}; time with fill < 50%: {under_t / span:.1%}")
    print("queue busy: " + ", ".join(f"q{q}: {v / span:.0%}" for q, v in sorted(qbusy.items())))
    print("kernels present while fill < 50% (ms per batch):")
    for k, v in under.most_common(a.top):
        print(f"  {k:32s} {v / 1e6 / max(nb, 1):7.3f}")
    tot = collections.Counter()
    for x in rows:
        tot[x[2]] += min(x[1], t1) - max(x[0], t0)
    print("queue time per batch (ms):")
    for k, v in tot.most_common(a.top):
        print(f"  {k:32s} {v / 1e6 / max(nb, 1):7.3f}")


if __name__ == "__main__":
    main()
