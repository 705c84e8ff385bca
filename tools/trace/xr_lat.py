"""Per-kernel durations of the isolation's active launches (longer than 50 us) in one or more rocprofv3 kernel traces
(tooling): median and p90 per kernel, side by side.   python tools/trace/xr_lat.py trace1.csv [trace2.csv ...]"""
import collections
import csv
import sys

import numpy as np

KERNELS = ["k_xg_sub", "k_xq_sum", "k_xg_prep", "k_xg_lines", "k_ck_miller2", "k_ck_easy", "k_ck_expsq2",
           "k_ck_expsq", "k_ck_expdec", "k_ck_explain", "k_ck_final", "k_pair_miller_coop", "k_final_coop",
           "k_msm_horner_coop", "k_exp_pm3d4"]


def main():
    cols = []
    for path in sys.argv[1:]:
        d = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"].split("(")[0]
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if us > 50:
                d[n].append(us)
        cols.append(d)
    print("kernel".ljust(22) + "".join(f"{'trace%d med/p90 (n)' % i:>30s}" for i in range(len(cols))))
    for k in KERNELS:
        row = k.ljust(22)
        for d in cols:
            v = np.array(d.get(k, [0.0]))
            row += f"{np.median(v):12.0f}{np.percentile(v, 90):10.0f} ({len(d.get(k, [])):4d})"
        print(row)


if __name__ == "__main__":
    main()
