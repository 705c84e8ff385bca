"""One line per A/B run of tools/gpu/r4_ab.sh: the value of the line it ran and the kernel times that matter to it."""
import json
import sys

kind, name = sys.argv[1], sys.argv[2]
d = json.loads(open("gpurun_out/%s_%s.json" % (kind, name)).read().strip().splitlines()[-1])
t = json.load(open("gpurun_out/%s_%s_tables.json" % (kind, name)))
if kind == "head":
    print("head %-10s %.0f rounds/s %.3f ms/step" % (name, d["value"], d["ms_per_step"]), flush=True)
    ks = t.get("kernel_avg_us") or {}
    print("   ", json.dumps({k: v for k, v in ks.items() if k.startswith(("k_msm", "k_sum_rows", "k_exp"))}))
else:
    key = "adversarial" if kind == "c5" else "recover"
    a = d[key]
    ks = t.get(key, {}).get("kernel_avg_us") or {}
    print("%s %-10s %.0f /s  %.4f s/step" % (kind, name, a["value"], a["s_per_step"]), flush=True)
    print("   ", json.dumps({k: v for k, v in ks.items() if k.startswith(("k_rs_", "k_rc_", "k_kmsm", "k_msm", "k_ck_", "k_sum"))}))
