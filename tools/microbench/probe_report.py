"""Every form of the peak probe (tools/microbench/probe.hip) on one GPU, 2 s of launches each, as JSON:
lane-ops/s, the in-kernel clock, SIMD cycles per wave64 instruction.  Tooling (profiles/r3_probe.json)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drand_amd import shard  # noqa: E402

FORMS = {0: "v_mad_u64_u32, carry into VCC for every chain (round-2 probe)",
         1: "v_mad_u64_u32, distinct SGPR carry per chain (roofline denominator)",
         2: "v_mad_u64_u32, compiler form of (uint64_t)a*b + acc",
         3: "v_mad_u32_u24", 4: "v_mul_lo_u32", 5: "v_mul_hi_u32", 6: "v_add_u32 (full-rate calibration)",
         7: "v_fma_f32 (full-rate calibration)", 8: "v_fma_f32 on normal floats (form 7 runs on denormals)",
         9: "v_fma_f32 with an inline-constant addend (two VGPR sources)"}

if __name__ == "__main__":
    dev = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    out = {}
    for k, name in FORMS.items():
        out[name] = shard.probe_form(dev, k, warm_s=2.0)
        print(name, out[name], file=sys.stderr, flush=True)
    pk = shard.mad_peak(dev)
    out["mad_peak"] = pk
    print(json.dumps(out, indent=1))
