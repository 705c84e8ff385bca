"""Per-kernel register / scratch / spill counts of the built library, read from the gfx950 code objects'
metadata notes (no GPU needed).  Tooling only.

    python tools/resource_usage.py profiles/r2_kernel_resources.csv

Each translation unit's object (drand_amd/csrc/*.o, left by __graft_entry__.build()) carries the device
code in its .hip_fatbin section; clang-offload-bundler unbundles the gfx950 code object and llvm-readelf
prints its AMDGPU metadata.
"""
import csv
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = [".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size", ".max_flat_workgroup_size"]


def kernels_of(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*(?:- )?(\.[a-z_]+):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if line.lstrip().startswith("- ") and key in FIELDS + [".name", ".args"]:
            cur = {}
            out.append(cur)
        if cur is not None and (key in FIELDS or key == ".name"):
            cur.setdefault(key, val)
    return [k for k in out if ".name" in k and not k[".name"].endswith(".kd")]


def main(dst):
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for tu in ("drand_gpu.o", "kernels_hot.o") + tuple("kernels_check_%s.o" % p for p in "abcdef"):
            for k in kernels_of(os.path.join(ROOT, "drand_amd", "csrc", tu), tmp):
                rows.append([tu.replace(".o", ""), k[".name"]] + [k.get(f, "") for f in FIELDS])
    rows.sort(key=lambda r: (-int(r[7] or 0), r[1]))
    w = csv.writer(open(dst, "w", newline="") if dst else sys.stdout)
    w.writerow(["tu", "kernel"] + [f.lstrip(".") for f in FIELDS])
    w.writerows(rows)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)  # no argument: print only
