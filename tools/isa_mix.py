"""Static instruction mix of every kernel of the built library (gfx950 disassembly of the three translation
units), and the v_mad_u64_u32 count of one Montgomery product in each form (the reconciliation of
profiles/opcounts.json's issue basis, 392 per multiplication and 301 per squaring).  Tooling only.

    python tools/isa_mix.py profiles/r3_vmad_counts.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
sys.path.insert(0, ROOT)


def disasm(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def mix(text):
    cur, out = None, {}
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <([\w.$]+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        t = line.strip().split()
        if cur is None or not t or t[0].startswith(";"):
            continue
        out[cur][t[0]] = out[cur].get(t[0], 0) + 1
    return out


def product_counts(tmp):
    """v_mad_u64_u32 of one fp28_sos_mul_d and one fp28_sos_sqr_d (a kernel around each, compiled here)."""
    src = os.path.join(tmp, "one.hip")
    open(src, "w").write('#include "%s/drand_amd/csrc/field.h"\nusing namespace dg;\n' % ROOT + "".join(
        'extern "C" __global__ void k_%s(const uint32_t* a, uint32_t* o) {\n'
        '  const uint32_t i = threadIdx.x;  // per-lane operands (uniform ones compile to scalar code)\n'
        '  uint32_t x[14], y[14], r[14];\n  for (int j = 0; j < 14; ++j) { x[j] = a[28 * i + j]; y[j] = a[28 * i + 14 + j]; }\n'
        '  %s;\n  for (int j = 0; j < 14; ++j) o[14 * i + j] = r[j];\n}\n' % (n, c)
        for n, c in (("mul", "fp28_sos_mul_d(x, y, r)"), ("sqr", "fp28_sos_sqr_d(x, r)"))))
    obj = os.path.join(tmp, "one.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-o", obj, src],
                   check=True, capture_output=True)
    m = mix(disasm(obj, tmp))
    return {k: v.get("v_mad_u64_u32", 0) for k, v in m.items()}


def main(dst):
    lines = []
    with tempfile.TemporaryDirectory() as tmp:
        pc = product_counts(tmp)
        lines.append("# v_mad_u64_u32 per product (fp28.h, radix 2^28, 14 digits): %s" % pc)
        lines.append("# kernel  total  v_mad_u64_u32  share   (static instruction counts of the built objects)")
        for tu in ("drand_gpu.o", "kernels_hot.o"):
            m = mix(disasm(os.path.join(ROOT, "drand_amd", "csrc", tu), tmp))
            for k, v in sorted(m.items()):
                if not k.startswith("k_"):
                    continue
                tot = sum(v.values())
                vm = v.get("v_mad_u64_u32", 0)
                lines.append("%-26s %-16s %7d %7d  %.3f" % (k, tu.replace(".o", ""), tot, vm, vm / max(tot, 1)))
    open(dst, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r3_vmad_counts.txt"))
