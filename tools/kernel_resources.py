"""Kernel resource table of the SHIPPED objects (csrc/_build/*.o): unbundle each gfx950 code
object and read its AMDGPU metadata (VGPRs, AGPRs, spills, scratch bytes per lane, LDS).

    python tools/kernel_resources.py [filter-substring] > profiles/r04_kernel_resources.txt
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


def kernels(obj):
    with tempfile.TemporaryDirectory() as td:
        co, fb = os.path.join(td, "co"), os.path.join(td, "fb")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj,
                        os.path.join(td, "x.o")], capture_output=True)
        if not os.path.exists(fb):
            return []  # host-only object
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle", f"--input={fb}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
        if not os.path.exists(co) or os.path.getsize(co) == 0:
            return []  # host-only object
        notes = subprocess.run([os.path.join(LLVM, "llvm-readobj"), "--notes", co], capture_output=True,
                               text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        def f(key):
            m = re.search(r"\." + key + r":\s+(\S+)", blk)
            return m.group(1) if m else "?"
        agpr = re.match(r"\s*(\d+)", blk).group(1)
        out.append((f("name"), f("vgpr_count"), agpr, f("vgpr_spill_count"), f("sgpr_spill_count"),
                    f("private_segment_fixed_size"), f("group_segment_fixed_size")))
    return out


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    rows = []
    for obj in sorted(glob.glob(os.path.join(ROOT, "ptv_interpolation_amd", "csrc", os.environ.get("PTV_RES_BUILD", "_build"), "*.o"))):
        for r in kernels(obj):
            rows.append((os.path.basename(obj),) + r)
    names = demangle([r[1] for r in rows])
    print("object\tkernel\tVGPRs\tAGPRs\tVGPR spills\tSGPR spills\tscratch B/lane\tLDS B/block")
    for r, n in zip(rows, names):
        if flt in n:
            n = re.sub(r"\(.*", "", n).replace("ptv::", "")
            print("\t".join([r[0], n] + list(r[2:])))


if __name__ == "__main__":
    main()
