"""Per-kernel register / spill / LDS metadata of the gfx950 code objects in build objects.
usage: python tools/kmeta.py <obj dir> [<filter substr>]   (one line per kernel: vgpr, agpr, spills, lds)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True,
                       capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", dev], check=True, capture_output=True,
                               text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|vgpr_spill_count|agpr_count|sgpr_spill_count|group_segment_fixed_size|"
                     r"wavefront_size):\s+(\S+)", line)
        if m:
            k, v = m.groups()
            cur[k] = v
            if k == "wavefront_size":  # the last key of a kernel's entry
                out.append(cur)
                cur = {}
    if cur.get("name"):
        out.append(cur)
    return out


def main():
    d = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for f in sorted(os.listdir(d)):
        if not f.endswith(".o"):
            continue
        for k in kernels(os.path.join(d, f)):
            n = subprocess.run(["c++filt"], input=k.get("name", "?"), capture_output=True, text=True).stdout.strip()
            if flt in n:
                print(f"{f:24s} vgpr {k.get('vgpr_count','?'):>4} agpr {k.get('agpr_count','?'):>3} "
                      f"spill {k.get('vgpr_spill_count','?'):>3} lds {k.get('group_segment_fixed_size','?'):>6}  {n}")


if __name__ == "__main__":
    main()
