"""Per-kernel VGPR / spill / scratch report of every HIP source of the library (gfx950 code
objects via -save-temps): a kernel that spills to scratch runs at a fraction of its speed
(r03: layernorm_rows spilled 6214 VGPRs). usage: python tools/spill_report.py [--all]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "person_capture_amd", "csrc")


def main():
    show_all = "--all" in sys.argv
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for f in sorted(os.listdir(CSRC)):
            if not f.endswith(".hip"):
                continue
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-c",
                            os.path.join(CSRC, f), "-o", os.path.join(tmp, f + ".o"), "-save-temps=obj",
                            "-Wno-unused-result", "-I", CSRC], cwd=tmp, check=True, capture_output=True)
            asm = [x for x in os.listdir(tmp) if x.startswith(f[:-4] + "-hip-amdgcn") and x.endswith(".s")]
            s = open(os.path.join(tmp, asm[0])).read()
            for m in re.finditer(r"- \.agpr_count:\s+(\d+).*?\.name:\s+(\S+).*?\.private_segment_fixed_size:\s+(\d+)"
                                 r".*?\.vgpr_count:\s+(\d+).*?\.vgpr_spill_count:\s+(\d+)", s, re.S):
                agpr, name, scratch, vgpr, spill = m.groups()
                if show_all or int(spill) or int(scratch):
                    bad += int(spill) > 0
                    print(f"{f:24s} {name[:90]:90s} vgpr {vgpr:>3} agpr {agpr:>3} spill {spill:>5} scratch {scratch}")
            for x in os.listdir(tmp):
                os.remove(os.path.join(tmp, x))
    print(f"kernels with VGPR spills: {bad}")


if __name__ == "__main__":
    main()
