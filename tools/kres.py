"""Per-kernel register / spill / LDS table of one csrc/*.hip file (hipcc -Rpass-analysis=kernel-resource-usage), so a
source change can be checked for new spills on the CPU before a GPU run.

    python tools/kres.py conv_stream.hip [filter-substring] [-D...]
"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-visual-speech-enhancement_amd",
                    "csrc")


def table(src, defs=(), flt=""):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-c", os.path.join(CSRC, src), "-o",
           "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage", *defs]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"\bAGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                         ("sspill", r"SGPRs Spill: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return [r for r in rows if flt in r["name"]]


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("-D")]
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    for r in table(args[0], defs, args[1] if len(args) > 1 else ""):
        print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('agpr', 0):>4} agpr {r.get('vspill', '?'):>4} spill "
              f"{r.get('lds', '?'):>6} lds occ {r.get('occ', '?')}  {r['name'][:110]}")
