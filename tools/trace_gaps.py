"""Summarise a rocprofv3 kernel-trace CSV: for the last forward pass, each kernel's duration and the
idle gap before it (launch overhead between dependent kernels)."""
import csv
import glob
import re
import sys


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one forward = the kernels after the last spectrogram launch
    spec = [i for i, r in enumerate(rows) if "spec" in r["Kernel_Name"]]
    i0 = spec[-1] if spec else 0
    while i0 > 0 and "spec" in rows[i0 - 1]["Kernel_Name"]:
        i0 -= 1
    prev_end = None
    tot_k = tot_g = 0.0
    for r in rows[i0:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        dur = (e - s) / 1e3
        tot_k += dur
        tot_g += max(gap, 0.0)
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:70]
        print(f"{dur:9.2f} us  gap {gap:8.2f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8}  {name}")
        prev_end = e
    print(f"kernels {tot_k:.1f} us, gaps {tot_g:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
