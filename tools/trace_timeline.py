"""Timeline (start / end relative to the spectrogram launch) of the last forwards in a rocprofv3 kernel trace.
    python3 tools/trace_timeline.py gpurun_out/<dir> [n_forwards]"""
import csv
import glob
import re
import sys


def main(d, nf=2):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    spec = [i for i, r in enumerate(rows) if "spec" in r["Kernel_Name"]]
    for k, i0 in enumerate(spec[-nf - 1:-1]):
        i1 = spec[spec.index(i0) + 1]
        t0 = int(rows[i0]["Start_Timestamp"])
        end = 0
        for r in rows[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            end = max(end, e)
            name = re.sub(r"\(.*", "", r["Kernel_Name"])[-58:]
            print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {r.get('Grid_Size', '?'):>8} {name}")
        print(f"forward span {(end - t0) / 1e3:.1f} us\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
