"""Median per-dispatch FETCH_SIZE / WRITE_SIZE (corrected as tools/pmc_summary.py) and duration of each labelled
forward kernel in one rocprofv3 --pmc pass directory:   python tools/ab_fetch.py gpurun_out/<pass dir> [label ...]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as P  # noqa: E402


def main():
    d = P.read_pass(sys.argv[1])
    want = sys.argv[2:] or sorted(d)
    for lab in want:
        rows = d.get(lab, [])
        if not rows:
            continue
        f = statistics.median([c.get("FETCH_SIZE", 0.0) * 1024 * 2 for _, c in rows])
        w = statistics.median([c.get("WRITE_SIZE", 0.0) * 1024 for _, c in rows])
        t = statistics.median([dur for dur, _ in rows])
        print(f"{lab:14s} n={len(rows):3d} fetch {f / 1e6:9.1f} MB  write {w / 1e6:9.1f} MB  {t / 1e6:8.4f} ms")


if __name__ == "__main__":
    main()
