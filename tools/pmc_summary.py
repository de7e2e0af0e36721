"""Summarise a tools/profile.sh run into profiles/<tag>_kernel_stats.csv and profiles/<tag>_pmc_traffic.json.

HBM traffic per launch of the dominant kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, so the read side is doubled; WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path, name):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(out, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = counter(os.path.join(out, f"pmc_{tag}_fetch"), "FETCH_SIZE")
    write = counter(os.path.join(out, f"pmc_{tag}_write"), "WRITE_SIZE")
    res = {"kernel": "k_conv_stream<5, 16, 16, 1, 10, 0> (v_conv2)", "batch": 512,
           "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tools/fwd_loop.py (B=512 bf16)",
           "dispatches": [len(fetch), len(write)]}
    if fetch and write:
        f = statistics.median(fetch) * 1024
        w = statistics.median(write) * 1024
        res.update({"fetch_size_bytes_raw": f, "fetch_bytes_corrected": 2 * f, "write_bytes": w,
                    "traffic_bytes_per_launch": 2 * f + w,
                    "algorithmic_bytes_per_launch": 512 * (64 * 64 * 128 * 2 + 32 * 32 * 128 * 2) + 128 * 3200 * 2})
    with open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
