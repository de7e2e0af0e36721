"""Per-launch PMC summary of a tools/pmc_layers.sh run: dispatches of the matched kernel are grouped by their
position within one forward (the loop runs the forward several times) and averaged.
    python3 tools/pmc_layer_summary.py gpurun_out/pmcl_<tag>"""
import collections
import csv
import glob
import sys


def main(d):
    per = collections.defaultdict(dict)          # dispatch id -> counter -> value
    meta = {}
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        grp = f.split("/p")[-1].split("/")[0]
        for r in csv.DictReader(open(f)):
            key = (grp, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[key] = (int(r["Grid_Size"]), r["Kernel_Name"][:60],
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    # within each pass, order dispatches; position within a forward = index mod launches per forward
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for grp in sorted({k[0] for k in per}):
        ids = sorted(k[1] for k in per if k[0] == grp)
        keys = [(grp, i) for i in ids]
        grids = [meta[k][0] for k in keys]
        # launches per forward: smallest period of the grid-size sequence
        n = len(grids)
        period = next(p for p in range(1, n + 1) if all(grids[i] == grids[i % p] for i in range(n)))
        for j, k in enumerate(keys):
            pos = j % period
            for c, v in per[k].items():
                out[pos][c].append(v)
            out[pos]["_grid"] = [meta[k][0]]
            out[pos]["_us_" + grp].append(meta[k][2])
    for pos in sorted(out):
        o = out[pos]
        print(f"--- launch {pos} grid {o['_grid'][0]}")
        for c in sorted(o):
            if c.startswith("_grid"):
                continue
            v = sorted(o[c])[len(o[c]) // 2]
            print(f"   {c:32s} {v:16.1f}")
        h, m = o.get("TCC_HIT_sum"), o.get("TCC_MISS_sum")
        if h and m:
            hh, mm = sorted(h)[len(h) // 2], sorted(m)[len(m) // 2]
            print(f"   L2 hit rate                      {hh / max(hh + mm, 1):16.3f}")
        lat, req = o.get("TCP_TCC_READ_REQ_LATENCY_sum"), o.get("TCP_TCC_READ_REQ_sum")
        if lat and req:
            print(f"   L1->L2 read latency (cycles)     {sorted(lat)[len(lat)//2] / max(sorted(req)[len(req)//2], 1):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
