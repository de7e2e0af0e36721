"""Print selected stages of tools/gpu_envab.sh output:  python3 tools/envab_show.py stage1,stage2,..."""
import json
import sys

keys = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for line in open("gpurun_out/envab.log"):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    st = d["stage_ms"]
    ks = keys or list(st)
    print(f"{d['label'][:40]:40s} total={d['total_ms']:.4f} " + " ".join(f"{k}={st[k]:.4f}" for k in ks))
