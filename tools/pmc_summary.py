"""Summarise a tools/profile.sh run into profiles/<tag>_kernel_stats.csv and profiles/<tag>_pmc.json.

Per compute dtype profiled (tools/fwd_loop.py passes: AVSE_F32_SPLIT = "fp32_split", bf16) and per forward kernel
(labelled by its position in the launch sequence) the median over dispatches of:
  * HBM traffic, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
    FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so the read side is
    doubled; WRITE_SIZE is taken as is;
  * MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1,024 SIMDs (= 16 cycles per 16x16x32 bf16 MFMA);
    GRBM_GUI_ACTIVE is summed over the 8 XCDs, so active cycles = GUI / 8 and
    mfma_busy_frac = BUSY / (1024 * GUI / 8); eff_clock = (GUI / 8) / dispatch duration (profiled run).
"""
import collections
import csv
import glob
import json
import re
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernel-name prefix -> labels in launch order within one forward
LABELS = [("k_spec_seg", ["stft"]), ("k_spec640", ["stft"]), ("k_spec_dft", ["stft"]), ("k_aud_enc", ["audio_enc"]),
          ("k_conv_v1r", ["v_conv1"]), ("k_conv_v1s", ["v_conv1"]), ("k_conv_v1p", ["v_conv1"]),
          ("k_splitk_reduce", ["splitk_reduce"]),
          ("k_conv_stream<5,", ["v_conv2"]), ("k_conv_stream<3, 16, 16", ["v_conv3", "v_conv4"]),
          ("k_conv_stream<3, 8, 8", ["v_conv5"]), ("k_gemm<1>", ["v_conv6"]),
          ("k_gemm<0>", ["enc_dense", "dec_dense1", "dec_dense2"]), ("k_dec_head", ["dec_head"]),
          ("k_dec_tail", ["dec_tail"]), ("k_conv<", ["k_conv"]), ("k_istft", ["istft"]), ("k_ola", ["istft_ola"])]
ALGO_BYTES = {  # algorithmic HBM bytes per launch: bf16 2 B per value; split pairs 4 B
    ("bf16", "v_conv2", 512): 512 * (64 * 64 * 128 * 2 + 32 * 32 * 128 * 2) + 128 * 3200 * 2,
    ("fp32_split", "v_conv2", 512): 512 * (64 * 64 * 128 * 4 + 32 * 32 * 128 * 4) + 128 * 3200 * 4,
    ("stft", "stft", 4096): 4096 * (3200 * 4 + 80 * 20 * 4),
}
DTYPES = ("fp32_split", "bf16")   # tools/profile.sh passes pmc_<tag>_<dtype>_<counter>


def short(name):
    """'void avse::(anonymous namespace)::k_conv_stream<5, 16, ...>(avse::HaloArgs)' -> 'k_conv_stream<5, 16, ...>'.
    rocprofv3 leaves the _Float16 instantiations mangled ('_ZN4avse12_GLOBAL__N_16k_convIDF16_Li64ELb1ELb1EEEv...'):
    those are spelled out by hand."""
    m = re.search(r"k_convIDF16_Li(\d+)ELb([01])ELb([01])E", name)
    if m:
        tf = {"0": "false", "1": "true"}
        return f"k_conv<_Float16, {m.group(1)}, {tf[m.group(2)]}, {tf[m.group(3)]}>"
    m = re.search(r"\b(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name


def label_dispatches(rows):
    """rows: {dispatch_id: (kernel_name, duration_ns, {counter: value})} -> {label: [counters dicts]}"""
    seen = collections.Counter()
    out = collections.defaultdict(list)
    for d in sorted(rows):
        name, dur, ctr = rows[d]
        k = short(name)
        if "avse" not in name:
            continue
        for prefix, labels in LABELS:
            if k.startswith(prefix):
                lab = labels[seen[prefix] % len(labels)]
                seen[prefix] += 1
                out[lab].append((dur, ctr))
                break
    return out


def read_pass(path):
    rows = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if d not in rows:
                rows[d] = (r["Kernel_Name"], dur, {})
            c = rows[d][2]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return label_dispatches(rows)


def med(xs):
    return statistics.median(xs) if xs else None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(out, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    groups = {}
    passes = [(dt, 512, (f"{dt}_fetch", f"{dt}_write", f"{dt}_mfma")) for dt in DTYPES] + \
             [("stft", 4096, ("sfetch", "swrite", None))]
    for dt, batch, (pf, pw, pm) in passes:
        kern = groups.setdefault(dt, collections.defaultdict(dict))
        fetch = read_pass(os.path.join(out, f"pmc_{tag}_{pf}"))
        write = read_pass(os.path.join(out, f"pmc_{tag}_{pw}"))
        mfma = read_pass(os.path.join(out, f"pmc_{tag}_{pm}")) if pm else {}
        for lab in sorted(set(fetch) | set(write) | set(mfma)):
            e = kern[lab]
            e["batch"] = batch
            f = med([c.get("FETCH_SIZE", 0.0) * 1024 for _, c in fetch.get(lab, [])])
            w = med([c.get("WRITE_SIZE", 0.0) * 1024 for _, c in write.get(lab, [])])
            if f is not None:
                e["fetch_bytes_raw"] = f
                e["fetch_bytes_corrected"] = 2 * f
            if w is not None:
                e["write_bytes"] = w
            if f is not None and w is not None:
                e["traffic_bytes"] = 2 * f + w
            if (dt, lab, batch) in ALGO_BYTES:
                e["algorithmic_bytes"] = ALGO_BYTES[(dt, lab, batch)]
            if lab in mfma:
                busy = med([c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for _, c in mfma[lab]])
                gui = med([c.get("GRBM_GUI_ACTIVE", 0.0) for _, c in mfma[lab]])
                dur = med([d for d, _ in mfma[lab]])
                e.update({"mfma_busy_cycles": busy, "grbm_gui_active": gui, "profiled_ns": dur})
                if gui:
                    e["mfma_busy_frac"] = round(busy / (1024 * gui / 8), 4)
                    e["eff_clock_ghz"] = round(gui / 8 / dur, 3) if dur else None
            e["dispatches"] = len(fetch.get(lab, []))
    # rocprofv3 --kernel-trace --stats averages of the same tree (the bench's HIP-event figure is a separate run)
    # keyed by the full kernel symbol (template arguments tell the dtype variants apart)
    stats_avg_ms = {}
    if stats:
        for r in csv.DictReader(open(stats[0])):
            stats_avg_ms[short(r["Name"])] = round(float(r["AverageNs"]) / 1e6, 5)
    # the same averages over the headline-batch launches only: a symbol's dispatches in the profiled bench run also
    # include the one-clip zero-video encoder of the configs[2] leg (the --stats average of 29 calls mixed
    # a 0.09 ms N = 1 launch into the B = 512 figure).  A dispatch belongs to the headline batch when its grid is the
    # largest this symbol was launched with (the persistent convolutions' grid is min(tiles, CUs), so N = 1 launches
    # have a smaller one) — and, for kernels with a grid independent of N, when its duration is within 3x of the
    # median of those (the N = 1 launch of a full-chip grid is far shorter).
    stats_b512_ms, stats_b512_n = {}, {}
    traces = glob.glob(os.path.join(out, f"prof_{tag}", "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        disp = collections.defaultdict(list)
        for r in csv.DictReader(open(traces[0])):
            if "avse" not in r["Kernel_Name"]:
                continue
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            disp[short(r["Kernel_Name"])].append((grid, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for k, v in disp.items():
            gmax = max(g for g, _ in v)
            durs = [d for g, d in v if g == gmax]
            m = statistics.median(durs)
            durs = [d for d in durs if d * 3 >= m]
            stats_b512_ms[k] = round(statistics.mean(durs) / 1e6, 5)
            stats_b512_n[k] = len(durs)
    sys.path.insert(0, ROOT)
    import avse_pkg
    avse_pkg.load()
    from avse_amd import _lib
    res = {"tag": tag, "batch": 512, "source_digest": _lib.source_digest(),
           "source": "rocprofv3 --kernel-trace --stats of `bench.py --steps 20` (kernel_stats_avg_ms, by kernel "
           "symbol); --pmc passes FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE over "
           "tools/fwd_loop.py (B=512 spectrogram + forward, AVSE_DTYPE per dtype) and FETCH_SIZE | WRITE_SIZE over "
           "AVSE_MODE=stft (B=4096, 5 rotated buffer sets)",
           "dtypes": {dt: {"kernels": groups.get(dt, {}), "kernel_stats_avg_ms": stats_avg_ms,
                           "kernel_trace_headline_avg_ms": stats_b512_ms, "kernel_trace_headline_dispatches": stats_b512_n}
                      for dt in DTYPES},
           "stft_b4096": groups.get("stft", {})}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res)[:3000])


if __name__ == "__main__":
    main()
