"""Probe: does running consecutive bench steps on two streams (two contexts, i.e. two activation arenas, one set of
weights) raise throughput?  Step i = STFT + split forward of its own 512-clip batch on stream i % 2, so batch i+1's
video encoder can start while batch i's decoder runs.  Prints ms per step for one stream and for two.
    python tools/overlap_probe.py [steps] [dtype]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
import bench  # noqa: E402
from avse_amd import _lib, ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dtype = sys.argv[2] if len(sys.argv) > 2 else "float32_split"
    B = 512
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = KerasModel.init(seed=0, randomize=True)
    # options read when weights are loaded (no_halo) must be set before DeviceWeights
    for opt in os.environ.get("PROBE_OPTS", "").split(","):
        if opt:
            _lib.check(_lib.load().avse_ctx_set_option(_lib.context(dev).handle, opt.encode(), 1), "set_option " + opt)
    dw = ops.DeviceWeights(model, dtype, dev)
    ctxs = [dw.ctx, _lib.Context(0)]
    for c in ctxs:
        _lib.check(_lib.load().avse_ctx_reserve_weights(c.handle, dw.handle, B), "reserve")
    rng = np.random.default_rng(1)
    sets = []
    for _ in range(2):
        a, v = bench.synth(rng, B)
        sets.append(dict(audio=torch.from_numpy(a).to(dev), video=torch.from_numpy(v).to(dev),
                         mean=torch.from_numpy(v.mean(axis=(0, 3)).astype(np.float32)).to(dev),
                         std=torch.from_numpy(v.std(axis=(0, 3)).astype(np.float32)).to(dev),
                         mel=torch.empty((B, 1, 80, 20), dtype=torch.float32, device=dev),
                         out=torch.empty((B, 80, 20), dtype=torch.float32, device=dev)))
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    lib = _lib.load()
    for opt in os.environ.get("PROBE_OPTS", "").split(","):   # e.g. PROBE_OPTS=no_win,serial
        if opt:
            for c in ctxs:
                _lib.check(lib.avse_ctx_set_option(c.handle, opt.encode(), 1), "set_option " + opt)

    def step(i, two):
        d = i % 2                      # the batch (both modes alternate the two input sets)
        k = d if two else 0            # stream / context
        s, c, st = sets[d], ctxs[k], streams[k]
        with torch.cuda.stream(st):
            ops.spectrogram(s["audio"], frames_per_slice=20, out=s["mel"])
            _lib.check(lib.avse_forward(c.handle, dw.handle, _lib.ptr(s["mel"]), _lib.ptr(s["video"]),
                                        _lib.ptr(s["mean"]), _lib.ptr(s["std"]), B, _lib.ptr(s["out"]),
                                        ctypes.c_void_p(st.cuda_stream)), "avse_forward")

    if len(sys.argv) > 3 and sys.argv[3] in ("istft", "istft_dense", "istft533"):
        # the ISTFT (k_istft_fused; istft_dense: k_istft640 + k_ola; istft533: k_istft532) alone, then beside the MFMA
        # stress kernels on another stream, 3-s utterances
        st = ctypes.CDLL(os.path.join(ROOT, "tools", "_stress", "libmfma_stress.so"))
        sbuf = torch.empty(4096 * 256 * 4, dtype=torch.float32, device=dev)
        n_fft, hop, spf = (533, 133, 24) if sys.argv[3] == "istft533" else (640, 160, 20)
        xu = torch.from_numpy(np.random.default_rng(5).normal(0, 3000, (64, 48000)).astype(np.float32)).to(dev)
        mel, D = ops.spectrogram(xu, n_fft=n_fft, hop_length=hop, frames_per_slice=spf, return_stft=True)
        ictx = _lib.context(dev)
        if sys.argv[3] == "istft_dense":
            _lib.check(lib.avse_ctx_set_option(ictx.handle, b"dense_istft", 1), "dense_istft")
        ref = ops.istft(mel, D, n_fft=n_fft, hop_length=hop)
        torch.cuda.synchronize()
        reps = int(os.environ.get("PROBE_REPS", "24"))
        for what in ("solo", "beside stress0"):
            nbad = 0
            for rep in range(reps):
                for i in range(steps):
                    if what != "solo":
                        st.mfma_stress(0, ctypes.c_void_p(sbuf.data_ptr()), 4096, 2000,
                                       ctypes.c_void_p(streams[1].cuda_stream))
                    y = ops.istft(mel, D, n_fft=n_fft, hop_length=hop)
                torch.cuda.synchronize()
                nbad += bool((y != ref).any())
            print(f"{sys.argv[3]} {what}: {nbad} of {reps} reps differ", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "oob":
        # one stream: STFT + forward of both sets once, snapshot every buffer, then forwards of set 1 only; any change
        # in a buffer the forward does not own (set 0's, set 1's inputs) is a stray store
        for d in (0, 1):
            step(d, False)
        torch.cuda.synchronize()
        snap = {(d, k): v.clone() for d, st_ in enumerate(sets) for k, v in st_.items()}
        s1 = sets[1]
        for i in range(steps):
            _lib.check(lib.avse_forward(ctxs[0].handle, dw.handle, _lib.ptr(s1["mel"]), _lib.ptr(s1["video"]),
                                        _lib.ptr(s1["mean"]), _lib.ptr(s1["std"]), B, _lib.ptr(s1["out"]),
                                        ctypes.c_void_p(streams[0].cuda_stream)), "avse_forward")
        torch.cuda.synchronize()
        for (d, k), v in snap.items():
            cur = sets[d][k]
            n = int((cur != v).sum())
            if n:
                idx = (cur != v).flatten().nonzero().flatten()
                print(f"set {d} {k}: {n} elements changed, flat offsets {idx[:6].tolist()} .. {idx[-1].item()} of "
                      f"{cur.numel()}", flush=True)
        print("oob checked", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "dummy":
        # spectrograms on stream 0 while stream 1 runs other work: torch matmuls, then the forward alone
        d = 0
        if len(sys.argv) > 4 and sys.argv[4] == "k_spec640":   # unaligned mel: k_spec640 instead of the DMA kernel
            for st_ in sets:
                st_["mel_raw"] = torch.empty(B * 80 * 20 + 4, dtype=torch.float32, device=dev)
                st_["mel"] = st_["mel_raw"][1:1 + B * 80 * 20].view(B, 1, 80, 20)
            step(1, False)
        step(0, False)
        torch.cuda.synchronize()
        mref = sets[0]["mel"].clone()
        a_ = torch.randn(4096, 4096, device=dev)
        x_ = torch.randn(16384, 2048, device=dev)
        _stress = None
        if "stress" in os.environ.get("PROBE_KINDS", ""):
            _stress = ctypes.CDLL(os.path.join(ROOT, "tools", "_stress", "libmfma_stress.so"))
            stress_buf = torch.empty(4096 * 256 * 4, dtype=torch.float32, device=dev)
        reps = int(os.environ.get("PROBE_REPS", "12"))
        kinds = os.environ.get("PROBE_KINDS", "matmul,torch mix,forward").split(",")
        for what in kinds:
            nbad = 0
            for rep in range(reps):
                for i in range(steps):
                    with torch.cuda.stream(streams[1]):
                        if what == "matmul":
                            a_ @ a_
                        elif what.startswith("stress"):   # tools/mfma_stress.hip: kind 0 f16, 1 bf16, 2 f16 + fp32 stores
                            _stress.mfma_stress(int(what[-1]), ctypes.c_void_p(stress_buf.data_ptr()), 4096, 2000,
                                                ctypes.c_void_p(streams[1].cuda_stream))
                        elif what == "torch mix":   # many small LDS-using workgroups (reductions, norms, sorts)
                            torch.softmax(x_, dim=-1)
                            torch.nn.functional.layer_norm(x_, (2048,))
                            x_.sum(dim=0)
                            torch.sort(x_[:2048], dim=-1)
                        else:
                            s1 = sets[1]
                            _lib.check(lib.avse_forward(ctxs[1].handle, dw.handle, _lib.ptr(s1["mel"]),
                                                        _lib.ptr(s1["video"]), _lib.ptr(s1["mean"]), _lib.ptr(s1["std"]),
                                                        B, _lib.ptr(s1["out"]), ctypes.c_void_p(streams[1].cuda_stream)),
                                       "avse_forward")
                    with torch.cuda.stream(streams[0]):
                        ops.spectrogram(sets[0]["audio"], frames_per_slice=20, out=sets[0]["mel"])
                torch.cuda.synchronize()
                bad = int((sets[0]["mel"] != mref).sum())
                nbad += bad > 0
                if bad:
                    m, r = sets[0]["mel"].view(B, 80, 20), mref.view(B, 80, 20)
                    idx = (m != r).nonzero()
                    frames = sorted(set(idx[:, 2].tolist()))
                    print(f"  rep {rep}: {bad} mel values differ in {len(set(idx[:, 0].tolist()))} clips, frames {frames}",
                          flush=True)
                    sets[0]["mel"].copy_(mref)
            print(f"spectrogram beside {what}: {nbad} of {reps} reps with a wrong mel", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "guards":
        # every buffer a step writes or reads sits between two 1-MiB sentinel regions; after single-stream steps any
        # changed sentinel is an out-of-bounds store by the kernel that owns the buffer
        G = 1 << 18   # floats per guard
        raw = {}
        for d, st_ in enumerate(sets):
            for key in ("mel", "out"):
                n = st_[key].numel()
                r = torch.full((G + n + G,), -12345.0, dtype=torch.float32, device=dev)
                raw[(d, key)] = r
                st_[key] = r[G:G + n].view(st_[key].shape)
        for i in range(steps):
            step(i, False)
        torch.cuda.synchronize()
        for (d, key), r in raw.items():
            for side, g in (("before", r[:G]), ("after", r[-G:])):
                bad = (g != -12345.0).nonzero().flatten()
                if bad.numel():
                    print(f"set {d} {key}: {bad.numel()} sentinel floats changed {side} the buffer, offsets "
                          f"{bad[:8].tolist()} .. {bad[-1].item()} (guard of {G})", flush=True)
        print("guards checked", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "combined":
        # the whole step pipelined on two streams, 12 reps, with the spectrogram on the shared per-device context
        # (ops.spectrogram) or on the step's own context
        def step_own(i):
            d = i % 2
            s, c, st = sets[d], ctxs[d], streams[d]
            with torch.cuda.stream(st):
                _lib.check(lib.avse_spectrogram(c.handle, _lib.ptr(s["audio"]), B, 3200, 16000, 640, 160, 80, 0.0,
                                                8000.0, 1e-5, 80.0, _lib.AVSE_PAD_REFLECT, 20, _lib.ptr(s["mel"]),
                                                _lib.ptr(None), ctypes.c_void_p(st.cuda_stream)), "avse_spectrogram")
                _lib.check(lib.avse_forward(c.handle, dw.handle, _lib.ptr(s["mel"]), _lib.ptr(s["video"]),
                                            _lib.ptr(s["mean"]), _lib.ptr(s["std"]), B, _lib.ptr(s["out"]),
                                            ctypes.c_void_p(st.cuda_stream)), "avse_forward")
        unaligned = len(sys.argv) > 4 and sys.argv[4] == "k_spec640"
        if unaligned:
            # a mel buffer 4 B off 16-B alignment: the segment kernel (LDS-DMA) declines it, k_spec640 runs instead
            for st_ in sets:
                st_["mel_raw"] = torch.empty(B * 80 * 20 + 4, dtype=torch.float32, device=dev)
                st_["mel"] = st_["mel_raw"][1:1 + B * 80 * 20].view(B, 1, 80, 20)
        for d in (0, 1):
            step(d, False)
        torch.cuda.synchronize()
        oref = {d: sets[d]["out"].clone() for d in (0, 1)}
        mref = {d: sets[d]["mel"].clone() for d in (0, 1)}
        for what in ("shared spectrogram ctx", "own spectrogram ctx"):
            nbad = 0
            for rep in range(12):
                for i in range(steps):
                    if what.startswith("shared"):
                        step(i, True)
                    else:
                        step_own(i)
                torch.cuda.synchronize()
                res = [int((sets[d]["out"] != oref[d]).sum()) for d in (0, 1)]
                mres = [int((sets[d]["mel"] != mref[d]).sum()) for d in (0, 1)]
                nbad += any(res)
                if any(res) or any(mres):
                    print(f"  {what} rep {rep}: differing output elements per batch {res}, mel elements {mres}",
                          flush=True)
                    for d in (0, 1):
                        m, r = sets[d]["mel"].view(B, 80, 20), mref[d].view(B, 80, 20)
                        idx = (m != r).nonzero()
                        for clip in sorted(set(idx[:, 0].tolist()))[:3]:
                            sel = idx[idx[:, 0] == clip]
                            vals = [(int(b), int(f), round(float(m[clip, b, f]), 3), round(float(r[clip, b, f]), 3))
                                    for _, b, f in sel[:6].tolist()]
                            print(f"    set {d} clip {clip}: {sel.shape[0]} values differ; ref max "
                                  f"{float(r[clip].max()):.3f} floor {float(r[clip].max()) - 80:.3f}; ref min "
                                  f"{float(r[clip].min()):.3f}; (band, frame, got, ref) {vals}", flush=True)
                        if (sets[d]["mel"] != mref[d]).any():
                            sets[d]["mel"].copy_(mref[d])
            print(f"{what}: {nbad} of 12 reps differ", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "isolate":
        # which part races across the two streams: forwards alone (mel fixed), or spectrograms alone
        def fwd(i, two):
            d = i % 2
            k = d if two else 0
            s, c, st = sets[d], ctxs[k], streams[k]
            with torch.cuda.stream(st):
                _lib.check(lib.avse_forward(c.handle, dw.handle, _lib.ptr(s["mel"]), _lib.ptr(s["video"]),
                                            _lib.ptr(s["mean"]), _lib.ptr(s["std"]), B, _lib.ptr(s["out"]),
                                            ctypes.c_void_p(st.cuda_stream)), "avse_forward")

        def spec(i, two):
            d = i % 2
            st = streams[d if two else 0]
            with torch.cuda.stream(st):
                ops.spectrogram(sets[d]["audio"], frames_per_slice=20, out=sets[d]["mel"])
        for d in (0, 1):
            step(d, False)
        torch.cuda.synchronize()
        mref = {d: sets[d]["mel"].clone() for d in (0, 1)}
        oref = {d: sets[d]["out"].clone() for d in (0, 1)}
        for what, fn, ref, key in (("forward only", fwd, oref, "out"), ("spectrogram only", spec, mref, "mel")):
            for rep in range(6):
                for i in range(steps):
                    fn(i, True)
                torch.cuda.synchronize()
                res = [int((sets[d][key] != ref[d]).sum()) for d in (0, 1)]
                print(f"{what} rep {rep}: differing elements per batch {res}", flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "pipelined":
        # synchronized reference per batch, then pipelined runs (no host sync between steps) compared with it
        refs = {}
        for d in (0, 1):
            step(d, False)
            torch.cuda.synchronize()
            refs[d] = sets[d]["out"].clone()
        for rep in range(4):
            for two in (False, True):
                for i in range(steps):
                    step(i, two)
                torch.cuda.synchronize()
                res = []
                for d in (0, 1):
                    diff = (sets[d]["out"] - refs[d]).abs()
                    res.append((float(diff.max()), int((diff > 0).sum())))
                print(f"rep {rep} {'two streams' if two else 'one stream '}: (max |diff|, elements) per batch {res}",
                      flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "determinism":
        # every step's output against the first of its batch, one stream then two
        for two in (False, True):
            firsts, bad = {}, []
            for i in range(steps):
                step(i, two)
                torch.cuda.synchronize()
                d = i % 2
                o = sets[d]["out"].clone()
                if d not in firsts:
                    firsts[d] = o
                elif not torch.equal(o, firsts[d]):
                    diff = (o - firsts[d]).abs()
                    bad.append((i, float(diff.max()), int((diff > 0).sum())))
            print(f"{'two streams' if two else 'one stream '}: {len(bad)} of {steps - 2} repeated steps differ "
                  f"(step, max |diff|, elements): {bad[:6]}", flush=True)
        return
    ref = []
    for two in (False, True, False, True):
        for i in range(6):
            step(i, two)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i, two)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        outs = [s["out"].clone() for s in sets]
        if not two:
            ref = outs
        else:
            same = all(torch.equal(a, b) for a, b in zip(outs, ref))
        print(f"{'two streams' if two else 'one stream '}: {ms:.4f} ms per step = {B / ms * 1e3:9.1f} clips/s"
              + (f" (outputs equal to one stream: {same})" if two else ""), flush=True)


if __name__ == "__main__":
    main()
