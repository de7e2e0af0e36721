"""Benchmark: clips/sec of the fused STFT + audio-visual CNN forward on MI355X.

One "step" = one pass of the hot path over one batch of synthetic 200-ms clips already resident in
HBM: K1 spectrogram of B x 3200 samples -> mel-dB [B, 80, 20] -> full fusion forward (BASELINE.json
configs[3], bf16, batch 512 per GPU) -> [B, 80, 20] predicted speech spectrograms; for N > 1 the
outputs are all-gathered over RCCL (the north star's final gather).  Weak scaling: every rank
processes B clips per step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints ONE JSON line (see README / DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import _lib, ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402

METRIC = "clips/sec (STFT+CNN forward) on 200-ms@16kHz segments, 1/2/4/8 MI355X"
SR, SEG = 16000, 3200
# algorithmic work per clip
FLOP_PER_CLIP = 2 * 2688.4e6                     # whole forward, 5.377 GFLOP
FLOP_V_CONV2 = 2 * 64 * 64 * 128 * 3200          # dominant kernel: v_conv2 implicit GEMM (M=4096, N=128, K=3200)
STFT_BYTES_PER_CLIP = SEG * 4 + 80 * 20 * 4      # 12,800 B in + 6,400 B out
PEAK_TFLOPS = {"bf16": 256 * 4 * 2.4e9 * 1024 / 1e12, "fp32": 256 * 4 * 2.4e9 * 64 / 1e12}   # 2516.6 / 157.3
PEAK_HBM_GBS = 8000.0


def synth(rng, B):
    t = np.arange(SEG) / SR
    f0 = rng.uniform(200, 3000, size=(B, 1))
    audio = rng.normal(0, 3000, (B, SEG)) + 3000 * np.sin(2 * np.pi * f0 * t[None, :])
    audio = np.clip(np.round(audio), -32768, 32767).astype(np.float32)
    video = rng.integers(0, 256, (B, 128, 128, 5), dtype=np.uint8).astype(np.float32)
    return audio, video


def pmc_traffic(B, dtype):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/<round>_pmc_traffic.json, written by tools/profile.sh from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes at this batch), or None when no matching profile exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if d.get("batch") == B and dtype == "bf16" and "traffic_bytes_per_launch" in d:
            return int(d["traffic_bytes_per_launch"])
    return None


def cpu_baseline(audio, video, mean, std, model, budget_s=12.0, max_s=30.0):
    """The CPU oracle (numpy librosa restatement + torch-CPU fp32 Keras graph) on a bounded sample."""
    from oracle import keras_ref, librosa_ref
    cores = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        cores = min(cores, int(env))
    torch.set_num_threads(cores)
    sample = 16
    a, v = audio[:sample], video[:sample]
    wd = model.layer_dict()
    vn = librosa_ref.video_normalize(v, mean, std).astype(np.float32)
    clips, t0 = 0, time.perf_counter()
    while True:
        mel = np.stack([librosa_ref.preprocess_audio_signal(a[i], SR, 200, 1, 25.0)[0] for i in range(sample)])
        keras_ref.forward(wd, mel.astype(np.float32), vn, dtype=torch.float32)
        clips += sample
        el = time.perf_counter() - t0
        if el >= budget_s or el >= max_s:
            break
    return {"value": clips / el, "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"{sample} clips x {clips // sample} reps ({el:.1f} s): numpy STFT/mel/dB + torch-CPU fp32 "
                      "Keras-semantics forward (oracle/), same synthetic inputs"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="clips per GPU per step")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-reps", type=int, default=5)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    B = args.batch

    # weights: seeded Keras-layout init on rank 0, broadcast once over RCCL (not timed)
    blob = torch.from_numpy(KerasModel.init(seed=0, randomize=True).to_blob()).to(dev)
    if world > 1:
        dist.broadcast(blob, 0)
    from avse_amd.model import tensor_names
    host = blob.cpu().numpy()
    tensors, off = {}, 0
    for name, shape in tensor_names():
        n = int(np.prod(shape))
        tensors[name] = host[off:off + n].reshape(shape)
        off += n
    model = KerasModel(tensors)
    dw = ops.DeviceWeights(model, args.dtype, dev)
    dw.ctx.reserve(B, dw.dtype)

    rng = np.random.default_rng(1234 + rank)
    audio_np, video_np = synth(rng, B)
    mean_np = video_np.mean(axis=(0, 3)).astype(np.float32)
    std_np = video_np.std(axis=(0, 3)).astype(np.float32)
    audio = torch.from_numpy(audio_np).to(dev)
    video = torch.from_numpy(video_np).to(dev)
    mean, std = torch.from_numpy(mean_np).to(dev), torch.from_numpy(std_np).to(dev)
    out = torch.empty((B, 80, 20), dtype=torch.float32, device=dev)
    gathered = torch.empty((world * B, 80, 20), dtype=torch.float32, device=dev) if world > 1 else None

    def step():
        mel = ops.spectrogram(audio, frames_per_slice=20)          # [B, 1, 80, 20]
        ops.forward(dw, mel.view(B, 80, 20), video, mean, std, out=out)
        if world > 1:
            dist.all_gather_into_tensor(gathered, out)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * B * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # ---- live per-kernel durations (HIP events on the launch stream) for the roofline ----
    stage_ms = {}
    for _ in range(args.profile_reps):
        mel = ops.spectrogram(audio, frames_per_slice=20)
        _, st = ops.forward_profile(dw, mel.view(B, 80, 20), video, mean, std, out=out)
        for k, v in st.items():
            stage_ms[k] = stage_ms.get(k, 0.0) + v / args.profile_reps
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.profile_reps):
        ops.spectrogram(audio, frames_per_slice=20)
    e1.record()
    torch.cuda.synchronize()
    stft_ms = e0.elapsed_time(e1) / args.profile_reps

    dom = "v_conv2"
    achieved = FLOP_V_CONV2 * B / (stage_ms[dom] * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    traffic = pmc_traffic(B, args.dtype)
    fwd_ms = sum(stage_ms.values())
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "clips/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: seeded int16-scale noise+harmonic audio (3200 samples/clip), uint8-valued 128x128x5 "
                "mouth crops, random-init Keras-layout weights with randomised BN; inputs resident in HBM",
        "config": {"workload": "STFT (n_fft 640, hop 160, 80 mel, dB) + full audio-visual fusion forward "
                               "(BASELINE configs[3]) on 200-ms@16kHz clips",
                   "global_batch": world * B, "per_gpu_batch": B, "parallelism": f"dp{world}"},
        "roofline": {"kernel": f"{dom} (k_conv_stream<5,16,16,1>: persistent warp-specialised implicit GEMM "
                               "M=4096/clip N=128 K=3200, fused BN+LReLU+2x2 maxpool)" if args.dtype == "bf16" else
                               f"{dom} (k_conv<float,128> implicit GEMM, exact-fp32 MFMA)",
                     "bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "per_launch_flop": FLOP_V_CONV2 * B, "avg_launch_ms": round(stage_ms[dom], 4)},
        "breakdown": {
            "stft_ms": round(stft_ms, 4),
            "stft_hbm_gbs": round(STFT_BYTES_PER_CLIP * B / (stft_ms * 1e-3) / 1e9, 1),
            "stft_hbm_frac": round(STFT_BYTES_PER_CLIP * B / (stft_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "forward_ms": round(fwd_ms, 4),
            "forward_tflops": round(FLOP_PER_CLIP * B / (fwd_ms * 1e-3) / 1e12, 2),
            "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(audio_np, video_np, mean_np, std_np, model)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
