"""preprocess / train / predict CLI with the flags of /root/reference/speech_enhancer.py:265-293.

    python -m avse_amd.speech_enhancer -bd BASE preprocess -dn NAME -ds DATASET -n NOISE_DIR [-s SPK ...]
    python -m avse_amd.speech_enhancer -bd BASE train -mn MODEL -tdn NAME ... -vdn NAME ... --init-only
    python -m avse_amd.speech_enhancer -bd BASE predict -mn MODEL -dn NAME [-g GPUS]

Same cache / output layout as the reference (speech_enhancer.py:91-184; corpus.py).
Differences (host plumbing outside the hot path):
  * video: the reference decodes with ffmpeg and crops the mouth with dlib (data_processor.py:12-32);
    this build reads pre-cropped mouth stacks <name>.npy [frames, 128, 128] (25 fps unless a
    <name>.fps text file says otherwise);
  * train: Keras-semantics fit on libavse's training step (network.train, fit.py); `--epochs` (default 1000
    like the reference) bounds it, `--init-only` writes only the initialised model + normaliser;
  * the enhanced/mixture .mp4 muxing (mediaio.ffmpeg.merge) runs only when ffmpeg is installed;
  * caches hold no pickles: preprocessed samples are <name>.npz (arrays + a JSON metadata string, read with
    allow_pickle=False), the normaliser normalization.npz, the model model.safetensors (a Keras model.h5py
    is converted once by tools/keras_h5_to_avse.py); the reference's own .pkl caches are not read (this
    build never unpickles);
  * predict runs ONE forward per sample: the printed loss (speech_enhancer.py:76-77, an MSE over the
    sample like Model.evaluate) is computed from the same prediction that is reconstructed (the reference
    runs evaluate and predict, two forwards of the same input);
  * predict batches: samples of one shape (slice count, frame rate, mixture length) run as one forward and one
    batched STFT / ISTFT (BatchPredictor) — every result equals the per-sample path's bit for bit (the fp32 forward
    is batch-invariant, csrc/capi.hip choose_ksplit); `-g N` (parsed and ignored by the reference,
    speech_enhancer.py:289) runs N ranks, one per GPU, each on a contiguous block of the samples.
All spectrogram / network / reconstruction arithmetic goes through libavse (K1, forward, K6).
"""
import argparse
import json
import logging
import os
import random
import socket
import subprocess
import sys
from collections import namedtuple

import numpy as np

from . import data_processor
from .audio_io import AudioMixer, AudioSignal
from .corpus import Layout, pair_speech_with_noise, speakers, write_prediction
from .network import SpeechEnhancementNetwork

Sample = namedtuple("Sample", ["speaker_id", "video_file_path", "speech_file_path", "noise_file_path", "video_samples",
                               "mixed_spectrograms", "speech_spectrograms", "noise_spectrograms", "mixed_signal",
                               "video_frame_rate"])


# ------------------------------------------------------------------------ preprocessing (host side)
def preprocess_video_sample(video_file_path, slice_duration_ms, mouth_height=128, mouth_width=128):
    """Stand-in for data_processor.py:12-32 on pre-cropped mouth stacks -> ([S, H, W, frames], fps)."""
    frames = np.load(video_file_path, allow_pickle=False).astype(np.float32)       # [F, H, W]
    if frames.shape[1:] != (mouth_height, mouth_width):
        raise ValueError(f"{video_file_path}: expected [F, {mouth_height}, {mouth_width}] mouth crops")
    fps_path = os.path.splitext(video_file_path)[0] + ".fps"
    fps = float(open(fps_path).read()) if os.path.exists(fps_path) else 25.0
    fps_slice = int((float(slice_duration_ms) / 1000) * fps)
    n_slices = int(float(frames.shape[0]) / fps_slice)
    crops = np.transpose(frames, (1, 2, 0))
    slices = [crops[:, :, i * fps_slice:(i + 1) * fps_slice] for i in range(n_slices)]
    return np.stack(slices), fps


def noise_at_snr(noise_signal, n_samples, speech_signal, snr_db=0):
    """The noise of data_processor.py:124-130 as one array: the reference doubles the noise signal until it is at
    least as long as the speech and truncates it, which is the noise repeated cyclically to n_samples (np.resize);
    then the 0-dB SNR gain against the speech."""
    looped = AudioSignal(np.resize(noise_signal.get_data(), (n_samples, noise_signal.get_number_of_channels())),
                         noise_signal.get_sample_rate())
    looped.amplify_by_factor(AudioMixer.snr_factor(speech_signal, looped, snr_db=snr_db))
    return looped


def preprocess_audio_pair(speech_file_path, noise_file_path, slice_duration_ms, n_video_slices, video_frame_rate):
    """data_processor.py:119-139: (mixed, speech, noise) slice stacks and the mixed signal.  Each stack comes from
    preprocess_audio_signal, which also pads / truncates its signal in place (the returned mixture is that one)."""
    speech = AudioSignal.from_wav_file(speech_file_path)
    noise = noise_at_snr(AudioSignal.from_wav_file(noise_file_path), speech.get_number_of_samples(), speech)
    mixture = AudioMixer.mix([speech, noise], mixing_weights=[1, 1])
    stacks = [data_processor.preprocess_audio_signal(sig, slice_duration_ms, n_video_slices, video_frame_rate)
              for sig in (mixture, speech, noise)]
    return stacks[0], stacks[1], stacks[2], mixture


def preprocess_sample(speech_entry, noise_file_path, slice_duration_ms=200):
    """data_processor.py:156-177."""
    video_samples, fps = preprocess_video_sample(speech_entry.video_path, slice_duration_ms)
    mixed, speech, noise, mixed_signal = preprocess_audio_pair(speech_entry.audio_path, noise_file_path,
                                                               slice_duration_ms, video_samples.shape[0], fps)
    n = min(video_samples.shape[0], mixed.shape[0])
    return Sample(speech_entry.speaker_id, speech_entry.video_path, speech_entry.audio_path, noise_file_path,
                  video_samples[:n], mixed[:n], speech[:n], noise[:n], mixed_signal, fps)


def preprocess_data(speech_entries, noise_file_paths):
    """data_processor.py:180-198 (catch-and-skip per sample; the GPU does the spectrograms, so no Pool)."""
    samples = []
    for entry, noise in zip(speech_entries, noise_file_paths):
        try:
            samples.append(preprocess_sample(entry, noise))
        except Exception as e:  # noqa: BLE001 — mirrors try_preprocess_sample
            print("failed to preprocess %s (%s)" % ((entry, noise), e))
    return samples


SAMPLE_ARRAYS = ("video_samples", "mixed_spectrograms", "speech_spectrograms", "noise_spectrograms")


def save_preprocessed_blob(path, samples):
    """list[Sample] -> one .npz: per sample its arrays and the mixture's samples, plus a JSON metadata string."""
    arrays, meta = {}, []
    for i, smp in enumerate(samples):
        for f in SAMPLE_ARRAYS:
            arrays["s%d_%s" % (i, f)] = np.asarray(getattr(smp, f))
        arrays["s%d_mixed_signal" % i] = np.asarray(smp.mixed_signal.get_data())
        meta.append({"speaker_id": smp.speaker_id, "video_file_path": smp.video_file_path,
                     "speech_file_path": smp.speech_file_path, "noise_file_path": smp.noise_file_path,
                     "video_frame_rate": float(smp.video_frame_rate),
                     "sample_rate": int(smp.mixed_signal.get_sample_rate())})
    arrays["meta"] = np.array(json.dumps(meta))
    with open(path, "wb") as fd:
        np.savez(fd, **arrays)


def load_preprocessed_blob(path):
    print("loading preprocessed samples from %s" % path)
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z["meta"]))
        out = []
        for i, m in enumerate(meta):
            arrs = {f: z["s%d_%s" % (i, f)] for f in SAMPLE_ARRAYS}
            signal = AudioSignal(z["s%d_mixed_signal" % i], m["sample_rate"])
            out.append(Sample(m["speaker_id"], m["video_file_path"], m["speech_file_path"], m["noise_file_path"],
                              arrs["video_samples"], arrs["mixed_spectrograms"], arrs["speech_spectrograms"],
                              arrs["noise_spectrograms"], signal, m["video_frame_rate"]))
    return out


def load_preprocessed_blobs(paths, max_samples_per_blob=None):
    return [smp for p in paths for smp in load_preprocessed_blob(p)[:max_samples_per_blob]]


def make_sample_set(samples, max_samples=None):
    """speech_enhancer.py:241-262: a random subset of the samples, their slices pooled and shuffled together ->
    (video [S, H, W, F], mixed [S, 80, T], speech [S, 80, T])."""
    chosen = random.sample(samples, len(samples) if max_samples is None else min(len(samples), max_samples))
    fields = ("video_samples", "mixed_spectrograms", "speech_spectrograms")
    pooled = [np.concatenate([getattr(smp, f) for smp in chosen], axis=0) for f in fields]
    order = np.random.permutation(pooled[0].shape[0])
    return tuple(a[order] for a in pooled)


# ------------------------------------------------------------------------ subcommands
def selected_speakers(args):
    """-s / -is flags: the listed speakers (default: every speaker directory) minus the ignored ones."""
    chosen = list(args.speakers) if args.speakers is not None else speakers(args.dataset_dir)
    return [s for s in chosen if s not in set(args.ignored_speakers or ())]


def preprocess(args):
    layout = Layout(args.base_dir)
    speech_entries, noise_file_paths = pair_speech_with_noise(args.dataset_dir, selected_speakers(args),
                                                              args.noise_dirs, limit=1000, shuffle=True)
    samples = preprocess_data(speech_entries, noise_file_paths)
    save_preprocessed_blob(layout.preprocessed(args.data_name), samples)
    print("preprocessed %d samples" % len(samples))


def train(args):
    """speech_enhancer.py:31-58: sample sets, VideoNormalizer fitted on the training video and applied in place to
    both sets, the normaliser saved, network built, fit with the model checkpointed every epoch, saved."""
    layout = Layout(args.base_dir)
    samples = load_preprocessed_blobs([layout.preprocessed(d) for d in args.train_data_names])
    video, mixed, speech = make_sample_set(samples)
    normalizer = data_processor.VideoNormalizer(video)
    normalizer.save(layout.normalizer_file(args.model))
    network = SpeechEnhancementNetwork.build(mixed.shape[1:], video.shape[1:], seed=args.seed)
    if not args.init_only:
        vsamples = load_preprocessed_blobs([layout.preprocessed(d) for d in args.validation_data_names])
        vvideo, vmixed, vspeech = make_sample_set(vsamples)
        normalizer.normalize(video)
        normalizer.normalize(vvideo)
        network.train(mixed, video, speech, vmixed, vvideo, vspeech, layout.model_file(args.model),
                      epochs=args.epochs, seed=args.seed)
    network.save(layout.model_file(args.model))


def predict_one(network, video_normalizer, sample):
    """The per-sample predict path of speech_enhancer.py:66-81: normalise + evaluate + predict as ONE forward (the
    normaliser fused into the first video conv), then reconstruct -> (loss, enhanced AudioSignal)."""
    pred, loss = network.predict_and_evaluate(sample.mixed_spectrograms, sample.video_samples,
                                              sample.speech_spectrograms, video_normalizer=video_normalizer)
    return loss, data_processor.reconstruct_speech_signal(sample.mixed_signal, pred, sample.video_frame_rate)


def sample_groups(samples):
    """Indices of the samples that run as one batch — same slice count and shapes, frame rate and mixture length
    (the batched ISTFT takes equal-length utterances) — in first-seen order."""
    groups = {}
    for i, smp in enumerate(samples):
        key = (tuple(smp.mixed_spectrograms.shape), tuple(smp.video_samples.shape), float(smp.video_frame_rate),
               smp.mixed_signal.get_number_of_samples(), smp.mixed_signal.get_sample_rate())
        groups.setdefault(key, []).append(i)
    return list(groups.values())


class BatchPredictor:
    """predict + evaluate + reconstruct of a group of equal-shape samples as one batch on one device: one forward over
    all their slices (in chunks of <= `chunk` clips), one MSE per sample (the avse_mse of the per-sample path), one
    STFT of the stacked mixtures for the phase and one ISTFT.  Each result equals predict_one's bit for bit."""

    def __init__(self, network, video_normalizer=None, chunk=1024):
        self.network = network
        self.video_normalizer = video_normalizer
        self.chunk = int(chunk)

    def __call__(self, group):
        import torch
        from . import _lib, ops
        dw = self.network.device_weights()
        dev = torch.device("cuda", dw.ctx.device_index)
        U = len(group)
        S, nm, T = group[0].mixed_spectrograms.shape
        mixed = torch.from_numpy(np.stack([g.mixed_spectrograms for g in group]).astype(np.float32)).to(dev)
        video = torch.from_numpy(np.stack([g.video_samples for g in group]).astype(np.float32)).to(dev)
        speech = torch.from_numpy(np.stack([g.speech_spectrograms for g in group]).astype(np.float32)).to(dev)
        m = s = None
        if self.video_normalizer is not None:
            m, s = self.video_normalizer.device_stats(dev)
        n = U * S
        clips, frames = mixed.view(n, nm, T), video.view((n,) + tuple(video.shape[2:]))
        pred = torch.empty_like(clips)
        for a in range(0, n, self.chunk):
            b = min(n, a + self.chunk)
            # the CLI is synchronous anyway: a float32_split batch's range guard is read per chunk (avse_forward_checked)
            ops.forward(dw, clips[a:b], frames[a:b], m, s, out=pred[a:b], checked=dw.dtype == _lib.AVSE_F32_SPLIT)
        pred = pred.view(U, S, nm, T)
        losses = [ops.mse(pred[u], speech[u]) for u in range(U)]
        sr, fps = group[0].mixed_signal.get_sample_rate(), group[0].video_frame_rate
        n_fft = int(float(sr) / fps)
        hop = int(n_fft / 4)
        sig = torch.from_numpy(np.stack([np.asarray(g.mixed_signal.get_data(channel_index=0)) for g in group])
                               .astype(np.float32)).to(dev)
        _, D = ops.spectrogram(sig, sample_rate=sr, n_fft=n_fft, hop_length=hop, n_mels=data_processor.N_MELS,
                               fmin=data_processor.MEL_FMIN, fmax=data_processor.MEL_FMAX, return_stft=True)
        y = ops.istft(pred.contiguous(), D, sample_rate=sr, n_fft=n_fft, hop_length=hop, n_mels=data_processor.N_MELS,
                      fmin=data_processor.MEL_FMIN, fmax=data_processor.MEL_FMAX).cpu().numpy()
        return [(float(losses[u].item()), AudioSignal(y[u], sr)) for u in range(U)]


def predict_samples(samples, predictor, run_dir, world=1, rank=0, write=write_prediction, fallback=None):
    """The predict loop over this rank's contiguous block of `samples` (parallel.shard_bounds), a batch per
    sample_groups group; outputs are written by the rank that owns the sample (one node: a shared file system).  A
    group that fails is retried sample by sample (`fallback`, or the predictor on one sample) so that, as in the
    reference (speech_enhancer.py:87-88), only the failing sample is skipped.  Returns {sample index: loss or None}
    for every sample on rank 0 (gathered from all ranks), this rank's own otherwise."""
    from .parallel import shard_bounds
    lo, hi = shard_bounds(len(samples), world, rank)
    mine = samples[lo:hi]
    losses = {}
    for idxs in sample_groups(mine):
        try:
            outs = predictor([mine[i] for i in idxs])
        except Exception:  # noqa: BLE001 — isolate the failing sample below
            outs = None
        for k, i in enumerate(idxs):
            try:
                loss, signal = outs[k] if outs is not None else (fallback or (lambda smp: predictor([smp])[0]))(mine[i])
                write(run_dir, mine[i], signal)
                losses[lo + i] = loss
            except Exception:  # noqa: BLE001 — mirrors speech_enhancer.py:87-88
                logging.exception("failed to predict %s. skipping" % mine[i].video_file_path)
                losses[lo + i] = None
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, losses)
        if rank == 0:
            for p in parts:
                losses.update(p)
    return losses


# the reference-shaped command line (repo root speech_enhancer.py): what every rank of `predict -g N` runs
ENTRY_SCRIPT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "speech_enhancer.py")


def rank_command(n, argv, port):
    """The torch.distributed.run command line of `predict -g N`: one rank per GPU (rendezvous on 127.0.0.1), each
    running the entry script with the same arguments `main` parsed (argv, not sys.argv: main(argv) may be called
    programmatically, or the CLI run as a module)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
            "127.0.0.1", "--master-port", str(port), ENTRY_SCRIPT] + list(argv)


def _launch_ranks(n, argv):
    """`predict -g N` outside a launcher: the ranks as a child process group; nothing in this process has touched the
    GPU."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    return subprocess.call(rank_command(n, argv, port))


def predict(args):
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args.gpus, args.argv))
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    layout = Layout(args.base_dir)
    model_path, keras_path = layout.model_file(args.model), layout.keras_model_file(args.model)
    if not os.path.exists(model_path) and os.path.exists(keras_path):
        raise SystemExit("%s is a Keras model: convert it once with\n  /opt/conda/bin/python3.9 tools/keras_h5_to_avse.py "
                         "%s %s" % (keras_path, keras_path, model_path))
    if world > 1:
        import torch
        import torch.distributed as dist
        # AVSE_DIST_BACKEND=gloo runs the ranks' collectives (run directory broadcast, loss gather) over gloo instead
        # of RCCL, and then ranks may share a GPU (local rank modulo the visible devices): RCCL refuses two ranks on
        # one device, which is all a one-GPU box can offer (tests/test_gpu_dist.py)
        backend = os.environ.get("AVSE_DIST_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend != "nccl":
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))
        # one timestamped run directory for every rank: rank 0 creates it
        box = [str(layout.prediction_run_dir(args.model, args.data_name)) if rank == 0 else None]
        dist.broadcast_object_list(box, 0)
        run_dir = box[0]
    else:
        run_dir = layout.prediction_run_dir(args.model, args.data_name)
    network = SpeechEnhancementNetwork.load(model_path, compute_dtype=args.dtype)
    video_normalizer = data_processor.VideoNormalizer.load(layout.normalizer_file(args.model))
    samples = load_preprocessed_blob(layout.preprocessed(args.data_name))
    if args.per_sample:
        predictor = lambda group: [predict_one(network, video_normalizer, smp) for smp in group]  # noqa: E731
    else:
        predictor = BatchPredictor(network, video_normalizer)
    losses = predict_samples(samples, predictor, run_dir, world, rank,
                             fallback=lambda smp: predict_one(network, video_normalizer, smp))
    if rank == 0:
        for i, smp in enumerate(samples):
            print("predicting (%s, %s)..." % (smp.video_file_path, smp.noise_file_path))
            if losses.get(i) is not None:
                print("loss: %f" % losses[i])
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main(argv=None):
    parser = argparse.ArgumentParser(add_help=False)
    parser.add_argument("-bd", "--base_dir", type=str, required=True)
    sub = parser.add_subparsers()

    p = sub.add_parser("preprocess")
    p.add_argument("-dn", "--data_name", type=str, required=True)
    p.add_argument("-ds", "--dataset_dir", type=str, required=True)
    p.add_argument("-n", "--noise_dirs", nargs="+", type=str, required=True)
    p.add_argument("-s", "--speakers", nargs="+", type=str)
    p.add_argument("-is", "--ignored_speakers", nargs="+", type=str)
    p.set_defaults(func=preprocess)

    t = sub.add_parser("train")
    t.add_argument("-mn", "--model", type=str, required=True)
    t.add_argument("-tdn", "--train_data_names", nargs="+", type=str, required=True)
    t.add_argument("-vdn", "--validation_data_names", nargs="+", type=str, required=True)
    t.add_argument("-g", "--gpus", type=int, default=1)
    t.add_argument("--init-only", action="store_true")
    t.add_argument("--epochs", type=int, default=1000)
    t.add_argument("--seed", type=int, default=0)
    t.set_defaults(func=train)

    q = sub.add_parser("predict")
    q.add_argument("-mn", "--model", type=str, required=True)
    q.add_argument("-dn", "--data_name", type=str, required=True)
    q.add_argument("-g", "--gpus", type=int, default=1)
    q.add_argument("--dtype", default="float32_split", choices=["float32_split", "float32", "bfloat16"])
    q.add_argument("--per-sample", action="store_true", help="one forward / STFT / ISTFT per sample (unbatched)")
    q.set_defaults(func=predict)

    argv = sys.argv[1:] if argv is None else list(argv)
    args = parser.parse_args(argv)
    args.argv = argv
    args.func(args)


if __name__ == "__main__":
    main()
