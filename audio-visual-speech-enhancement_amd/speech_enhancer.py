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
    runs evaluate and predict, two forwards of the same input).
All spectrogram / network / reconstruction arithmetic goes through libavse (K1, forward, K6).
"""
import argparse
import json
import logging
import os
import random
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


def predict(args):
    layout = Layout(args.base_dir)
    run_dir = layout.prediction_run_dir(args.model, args.data_name)
    model_path, keras_path = layout.model_file(args.model), layout.keras_model_file(args.model)
    if not os.path.exists(model_path) and os.path.exists(keras_path):
        raise SystemExit("%s is a Keras model: convert it once with\n  /opt/conda/bin/python3.9 tools/keras_h5_to_avse.py "
                         "%s %s" % (keras_path, keras_path, model_path))
    network = SpeechEnhancementNetwork.load(model_path, compute_dtype=args.dtype)
    video_normalizer = data_processor.VideoNormalizer.load(layout.normalizer_file(args.model))
    samples = load_preprocessed_blob(layout.preprocessed(args.data_name))
    for sample in samples:
        try:
            print("predicting (%s, %s)..." % (sample.video_file_path, sample.noise_file_path))
            # normalize + evaluate + predict as ONE forward, the normaliser fused into the first video conv
            pred, loss = network.predict_and_evaluate(sample.mixed_spectrograms, sample.video_samples,
                                                      sample.speech_spectrograms, video_normalizer=video_normalizer)
            print("loss: %f" % loss)
            signal = data_processor.reconstruct_speech_signal(sample.mixed_signal, pred, sample.video_frame_rate)
            write_prediction(run_dir, sample, signal)
        except Exception:  # noqa: BLE001 — mirrors speech_enhancer.py:87-88
            logging.exception("failed to predict %s. skipping" % sample.video_file_path)


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
    q.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    q.set_defaults(func=predict)

    args = parser.parse_args(argv)
    args.func(args)


if __name__ == "__main__":
    main()
