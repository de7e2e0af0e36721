"""End-to-end enhancement of whole utterances on one GPU (BASELINE configs[4]): STFT -> fusion CNN -> ISTFT.

The reference's predict loop (speech_enhancer.py:61-88) handles one sample at a time: `preprocess_audio_signal`
(data_processor.py:35-57) slices the mixture's mel-dB spectrogram, the network predicts the speech slices
(network.py:208-212, with VideoNormalizer.normalize before it), and `reconstruct_speech_signal`
(data_processor.py:60-74) re-analyses the mixture for its phase and inverts the predicted mel-dB.  Here a batch of
equal-length utterances runs through the same three steps on device tensors:

  K1  avse_spectrogram  [U, L] -> mel-dB slices [U, S, 80, spf] + the complex STFT [U, 321, T] (kept for the phase,
                        so the mixture is analysed once, not twice as in the reference)
  fwd avse_forward      [U*S, 80, spf] x [U*S, 128, 128, frames] -> [U*S, 80, spf], in chunks of <= `chunk` clips
                        (the normaliser fused into v_conv1)
  K6  avse_istft        predicted slices + mixture phase -> [U, hop * (S*spf - 1)]

Every utterance is independent (top_db is per utterance), so a multi-GPU run shards utterances
(parallel.sharded_enhance) with no collective before the final gather.
"""
import torch

from . import _lib, data_processor, ops


class Enhancer:
    """Batched predict path for one device: `enhancer(signals, video, vmean, vstd)` -> enhanced signals."""

    def __init__(self, weights, video_frame_rate=25.0, sample_rate=16000, slice_duration_ms=200, chunk=1024):
        self.weights = weights
        self.fps = float(video_frame_rate)
        self.sr = int(sample_rate)
        self.slice_ms = slice_duration_ms
        self.chunk = int(chunk)
        self.range_bits = 0

    def geometry(self, n_video_slices):
        return data_processor.frame_geometry(self.sr, self.slice_ms, n_video_slices, self.fps)

    def __call__(self, signals, video, vmean=None, vstd=None, timings=None):
        """signals [U, L] float32 (int16-scale samples, padded / truncated to S slices like
        preprocess_audio_signal), video [U, S, 128, 128, frames] float32 raw mouth crops; vmean / vstd the
        VideoNormalizer images.  Returns [U, hop * (S * spf - 1)] float32 enhanced speech.
        `timings`, when a dict, receives the stages' HIP-event milliseconds (adds synchronisation)."""
        if signals.dim() != 2 or video.dim() != 5 or video.shape[0] != signals.shape[0]:
            raise ValueError("signals must be [U, L] and video [U, S, H, W, frames] with the same U")
        U, S = video.shape[0], video.shape[1]
        g = self.geometry(S)
        if g["n_slices"] != S:
            raise ValueError(f"{S} video slices but the audio geometry gives {g['n_slices']} spectrogram slices")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timings is not None else None
        if ev:
            ev[0].record()
        L = g["signal_length"]
        if signals.shape[1] != L:
            signals = torch.nn.functional.pad(signals, (0, max(0, L - signals.shape[1])))[:, :L].contiguous()
        spf = g["spectrogram_samples_per_slice"]
        if spf != self.weights.T or video.shape[-1] != self.weights.F:
            raise ValueError(f"{self.fps} fps gives [80, {spf}] slices with {video.shape[-1]} video frames; the weights "
                             f"are for [80, {self.weights.T}] x {self.weights.F} frames (build the network for this rate)")
        mel, stft = ops.spectrogram(signals, sample_rate=self.sr, n_fft=g["n_fft"], hop_length=g["hop_length"],
                                    n_mels=data_processor.N_MELS, fmin=data_processor.MEL_FMIN,
                                    fmax=data_processor.MEL_FMAX, frames_per_slice=spf, return_stft=True)
        if ev:
            ev[1].record()
        n = U * S
        clips = mel.view(n, data_processor.N_MELS, spf)
        frames = video.reshape((n,) + tuple(video.shape[2:]))
        pred = torch.empty_like(clips)
        # float32_split: each chunk's range guard is verified one chunk later (ops.RangePipeline), so the chunks'
        # forwards queue back to back; a flagged chunk is recomputed on the exact-fp32 kernels
        split = self.weights.dtype == _lib.AVSE_F32_SPLIT
        pipe = ops.RangePipeline(self.weights.ctx) if split else None
        if split:
            self.weights.ctx.set_aside_range()   # earlier forwards' bits stay readable by range_status()

        def chunk(a, b, checked):
            ops.forward(self.weights, clips[a:b], frames[a:b], vmean, vstd, out=pred[a:b], checked=checked)

        for a in range(0, n, self.chunk):
            b = min(n, a + self.chunk)
            chunk(a, b, False)
            if split:
                pipe.submit(lambda a=a, b=b: chunk(a, b, True))
        if ev:
            ev[2].record()
        def istft():
            return ops.istft(pred.view(U, S, data_processor.N_MELS, spf), stft, sample_rate=self.sr, n_fft=g["n_fft"],
                             hop_length=g["hop_length"], n_mels=data_processor.N_MELS, fmin=data_processor.MEL_FMIN,
                             fmax=data_processor.MEL_FMAX)
        out = istft()
        self.range_bits = 0
        if split:
            self.range_bits = pipe.drain()
            if pipe.recomputed:      # a chunk was redone after the ISTFT had been queued: redo the ISTFT after it
                out = istft()
        if ev:
            ev[3].record()
            ev[3].synchronize()
            timings.update(stft_ms=ev[0].elapsed_time(ev[1]), forward_ms=ev[1].elapsed_time(ev[2]),
                           istft_ms=ev[2].elapsed_time(ev[3]))
        return out
