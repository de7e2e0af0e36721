/*
 * avse.h — C-ABI of libavse.so, the MI355X-native (gfx950) hot path of
 * melspectrum007/audio-visual-speech-enhancement.
 *
 * The reference has no FFI layer: its hot path is the Python API below, whose arithmetic is
 * delegated to librosa / numpy / Keras.  Each entry point names the reference interface it
 * replaces (file:line into /root/reference).  The build's Python package
 * (audio-visual-speech-enhancement_amd/) binds these symbols with ctypes; INTEGRATION.md shows
 * the binding a maintainer of the reference would add.
 *
 * Conventions
 *  - Every data pointer is a DEVICE pointer into caller-owned memory, unless the parameter name
 *    starts with host_.
 *  - Calls are asynchronous and ordered on `stream` (a hipStream_t passed as void*; NULL = the
 *    legacy default stream).  No call synchronises the device.
 *  - Every call returns an int status (AVSE_OK = 0).  avse_last_error() returns a thread-local
 *    message for the last failing call on this thread.
 *  - A context belongs to one device; it is not thread-safe (lock externally).
 *  - Buffers are row-major, C-contiguous, float32 unless stated.
 */
#ifndef AVSE_H
#define AVSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: compute dtype AVSE_F32_SPLIT, avse_ctx_reserve_weights; option names tile_alt / aud_side removed (round 3);
 *    status AVSE_ERR_CHECK (checked build)
 * 3: AVSE_F32_SPLIT range guard (avse_forward_checked, avse_range_status, status AVSE_ERR_RANGE), per-layer activation
 *    exponents (avse_weights_act_exponents, option no_act_scale) */
#define AVSE_ABI_VERSION 3

enum avse_status {
    AVSE_OK = 0,
    AVSE_ERR_INVALID = 1,      /* bad argument / shape                                  */
    AVSE_ERR_HIP = 2,          /* HIP runtime error (message in avse_last_error)       */
    AVSE_ERR_UNSUPPORTED = 3,  /* configuration outside what the kernels implement      */
    AVSE_ERR_OOM = 4,          /* device allocation failed                             */
    AVSE_ERR_CHECK = 5,        /* checked build only: a device-side protocol / bounds check fired */
    AVSE_ERR_RANGE = 6         /* avse_forward_checked(AVSE_RANGE_ERROR): a split-f16 activation left the f16 range */
};

/* Compute dtypes of avse_weights_load (inputs, outputs and accumulation are float32 in all three):
 *   AVSE_F32        every layer on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain)
 *   AVSE_BF16       activations and weights rounded to bf16 (the fast path; ~2e-3 relative output error)
 *   AVSE_F32_SPLIT  float32 accuracy on the 16-bit matrix cores: every layer carries each fp32 operand as an f16 pair
 *                   x = h + l (h = f16(x), l = f16(x - h); weights scaled per output channel by a power of two) and
 *                   forms the products with v_mfma_f32_16x16x32_f16, each MFMA rounding its 32 exact products once
 *                   into the fp32 accumulator (a K = 3200 dot product: more accurate than exact-fp32 MFMA,
 *                   tools/split_probe.hip): h h, l h, h l in the video convolutions v_conv1..v_conv5 (l l, 2^-22 of
 *                   |a b|, dropped), all four in the other layers.  Activations pass between layers as the pairs
 *                   (about 22 significant bits; the float32 network inputs are split on load, the decoder's last
 *                   output is float32): whole-network error measured 1.3x AVSE_F32's (6.8e-5 vs
 *                   5.1e-5 absolute RMS on dB-scale outputs, tests/test_gpu_split.py), inside the north star's 1e-4.
 *                   Range: a pair holds |x| < 65520 (f16 overflow) at ~22 bits from 2^-3 up.  Each layer stores the
 *                   pairs of x 2^e_L with a power-of-two exponent e_L from its BatchNormalization parameters (0 for
 *                   layers whose |beta| + |gamma| lies in [2^-2, 2^8]; avse_weights_act_exponents), and every kernel
 *                   that stores a pair (or splits an fp32 input) reports a value outside the range into a range guard:
 *                   avse_forward_checked recomputes such a batch on the exact-fp32 kernels (or fails with
 *                   AVSE_ERR_RANGE); after plain avse_forward calls avse_range_status tells whether any did. */
enum avse_dtype { AVSE_F32 = 0, AVSE_BF16 = 1, AVSE_F32_SPLIT = 2 };
enum avse_pad_mode { AVSE_PAD_REFLECT = 0, AVSE_PAD_CONSTANT = 1 };

typedef struct avse_ctx avse_ctx;
typedef struct avse_weights avse_weights;

/* ---- library / context ----------------------------------------------------------------- */

int avse_abi_version(void);
const char* avse_last_error(void);

/* One context per device: owns the DFT twiddle / window / mel tables and the forward scratch. */
int avse_ctx_create(int device, avse_ctx** out);
void avse_ctx_destroy(avse_ctx* ctx);

/* Kernel-path switches of a context, by name (A/B experiments and layer-by-layer parity tests; the
 * defaults are the production path).  Each is initialised at avse_ctx_create from an AVSE_*
 * environment variable and never re-read afterwards:
 *   no_gemm (AVSE_NO_GEMM)           v_conv6 + dense layers on k_conv + split-K reduce, not k_gemm
 *   no_audenc (AVSE_NO_AUDENC)       audio encoder layer by layer, not the fused k_aud_enc
 *   no_dechead / no_dectail          decoder head (d_deconv1..3) / tail (d_deconv4..6) layer by layer
 *   unfused_tail (AVSE_UNFUSED_TAIL) d_deconv6 as its own kernel (d_deconv5 activation materialised)
 *   no_halo (AVSE_NO_HALO)           video convs on k_conv (applies to weights loaded afterwards)
 *   mfma32 (AVSE_MFMA32)             32x32x16 compute waves in the stream convolutions
 *   serial (AVSE_SERIAL)             the per-layer audio branch on the caller's stream (not the side stream)
 *   graph (AVSE_GRAPH)               avse_forward replays a hipGraph per argument set
 *   gemm_ksplit_cap (AVSE_GEMM_KSPLIT) cap on k_gemm's split-K factor (0 = none)
 *   dense_istft (AVSE_DENSE_ISTFT)   avse_istft through the dense pinv + frame scratch + overlap-add pass
 *   no_act_scale (AVSE_NO_ACT_SCALE) AVSE_F32_SPLIT weights loaded afterwards keep every activation exponent 0
 *   no_win (AVSE_NO_WIN)             AVSE_F32_SPLIT stride-1 gather layers (decoder phases, a_conv2) on the generic
 *                                    k_conv instead of the windowed kernel
 *   no_v1p (AVSE_NO_V1P)             AVSE_F32_SPLIT 5-frame v_conv1 on k_conv_v1s (K 160) instead of k_conv_v1p
 *                                    (K 128; applies to weights loaded afterwards)
 *   no_a1valu (AVSE_NO_A1VALU)       AVSE_F32_SPLIT a_conv1 on audio_prep + k_conv instead of k_aconv1_split
 *   side_prio (AVSE_SIDE_PRIO)       audio side stream priority: 0 default, 1 least, 2 greatest (set before the
 *                                    context's first concurrent forward)
 * Unknown names return AVSE_ERR_INVALID. */
int avse_ctx_set_option(avse_ctx* ctx, const char* name, int value);
int avse_ctx_get_option(avse_ctx* ctx, const char* name, int* value);

/* Pre-size the forward scratch for up to max_clips clips of the 25-fps network so that later avse_forward calls
 * never allocate (required before capturing avse_forward into a hipGraph). */
int avse_ctx_reserve(avse_ctx* ctx, int64_t max_clips, int compute_dtype);
/* The same for the network shape and compute dtype `weights` were loaded for (avse_weights_load_shape: e.g. the
 * 29.97 / 30-fps networks need a larger scratch).  avse_forward fails with AVSE_ERR_INVALID, instead of growing the
 * scratch, while its stream is being captured. */
int avse_ctx_reserve_weights(avse_ctx* ctx, const avse_weights* weights, int64_t max_clips);

/* ---- audio front end ------------------------------------------------------------------- */

/* Replaces signal_to_spectrogram(audio_signal, n_fft, hop_length, mel=True, db=True)
 * (data_processor.py:77-96): librosa.core.stft (:79, periodic Hann, centred, pad_mode) ->
 * magphase (:80) -> librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) (Slaney) np.dot (:83-91)
 * -> librosa.amplitude_to_db(ref=1, amin, top_db) (:94), the top_db clamp taken over each
 * utterance's WHOLE [n_mels, T] array, and — when frames_per_slice > 0 — the slicing of
 * preprocess_audio_signal (data_processor.py:49-57) fused into the store.
 *
 *   sig      [n_utt][n_samples]                  channel-0 samples (already padded/truncated)
 *   T        = 1 + n_samples / hop               (centred frames)
 *   mel_db   frames_per_slice == 0: [n_utt][n_mels][T]
 *            frames_per_slice  > 0: [n_utt][n_slices][n_mels][frames_per_slice],
 *                                   n_slices = T / frames_per_slice (trailing frames dropped
 *                                   from the output but still inside the top_db max)
 *   stft_ri  nullable; [n_utt][n_fft/2+1][T][2]  complex STFT (re, im), librosa layout
 *
 * n_fft == 640 runs the mixed-radix (16 x 20) FFT kernel; other n_fft <= 2048 (e.g. 533 at
 * 29.97 fps, data_processor.py:44) run a direct-DFT kernel. */
int avse_spectrogram(avse_ctx* ctx, const float* sig, int64_t n_utt, int64_t n_samples,
                     int sr, int n_fft, int hop, int n_mels, float fmin, float fmax,
                     float amin, float top_db, int pad_mode, int frames_per_slice,
                     float* mel_db, float* stft_ri, void* stream);

/* Replaces reconstruct_signal_from_spectrogram (data_processor.py:99-116) as called by
 * reconstruct_speech_signal (:60-74): db_to_amplitude (:101) -> np.dot(pinv(mel), .) (:112) ->
 * x exp(i angle D) of the mixture STFT -> librosa.istft(hop_length=hop) (:114: periodic Hann,
 * window-sum-square normalisation, n_fft/2 trimmed at both ends).
 *   mel_db   frames_per_slice > 0: [n_utt][n_frames/frames_per_slice][n_mels][frames_per_slice]
 *            (the network's [N][80][20] output of consecutive slices = np.concatenate(..., axis=1))
 *            frames_per_slice == 0: [n_utt][n_mels][n_frames]
 *   stft_ri  [n_utt][n_fft/2+1][stft_frames][2] complex STFT of the mixture (avse_spectrogram's
 *            stft_ri output); the first n_frames frames are used (min(T_pred, T_phase), :68-70)
 *   sig      [n_utt][hop * (n_frames - 1)]
 * n_fft is the ANALYSIS size (int(sr / fps)); the inverse size is 2 * (n_fft/2), like librosa. */
int avse_istft(avse_ctx* ctx, const float* mel_db, const float* stft_ri, int64_t n_utt, int n_frames,
               int stft_frames, int frames_per_slice, int sr, int n_fft, int hop, int n_mels,
               float fmin, float fmax, float* sig, void* stream);

/* ---- network --------------------------------------------------------------------------- */

/* Number of float32 values in a canonical weight blob (see avse_weights_load): the 25-fps network
 * (build((80, 20), (128, 128, 5))). */
int64_t avse_weights_blob_floats(void);

/* The same for the network SpeechEnhancementNetwork.build((80, spec_frames), (128, 128, video_frames)) builds
 * (network.py:17-40; data_processor.py:44-52: spec_frames = int(slice samples / hop) = 20 at 25 fps, 24 at
 * 29.97 / 30 fps; video_frames = int(0.2 * fps) = 5 at 25 / 29.97 fps, 6 at 30 fps).  The shapes set the audio
 * embedding (5 x ceil(spec_frames / 4) x 128), the concat width (+ 2048) and the dense widths (concat / 4,
 * network.py:55).  -1 for shapes the kernels do not implement (spec_frames not a multiple of 4 — the decoder
 * would not reproduce 80 x spec_frames — or video_frames outside 1..8). */
int64_t avse_weights_blob_floats_shape(int spec_frames, int video_frames);

/* Replaces SpeechEnhancementNetwork.load (network.py:222-226) for the build's own weight format.
 * host_blob: the Keras-layout tensors of network.py's layers in creation order (float32):
 *   for each conv / dense / transposed-conv layer: kernel, bias
 *     conv (kh, kw, cin, cout); transposed conv (kh, kw, cout, cin); dense (in, out)
 *   followed, when the layer has a BatchNormalization, by gamma, beta, moving_mean,
 *   moving_variance.
 *   order: a_conv1..5, v_conv1..6, enc_dense, dec_dense1, dec_dense2, d_deconv1..6
 *   (d_deconv6 has no BatchNormalization).
 * BN (eps 1e-3) is folded into per-channel scale/shift; kernels are repacked for the implicit
 * GEMM and uploaded in compute_dtype (avse_dtype).  Synchronous. */
int avse_weights_load(avse_ctx* ctx, const float* host_blob, int64_t n_floats, int compute_dtype,
                      avse_weights** out);
/* avse_weights_load for the network of build((80, spec_frames), (128, 128, video_frames)); the weights remember
 * the shape, and avse_forward then takes audio [N][80][spec_frames] and video [N][128][128][video_frames].
 * The fused per-clip kernels cover the 25-fps shape (and v_conv1's 5-frame kernel every 5-frame shape); other
 * shapes run the generic implicit-GEMM path.  AVSE_ERR_UNSUPPORTED as avse_weights_blob_floats_shape's -1. */
int avse_weights_load_shape(avse_ctx* ctx, const float* host_blob, int64_t n_floats, int compute_dtype,
                            int spec_frames, int video_frames, avse_weights** out);
/* The shape the weights were loaded for. */
int avse_weights_shape(const avse_weights* w, int* spec_frames, int* video_frames);
void avse_weights_destroy(avse_weights* w);

/* Replaces SpeechEnhancementNetwork.predict's Model.predict (network.py:208-212) and the
 * VideoNormalizer.normalize it is preceded by (data_processor.py:208-212,
 * speech_enhancer.py:74), fused:
 *   audio      [N][80][20]        mixed mel-dB spectrograms (the expand_dims(-1) is implicit);
 *                                 [N][80][T] for weights loaded with avse_weights_load_shape(T, F)
 *   video      [N][128][128][5]   mouth crops ([N][128][128][F]), NOT normalised; NULL = an all-zero video input (the audio
 *                                 branch alone, BASELINE configs[2]: the video encoder's output is then one
 *                                 constant vector, computed once per weights object and broadcast;
 *                                 vnorm_* must be NULL)
 *   vnorm_mean [128][128]         nullable: VideoNormalizer mean image (applied in-kernel)
 *   vnorm_std  [128][128]         nullable: VideoNormalizer std image
 *   out        [N][80][20]        predicted speech mel-dB spectrograms (float32; [N][80][T])
 * Computes in the weights' compute dtype, accumulating in float32. */
int avse_forward(avse_ctx* ctx, const avse_weights* w, const float* audio, const float* video,
                 const float* vnorm_mean, const float* vnorm_std, int64_t N, float* out,
                 void* stream);

/* avse_forward for AVSE_F32_SPLIT weights with the range guard read back: waits for `stream` after the forward (not
 * capturable) and, when a stored activation or a split input left the f16 pair range (|x| >= 65520 or NaN; bit i of
 * *host_bits = plan layer i, a_conv1 = 0 .. d_deconv5 = 18; bit 24 the audio input, bit 25 the video input):
 *   mode AVSE_RANGE_RECOMPUTE  recomputes the whole batch on the exact-fp32 kernels (the AVSE_F32 path of the same
 *                              network, built once per weights object from the blob they were loaded from) into `out`
 *                              and returns AVSE_OK — the outputs are then the AVSE_F32 forward's;
 *   mode AVSE_RANGE_ERROR      returns AVSE_ERR_RANGE (outputs not float32-accurate).
 * host_bits (nullable) receives the bits (0: every pair was in range).  Other dtypes: avse_forward, *host_bits = 0. */
enum avse_range_mode { AVSE_RANGE_RECOMPUTE = 0, AVSE_RANGE_ERROR = 1 };
int avse_forward_checked(avse_ctx* ctx, const avse_weights* w, const float* audio, const float* video,
                         const float* vnorm_mean, const float* vnorm_std, int64_t N, float* out, void* stream,
                         int mode, uint32_t* host_bits);

/* Range-guard bits (as avse_forward_checked's) raised by the AVSE_F32_SPLIT forwards of plain avse_forward /
 * avse_forward_profile calls on this context since the last avse_range_status; waits for `stream` (the stream those
 * forwards ran on) and clears them. */
int avse_range_status(avse_ctx* ctx, void* stream, uint32_t* host_bits);

/* Stream-ordered, non-blocking form of avse_range_status for pipelines (verify batch k while batch k + 1 runs): enqueues
 * on `stream` a copy of the guard bits raised so far into *host_word (pinned host memory, e.g. hipHostMalloc; valid
 * once the stream has reached this point: record an event after the call and wait for it) and a reset of the guard, so
 * the bits of the forwards enqueued between two snapshots land in the later one.
 *
 * Contract of the three guard readers: the guard words belong to the context.  Unchecked forwards of one context on
 * several streams (or threads) OR into the same word, and avse_forward_checked uses one word per context, so per-batch
 * attribution holds only while ONE stream at a time drives the context; concurrent pipelines each create their own
 * context (they may share the read-only avse_weights). */
int avse_range_snapshot(avse_ctx* ctx, void* stream, uint32_t* host_word);

/* AVSE_F32_SPLIT: the activation exponent e_L of each plan layer (host_exp[0..n), n <= 20; layer L stores the pairs of
 * x 2^e_L); 0 for every layer of the other dtypes. */
int avse_weights_act_exponents(const avse_weights* w, int* host_exp, int n);

/* Stages of the forward pass, in launch order (avse_forward_profile). */
#define AVSE_NUM_STAGES 22
/*  0 video prep (normalise + cast)   1 audio prep      2-6 a_conv1..a_conv5
 *  7-12 v_conv1..v_conv6              13 enc_dense  14 dec_dense1  15 dec_dense2
 *  16-20 d_deconv1..d_deconv5         21 d_deconv6 (1x1 -> float32 output)            */

/* avse_forward with a HIP event recorded between consecutive kernel launches; synchronises the
 * stream and writes each stage's elapsed milliseconds to host_ms[AVSE_NUM_STAGES]. */
int avse_forward_profile(avse_ctx* ctx, const avse_weights* w, const float* audio, const float* video,
                         const float* vnorm_mean, const float* vnorm_std, int64_t N, float* out,
                         void* stream, float* host_ms);

/* VideoNormalizer.normalize (data_processor.py:208-212), in place on device:
 *   video[s, :, :, f] = (video[s, :, :, f] - mean) / std   for video [S][H][W][F]. */
int avse_video_normalize(avse_ctx* ctx, float* video, int64_t S, int H, int W, int F,
                         const float* mean, const float* std, void* stream);

/* SpeechEnhancementNetwork.evaluate's loss (network.py:214-220, Keras mean_squared_error over
 * every element): *loss = mean((pred - target)^2) over n values; loss is a device float. */
int avse_mse(avse_ctx* ctx, const float* pred, const float* target, int64_t n, float* loss,
             void* stream);

/* ---- training (SpeechEnhancementNetwork.train, network.py:177-206) ---------------------- */

/* One Keras fit step of the model compiled at network.py:35-36 (Adam(lr) on mean_squared_error), in float32:
 * BatchNormalization on batch statistics (biased variance, eps 1e-3) with moving-average updates (momentum 0.99; the
 * moving variance takes the BIASED batch variance as Keras 2.0.x does — Keras >= 2.1.3 applies an n / (n - 1)
 * correction there; the reference pins only keras >= 2.0.4 (README), so which one it trained with is unpinned),
 * LeakyReLU(0.3), MaxPooling2D(2, 2), Dropout(dropout_rate) after each video pooling (the reference uses 0.25),
 * MSE over every element, Keras-2.0 Adam (beta1 0.9, beta2 0.999, epsilon 1e-8, bias-corrected step size).
 * Parameters, gradients and Adam moments are kept in the canonical blob layout of avse_weights_load. */
typedef struct avse_trainer avse_trainer;
enum avse_train_buffer { AVSE_TRAIN_PARAMS = 0, AVSE_TRAIN_GRADS = 1, AVSE_TRAIN_ADAM_M = 2, AVSE_TRAIN_ADAM_V = 3,
                         AVSE_TRAIN_DEBUG_DZ = 4 /* test aid: the first n_floats of the dz scratch */ };
/* AVSE_TRAIN_DEBUG_STOP | (layer << 8): test aid, end the backward pass right after layer's BN backward (its
 * dL/dz is then readable with AVSE_TRAIN_DEBUG_DZ; gradients of earlier layers are not computed) */
/* AVSE_TRAIN_DEBUG_GIN | (layer << 8): test aid, end the backward pass after layer's input gradient, copied to the
 * dz scratch */
enum avse_train_flags { AVSE_TRAIN_GRADS_ONLY = 1, AVSE_TRAIN_DEBUG_STOP = 2, AVSE_TRAIN_DEBUG_GIN = 4 };

/* host_blob: initial parameters (avse_weights_load layout); max_batch: largest N passed to avse_trainer_step,
 * 1..1023 (activation tensors stay below 2^31 elements). */
int avse_trainer_create(avse_ctx* ctx, const float* host_blob, int64_t n_floats, int64_t max_batch,
                        avse_trainer** out);
/* avse_trainer_create for the network of build((80, spec_frames), (128, 128, video_frames)) (see
 * avse_weights_blob_floats_shape); avse_trainer_step then takes audio / target [N][80][spec_frames] and video
 * [N][128][128][video_frames]. */
int avse_trainer_create_shape(avse_ctx* ctx, const float* host_blob, int64_t n_floats, int64_t max_batch,
                              int spec_frames, int video_frames, avse_trainer** out);
void avse_trainer_destroy(avse_trainer* t);

/* audio [N][80][20] mixed mel-dB, video [N][128][128][5] raw mouth crops (normalised in-kernel when vnorm_* are
 * given), target [N][80][20] speech mel-dB.  loss: nullable device float (the batch MSE before the update).
 * flags AVSE_TRAIN_GRADS_ONLY: forward (moving statistics updated) + backward, no Adam update.
 * The dropout mask of element e of video layer l is hash(dropout_seed, l, e) >= dropout_rate (train.hip). */
int avse_trainer_step(avse_trainer* t, const float* audio, const float* video, const float* target,
                      const float* vnorm_mean, const float* vnorm_std, int64_t N, float lr, float dropout_rate,
                      uint32_t dropout_seed, int flags, float* loss, void* stream);

/* Copy one of the trainer's blobs (avse_train_buffer) to the host; synchronises the device. */
int avse_trainer_read(avse_trainer* t, int what, float* host_blob, int64_t n_floats);
/* Adam iterations applied so far (Keras `optimizer.iterations`). */
int avse_trainer_iterations(avse_trainer* t, int64_t* iterations);

/* ---- diagnostics ----------------------------------------------------------------------- */

/* Build flags of the loaded library: bit 0 = checked build (make DEBUG=1 -> libavse_debug.so, -DAVSE_DEBUG).  A checked
 * build runs device-side protocol and bounds checks (v_conv1 window-slot tags, STFT sample staging and output bounds,
 * ISTFT chunk frame ranges); avse_spectrogram / avse_istft / avse_forward then synchronise their stream and return
 * AVSE_ERR_CHECK with the first failing check (kernel, check, block, thread, value, expected) in avse_last_error. */
int avse_build_flags(void);

/* Number of forward scratch buffers reported by avse_debug_scratch. */
#define AVSE_DEBUG_NBUF 20

/* Layout of the forward scratch for batch N in compute_dtype, valid after an avse_forward call
 * with that N: *base = device base pointer, offsets[i] = byte offset of buffer i, in launch order:
 *   0 video-in [N][128][128][8]  1 audio-in [N][80][20][8]  2-5 a_conv1..a_conv4
 *   6-10 v_conv1..v_conv5 (pooled)  11 concat [N][5248]  12 enc_dense  13 dec_dense1
 *   14 dec_dense2 [N][5][5][128]  15-19 d_deconv1..d_deconv5          (all NHWC, compute dtype)
 * Test / debugging aid only. */
int avse_debug_scratch(avse_ctx* ctx, int64_t N, int compute_dtype, void** base, int64_t* offsets);

#ifdef __cplusplus
}
#endif
#endif /* AVSE_H */
