// Shared device/host helpers for libavse (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

struct avse_ctx;

namespace avse {

void set_error(const std::string& msg);

// device index of a context (capi.hip; the training step, train.hip, allocates on the same device)
int ctx_device_index(const struct ::avse_ctx* c);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for `fn` on the CURRENT device, once per (kernel, device)
// (thread-safe; capi.hip).  Every launcher that needs more than 64 KB of dynamic LDS calls it first.
int ensure_lds_attr(const void* fn, int bytes);

// Kernel-path switches of one context.  Defaults are the production path; every field exists for an A/B
// experiment or a layer-by-layer parity test.  Initialised once from the AVSE_* environment at
// avse_ctx_create, changed with avse_ctx_set_option; launch code never reads the environment.
struct Options {
    int no_gemm = 0;          // AVSE_NO_GEMM: v_conv6 + dense layers on k_conv + split-K reduce (not k_gemm)
    int no_audenc = 0;        // AVSE_NO_AUDENC: audio encoder layer by layer (not k_aud_enc)
    int no_dechead = 0;       // AVSE_NO_DECHEAD: d_deconv1..3 layer by layer (not k_dec_head)
    int no_dectail = 0;       // AVSE_NO_DECTAIL: d_deconv4..6 layer by layer (not k_dec_tail)
    int unfused_tail = 0;     // AVSE_UNFUSED_TAIL: d_deconv6 as its own kernel (d_deconv5 activation materialised)
    int no_halo = 0;          // AVSE_NO_HALO: video convs on k_conv (read when weights are loaded)
    int mfma32 = 0;           // AVSE_MFMA32: 32x32x16 compute waves in the stream convolutions
    int serial = 0;           // AVSE_SERIAL: one stream for the whole forward
    int graph = 0;            // AVSE_GRAPH: avse_forward replays a hipGraph per argument set
    int gemm_ksplit_cap = 0;  // AVSE_GEMM_KSPLIT: cap k_gemm's split-K factor (0 = no cap)
    int dense_istft = 0;      // AVSE_DENSE_ISTFT: ISTFT through the dense pinv + scratch frames + k_ola (not fused)
    int no_act_scale = 0;     // AVSE_NO_ACT_SCALE: split weights loaded without per-layer activation exponents
    int no_win = 0;           // AVSE_NO_WIN: split stride-1 gather layers on k_conv, not the windowed conv_win.hip
    int no_v1p = 0;           // AVSE_NO_V1P: split 5-frame v_conv1 on k_conv_v1s (K 160), not k_conv_v1p (K 128; read at load)
    int no_a1valu = 0;        // AVSE_NO_A1VALU: split a_conv1 on k_conv after audio_prep, not k_aconv1_split
    int side_prio = 0;        // AVSE_SIDE_PRIO: audio side stream priority (0 default, 1 least, 2 greatest; read when created)
};

#define AVSE_HIP_CHECK(expr)                                                                   \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) {                                                                \
            ::avse::set_error(std::string(#expr " failed: ") + hipGetErrorString(_e));         \
            return 2; /* AVSE_ERR_HIP */                                                       \
        }                                                                                      \
    } while (0)

// ---- checked build (make DEBUG=1 -> libavse_debug.so, -DAVSE_DEBUG) -----------------------
// Device-side protocol / bounds checks that a release build compiles out.  A failing check records the first hit
// (kernel, check code, block, thread, observed and expected value) in its translation unit's record with one vector
// compare-and-swap and the kernel carries on (no trap: a trapped wave can take the whole GPU down); the C-ABI entry
// points synchronise their stream after launching and turn a hit into AVSE_ERR_CHECK with the record in
// avse_last_error (debug_poll, capi.hip).
struct DebugHit {
    unsigned hit, kernel, code, block, thread;
    int value, expect;
};
enum DebugKernel : unsigned {
    DK_V1R = 1,      // k_conv_v1r: window-slot tags (the loader's window k in slot k % 3 when the compute waves read)
    DK_SPEC = 3,     // k_spec_seg / k_spec640: output and LDS index bounds
    DK_ISTFT = 4,    // k_istft_fused: frame range and output bounds
};
#ifdef AVSE_DEBUG
inline constexpr bool kDebugBuild = true;
__device__ __forceinline__ void debug_record(DebugHit* h, unsigned kern, unsigned code, int value, int expect) {
    if (atomicCAS(&h->hit, 0u, 1u) == 0u) {
        h->kernel = kern;
        h->code = code;
        h->block = blockIdx.x;
        h->thread = threadIdx.x;
        h->value = value;
        h->expect = expect;
        __threadfence();
    }
}
// one record per translation unit (no relocatable device code): AVSE_DEBUG_RECORD(name) defines it and the host
// reader `int name(DebugHit* out)` (copy + reset) that debug_poll calls
#define AVSE_DEBUG_RECORD(reader)                                                                    \
    static __device__ ::avse::DebugHit g_avse_dbg;                                                   \
    int reader(::avse::DebugHit* out) {                                                              \
        ::avse::DebugHit zero{};                                                                     \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_avse_dbg), sizeof(zero)) != hipSuccess) return 2;   \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_avse_dbg), &zero, sizeof(zero)) == hipSuccess ? 0 : 2; \
    }
#define AVSE_CHECK_DEV(cond, kern, code, value, expect)                                              \
    do {                                                                                             \
        if (!(cond)) ::avse::debug_record(&g_avse_dbg, (kern), (code), (int)(value), (int)(expect)); \
    } while (0)
#else
inline constexpr bool kDebugBuild = false;
#define AVSE_DEBUG_RECORD(reader)              \
    int reader(::avse::DebugHit* out) {          \
        *out = ::avse::DebugHit{};               \
        return 0;                                \
    }
#define AVSE_CHECK_DEV(cond, kern, code, value, expect) \
    do {                                                 \
    } while (0)
#endif
int debug_read_v1r(DebugHit* out);
int debug_read_stft(DebugHit* out);
int debug_read_istft(DebugHit* out);

// ---- STFT / mel front end ---------------------------------------------------------------
struct MelTable {
    int n_mels = 0;
    int n_bins = 0;
    int max_width = 0;         // max non-zero bins per band
    int* start = nullptr;      // device [n_mels]
    int* width = nullptr;      // device [n_mels]
    float* weight = nullptr;   // device [n_mels][max_width]
    int seg_nq[4] = {6, 6, 6, 6};   // k_spec640: 4-bin weight quads its mel pass j (bands 64 j / 3 ..) needs
    int seg_nq4[4] = {7, 7, 7, 7};  // k_spec_seg: the same from the band start rounded down to a multiple of 4 bins
};

struct SpecArgs {
    const float* sig;
    int64_t n_utt;
    int64_t n_samples;
    int n_fft, hop, n_frames;
    int n_mels;
    float amin, top_db;
    float db_floor;           // 20*log10(amin) evaluated in double (bins <= amin)
    int pad_mode;
    int spf, n_slices;        // frames_per_slice (0 = plain [n_mels][T] layout)
    float* mel_db;
    float* stft_ri;           // nullable
    const float2* twiddle;    // [n_fft]  e^{-2 pi i k / n_fft}
    const float* window;      // [n_fft]  periodic Hann
    const int* mel_start;
    const int* mel_width;
    const float* mel_weight;
    int mel_max_width;
    int mel_seg_nq[4];        // MelTable::seg_nq
    int mel_seg_nq4[4];       // MelTable::seg_nq4
    unsigned int* umax;       // [n_utt] ordered-float max scratch (chunked mode)
};

int launch_spectrogram(const SpecArgs& a, hipStream_t s);

struct IstftArgs {
    const float* mel_db;      // spf > 0: [n_utt][n_slices][n_mels][spf], else [n_utt][n_mels][T]
    int spf, n_slices;
    const float2* stft;       // mixture STFT [n_utt][nb][stft_frames] (phase source)
    int stft_frames;
    int64_t n_utt;
    int T;                    // frames reconstructed
    int nb;                   // bins = 1 + n_fft_analysis / 2
    int N;                    // inverse size = 2 (nb - 1)
    int hop;
    int n_mels;
    const float* pinvT;       // [n_mels][nb] pinv(mel)^T
    const float2* twiddle;    // [N] e^{-2 pi i k / N}
    const float* window;      // [N] periodic Hann
    float* frames;            // scratch [n_utt][T][N] (unfused path only)
    float* sig;               // [n_utt][hop (T - 1)]
    // fused n_fft 640 / hop 160 path: pinv(M) y = M^T (M M^T)^{-1} y with M M^T tridiagonal (adjacent Slaney
    // triangles overlap, nothing else does), so the 321 x 80 dense pinv becomes an 80 x 80 solve + a 2-tap expansion
    const float4* bins;       // [nb] (M[j0][k], M[j0+1][k], j0 as int bits, 0): the <= 2 filters covering bin k
    const float* gram_inv;    // [80][80] (M M^T)^{-1} (symmetric; the fused kernel's MFMA solve), null = Thomas
};

int launch_istft(const IstftArgs& a, hipStream_t s);

// ---- implicit-GEMM convolution ----------------------------------------------------------
constexpr int MAX_TAPS = 25;
constexpr int MAX_PHASES = 4;

struct ConvPhase {
    int py, px;          // output phase offset (deconv); 0 for forward convs
    int ntaps;
    int kpad;            // ntaps * cin padded to the k-slab (multiple of 32)
    long long w_off;     // element offset of this phase's packed weights [cout][kpad]
    int tap_off;         // offset of this phase's (dy, dx) pairs in ConvArgs::taps
};

struct ConvArgs {
    const void* in;      // T [N][Hi][Wi][Ci] (clip stride in_clip_stride)
    void* out;           // T
    const void* w;       // T packed
    const float* scale;  // [Cout]  folded BN scale (or 1)
    const float* shift;  // [Cout]  folded bias/BN shift
    const int2* taps;    // device (dy, dx) per tap, all phases
    int N;
    int Hi, Wi, Ci;
    long long in_clip_stride;
    int Hq, Wq;          // per-phase conv output grid
    int sy, sx;          // input step per grid step
    int oys, oxs;        // output step per grid step (deconv stride)
    int Ho, Wo, Co;      // output tensor (after pool)
    long long out_clip_stride;
    int out_pix_stride;
    int out_c_off;
    int pool;            // fused 2x2 max pool
    int act;             // 1 = LeakyReLU(0.3)
    int nphase;
    int ksplit;          // >1: split-K over blockIdx.z, fp32 partials + k_splitk_reduce (nphase == 1)
    int ksplit_slabs;    // > 0: K slabs (16-k units) per split, else ceil(slabs / ksplit)
    float* partial;      // [ksplit][M][Co] workspace
    // fused trailing 1x1 Cout -> 1 layer (d_deconv6, network.py:133): out_f[pixel] = bias + sum_c w[c] * y[c],
    // y = this layer's output rounded to T; the T output is not stored (Co == 64, ksplit == 1, no pool)
    const float* fuse_w;
    float fuse_bias;
    float* fuse_out;
    int out_s16;         // 1: the output in the split pair layout (strides and offset in halves), else T / fp32
    // AVSE_F32_SPLIT range guard (pair_out_of_range): a stored pair value, or an fp32 input value split on load,
    // outside the f16 range ORs range_bit / range_in_bit into *range_flag (nullable)
    unsigned* range_flag;
    unsigned range_bit, range_in_bit;
    ConvPhase ph[MAX_PHASES];
};

// AVSE_F32_SPLIT range guard: x cannot be carried as the pair h = f16(x), l = f16(x - h) when h would be infinite
// (|x| >= 65520, the f16 overflow threshold under round-to-nearest-even) or x is NaN.  Kernels fold the test over the
// values a lane stores and report once (one vector atomic from the lanes that saw one; the flag word is sticky until
// avse_range_status / avse_forward_checked read it).
__device__ __forceinline__ bool pair_out_of_range(float x) { return !(__builtin_fabsf(x) < 65520.f); }
__device__ __forceinline__ void range_report(unsigned* flag, unsigned bit, bool bad) {
    if (bad && flag) atomicOr(flag, bit);
}
// range flag bits: bit i = layer i of the plan (a_conv1 = 0 .. d_deconv5 = 18), the split network inputs below
constexpr unsigned kRangeAudioIn = 1u << 24, kRangeVideoIn = 1u << 25;
int launch_flag_or(unsigned* flag, unsigned bits, hipStream_t s);

// k_conv's fp32 blocked summation: K-slabs (16 products each) summed FP32_BLOCK at a time into a zeroed partial that
// is added to the running sum in slab order.  A split-K whose every split is exactly one such block, reduced in split
// order, therefore reproduces the unsplit sums bit for bit (train.hip train_split).
constexpr int kFp32Block = 8;
// launch_conv dtype: 0 fp32 (exact-fp32 MFMA), 1 bf16, kConvSplit fp32 input with split-f16 products (the generic
// layers of AVSE_F32_SPLIT: weights packed [Cout][kpad] with each 16-k slab row [Bh(16) | Bl(16)] f16),
// kConvSplitPairs the same on an input already in the split pair layout (Ci, strides, kpad, w_off in halves)
constexpr int kConvSplit = 2, kConvSplitPairs = 3;
int launch_conv(const ConvArgs& a, int dtype, hipStream_t s);

// conv_win.hip: the split-pair layers whose every phase is a stride-1 gather over the input grid (the decoder's
// transposed convolutions, the stride-1 audio conv): k_conv's arithmetic with the A operand read from a per-tile input
// window staged once per 16-channel chunk in LDS (k_conv gathers every tap's im2col rows from global memory).
// htaps: host copy of a.taps.  Returns 0 when launched, -1 when the layer does not fit the kernel (the caller runs
// launch_conv), else an error status.
int launch_conv_win(const ConvArgs& a, const int2* htaps, hipStream_t s);

// fused decoder tail d_deconv4 -> d_deconv5 -> d_deconv6, one workgroup per clip (conv_dec.hip, bf16)
struct DecTailArgs {
    const bf16_t* in;        // d_deconv3 output [N][40][10][128]
    float* out;              // [N][80][20]
    int N;
    const bf16_t* w4;        // d_deconv4 packed [64][kpad4], k = tap * 128 + c
    const float* sc4;        // folded bias + BN
    const float* sh4;
    int nt4, kpad4;
    int pt4, pl4, rows4, pitch4;   // zero-padded input window: top / left pad, rows, pitch (pixels)
    int dy4, dx4, nx4;       // taps: t -> (dy4 - t / nx4, dx4 - t % nx4) (checked on the host)
    const bf16_t* w5;        // d_deconv5 packed, phase p at element w5 + woff5[p]: [64][kpad5[p]], k = tap * 64 + c
    const float* sc5;
    const float* sh5;
    int nt5[4], kpad5[4];
    int dy5[4], dx5[4], nx5[4];    // phase p's taps: t -> (dy5 - t / nx5, dx5 - t % nx5)
    long long woff5[4];
    int pt5, pl5, rows5, pitch5;   // zero-padded d_deconv4 output image
    const float* w6;         // d_deconv6 1x1 weights [64] + bias
    float b6;
    // split-f16 tail (conv_dects.hip, AVSE_F32_SPLIT): in = d_deconv3's split pairs [N][40][10][8 x (h(16) | l(16))],
    // w4 / w5 the layers' split packings ([Cout][2 kpad] halves, each 16-k slab row [Wh(16) | Wl(16)]); d_deconv4's
    // stored pairs report into the range guard
    unsigned* range_flag;
    unsigned range_bit;
};
bool dec_tail_supported(const DecTailArgs& a);
bool dec_tail_s16_supported(const DecTailArgs& a);
int launch_dec_tail_s16(const DecTailArgs& a, hipStream_t s);

// fused audio encoder a_conv1 -> a_conv5, one workgroup per clip (conv_aud.hip, bf16)
struct AudEncArgs {
    const float* mel;        // [N][80][20] network input
    bf16_t* out;             // concat buffer: a_conv5's HWC flatten at [clip * out_clip_stride, + 3200)
    long long out_clip_stride;
    int N;
    const bf16_t* w1;        // a_conv1 dense [64][32], k = ky * 5 + kx (25 real)
    const bf16_t* w2;        // a_conv2 packed [64][1024], k = tap * 64 + c
    const bf16_t* w3;        // a_conv3 packed [128][1024]
    const bf16_t* w4;        // a_conv4 packed [128][512], k = tap * 128 + c
    const bf16_t* w5;        // a_conv5 packed [128][512]
    const float* sc[5];      // folded bias + BN per layer
    const float* sh[5];
};
bool aud_enc_supported(const AudEncArgs& a);

// fused decoder head d_deconv1 -> d_deconv3, one workgroup per clip (conv_dech.hip, bf16)
struct DecHeadArgs {
    const bf16_t* in;        // dec_dense2 output [N][3200] (= [5][5][128])
    long long in_clip_stride;
    bf16_t* out;             // d_deconv3 output [N][40][10][128]
    long long out_clip_stride;
    int N;
    const bf16_t* w1;        // packed per phase [phase][128][kpad], k = tap * 128 + c (kpad 256, 256, 512)
    const bf16_t* w2;
    const bf16_t* w3;
    const float* sc[3];
    const float* sh[3];
};
bool dec_head_supported(const DecHeadArgs& a);
int launch_dec_head(const DecHeadArgs& a, hipStream_t s);

// batched-clip GEMM (gemm.hip, bf16): mode 0 dense rows, mode 1 v_conv6 (3x3 'same' on 4 x 4 x 512 + 2x2 pool)
struct GemmArgs {
    const bf16_t* a;         // mode 0: [M][lda]; mode 1: input [M / 16][4][4][512], clip stride lda
    long long lda;
    const bf16_t* w;         // [N][kpad] (k = tap * 512 + c in mode 1)
    int M, N, kpad;
    const float* scale;      // folded bias + BN
    const float* shift;
    int act;
    bf16_t* out;             // mode 0: out[m * ldo + out_off + n]; mode 1: out[clip * ldo + out_off + q * N + n]
    long long ldo;
    int out_off;
    int ksplit;              // split-K over blockIdx.z, reduced by the last workgroup of each tile
    float* partial;          // [tiles][ksplit][128 x 128] fp32
    int* counters;           // [tiles], zero between launches
    int split;               // 1 = AVSE_F32_SPLIT (k_gemm S16): a / out in the split-pair layout (lda, ldo, out_off in
                             // halves), w packed [Wh(16) | Wl(16)] per 16 k, kpad in k
    int slabs_per_split;     // split: slabs per split (whole kFp32Block blocks; 0 = one split)
    unsigned* range_flag;    // split: range guard of the stored pairs
    unsigned range_bit;
};
int gemm_ksplit(int M, int N, int kpad, int cap);   // cap > 0 limits the split (Options::gemm_ksplit_cap)
int gemm_s16_ksplit(int N, int kpad, int* slabs_per_split);   // split dense layers: plan from K and N only
size_t gemm_ws_bytes(int M, int N, int kpad, int cap);
int launch_gemm(const GemmArgs& g, int mode, hipStream_t s);
int launch_aud_enc(const AudEncArgs& a, hipStream_t s);
int launch_dec_tail(const DecTailArgs& a, hipStream_t s);

// ---- tiled bf16 video convolutions: conv_v1r.hip (v_conv1), conv_stream.hip (v_conv2..v_conv5) ----
enum HaloVariant { HALO_NONE = -1, HALO_V1 = 0, HALO_K5 = 1, HALO_K3_16 = 2, HALO_K3_8 = 3, HALO_V1P = 4 };
// output element format of the tiled video convolutions: bf16; split f16 pairs (per pixel and 16 channels,
// [h(16) | l(16)] with h = f16(x), l = f16(x - h): the next split layer's input); f32
enum HaloOut { OUT_BF16 = 0, OUT_S16 = 1, OUT_F32 = 2 };

struct HaloArgs {
    int variant;
    const void* in;          // bf16 [N][Hc][Wc][Ci]            (not V1)
    const float* video;      // f32  [N][Hc][Wc][5] raw video   (V1)
    const float* vmean;      // nullable [Hc][Wc]               (V1)
    const float* vstd;
    void* out;               // bf16, pooled [N][Hc/2][Wc/2][Co] at (clip stride, pixel stride, channel offset)
    const void* w;           // bf16 [step][Co][32] (V1: [5 kernel rows][Co][32], conv_v1r.hip)
    const float* scale;
    const float* shift;
    int N, Hc, Wc, Ci, Co;
    long long out_clip_stride;
    int out_pix_stride;
    int out_c_off;
    int mfma32;              // conv_stream.hip: 1 = v_mfma_f32_32x32x16_bf16 compute waves (A/B variant)
    int split;               // 1 = split-f16 operands (AVSE_F32_SPLIT): in is the split-pair layout, Ci counts halves
                             // (2 x channels), w holds [Bh | Bl] rows; out_mode OUT_S16 or OUT_F32
    int out_mode;            // HaloOut
    unsigned long long* prof;   // ablation harness only (ABL & 128): per-wave cycle counters, else unused
    unsigned* range_flag;    // split: range guard (ConvArgs::range_flag), nullable
    unsigned range_bit, range_in_bit;   // OUT_S16 stores / v_conv1's split of the (normalised) video input
};

int launch_conv_stream(const HaloArgs& a, hipStream_t s);   // conv_stream.hip (non-V1 variants)
int launch_conv_v1r(const HaloArgs& a, hipStream_t s);      // conv_v1r.hip (v_conv1, kernel-row runs)
int launch_video_prep(const float* video, const float* mean, const float* stdv, void* out, int64_t N,
                      int F, int dtype, hipStream_t s);
int launch_audio_prep(const float* audio, void* out, int64_t npix, int dtype, hipStream_t s);
// split dtype a_conv1 (one input channel) on the vector ALUs straight from the audio input (conv.hip k_aconv1_split)
int launch_aconv1_split(const float* in, const float* w, const float* scale, const float* shift, void* out, int64_t N,
                        int H, int W, int Ho, int Wo, int KH, int KW, int S, int pt, int pl, int Co, unsigned* range_flag,
                        unsigned range_bit, unsigned range_in_bit, hipStream_t s);
int launch_out_conv(const void* in, const float* w64, float bias, float* out, int64_t npix, int dtype,
                    hipStream_t s);
int launch_broadcast_row(const void* src, void* dst, int64_t rows, int64_t row_bytes, int64_t stride_bytes,
                         hipStream_t s);
int launch_video_normalize(float* video, int64_t S, int H, int W, int F, const float* mean,
                           const float* stdv, hipStream_t s);
int launch_mse(const float* a, const float* b, int64_t n, float* loss, float* partial, hipStream_t s);

}  // namespace avse
