// libavse C-ABI (include/avse.h): contexts, librosa-equivalent tables, weight folding/packing and
// the layer plan of /root/reference/network.py, executed as a sequence of HIP kernel launches on
// the caller's stream.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/avse.h"
#include "avse_common.h"
#include "netplan.h"

namespace avse {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

int ensure_lds_attr(const void* fn, int bytes) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;   // (kernel, device)
    int dev = 0;
    AVSE_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({fn, dev})) return 0;
    AVSE_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.insert({fn, dev});
    return 0;
}
}  // namespace avse

using namespace avse;

namespace {

int fail(int code, const std::string& msg) {
    set_error(msg);
    return code;
}

// ---------------------------------------------------------------------------------------------
// librosa-equivalent host tables (double precision, rounded to float once)
// ---------------------------------------------------------------------------------------------
double hz_to_mel(double f) {  // Slaney (htk=False)
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
    const double logstep = std::log(6.4) / 27.0;
    if (f >= min_log_hz) return min_log_mel + std::log(f / min_log_hz) / logstep;
    return f / f_sp;
}
double mel_to_hz(double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
    const double logstep = std::log(6.4) / 27.0;
    if (m >= min_log_mel) return min_log_hz * std::exp(logstep * (m - min_log_mel));
    return f_sp * m;
}

// librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm=1) -> [n_mels][n_bins] (double)
std::vector<double> mel_filterbank(int sr, int n_fft, int n_mels, double fmin, double fmax) {
    const int nb = 1 + n_fft / 2;
    std::vector<double> w((size_t)n_mels * nb, 0.0);
    std::vector<double> fftf(nb), melf(n_mels + 2);
    for (int k = 0; k < nb; ++k) fftf[k] = (nb == 1) ? 0.0 : (double)k * ((double)sr / 2) / (double)(nb - 1);
    const double lo = hz_to_mel(fmin), hi = hz_to_mel(fmax);
    for (int i = 0; i < n_mels + 2; ++i) melf[i] = mel_to_hz(lo + (hi - lo) * (double)i / (double)(n_mels + 1));
    for (int i = 0; i < n_mels; ++i) {
        const double d0 = melf[i + 1] - melf[i], d1 = melf[i + 2] - melf[i + 1];
        const double enorm = 2.0 / (melf[i + 2] - melf[i]);
        for (int k = 0; k < nb; ++k) {
            const double lower = -(melf[i] - fftf[k]) / d0;
            const double upper = (melf[i + 2] - fftf[k]) / d1;
            double v = std::fmin(lower, upper);
            if (v < 0) v = 0;
            w[(size_t)i * nb + k] = v * enorm;
        }
    }
    return w;
}

struct SpecTables {
    int sr = -1, n_fft = -1, n_mels = -1;
    double fmin = 0, fmax = 0;
    float2* twiddle = nullptr;
    float* window = nullptr;
    MelTable mel;
};

// ---------------------------------------------------------------------------------------------
// network plan (network.py:17-175)
// ---------------------------------------------------------------------------------------------
uint16_t f2h(float f) {   // f32 -> f16 bits, round to nearest even (hipcc's host _Float16 conversion)
    const _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}
float h2f(uint16_t u) {
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (float)h;
}

uint16_t f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

}  // namespace

struct IstftTables {
    int sr = -1, n_fft = -1, n_mels = -1;
    double fmin = 0, fmax = 0;
    float* pinvT = nullptr;     // [n_mels][nb]
    float2* twiddle = nullptr;  // [N]
    float* window = nullptr;    // [N]
    float4* bins = nullptr;     // [nb] the <= 2 adjacent filters covering each bin
    float* gram_inv = nullptr;  // [n_mels][n_mels] (M M^T)^{-1} in float (n_mels == 80 only)
};

struct avse_ctx {
    int device = 0;
    Options opt;                // kernel-path switches (read from AVSE_* once, at creation)
    SpecTables spec;
    IstftTables istft;
    float* frames = nullptr;    // ISTFT frame scratch
    size_t frames_bytes = 0;
    unsigned* umax = nullptr;
    int64_t umax_cap = 0;
    float* mse_partial = nullptr;
    float* zero_video = nullptr;    // one all-zero [128][128][8] clip (video == NULL forwards, any F <= 8)
    int* gemm_counters = nullptr;   // gemm.hip split-K tickets (zero between launches)
    // AVSE_F32_SPLIT range guard words (avse_common.h pair_out_of_range): [0] sticky for avse_forward (read and cleared
    // by avse_range_status), [1] cleared and read by each avse_forward_checked, [2] the all-zero-video embedding
    unsigned* range = nullptr;
    unsigned* range_host = nullptr;   // pinned readback word
    char* arena = nullptr;
    size_t arena_bytes = 0;
    NetPlan last_plan = kPlan25;    // the network shape of the last forward (avse_debug_scratch's arena layout)
    // side stream for the audio branch of the forward (runs concurrently with the video encoder)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // avse_forward's replay cache: the whole forward captured once per argument set into a hipGraph
    struct Graph {
        const void* key[9];
        int64_t n;
        Options opt;
        hipGraphExec_t exec;
    };
    std::vector<Graph> graphs;
    hipStream_t cap = nullptr;   // capture stream
};

namespace avse {
int ctx_device_index(const avse_ctx* c) { return c->device; }
}  // namespace avse

struct GpuLayer {
    LayerDef def;
    int cin_pad = 0;
    int hq = 0, wq = 0, ho = 0, wo = 0;
    int nphase = 1;
    ConvPhase ph[MAX_PHASES];
    void* w = nullptr;
    float* scale = nullptr;
    float* shift = nullptr;
    int2* taps = nullptr;
    int halo = HALO_NONE;     // halo-tiled kernel variant (bf16 video convs)
    void* w_halo = nullptr;   // bf16 packing for conv_stream.hip / conv_v1r.hip (see build_layer)
    void* w_dense = nullptr;  // a_conv1 only (bf16): [Cout][32], k = ky * kw + kx, for conv_aud.hip
    float* w_f32 = nullptr;   // a_conv1 only (split): [kh * kw][Cout] f32 x 2^e_n, for conv.hip k_aconv1_split
    float* scale_h = nullptr; // |scale| for w_halo: channels with a negative BN scale have negated weights
    int2 htaps[MAX_TAPS * MAX_PHASES] = {};   // host copy of taps (conv_dec.hip's kernel arguments)
};

// avse_ctx_set_option names (and the AVSE_* variables that initialise them at avse_ctx_create)
struct OptionName {
    const char* name;
    const char* env;
    int Options::*field;
};
const OptionName kOptionNames[] = {
    {"no_gemm", "AVSE_NO_GEMM", &Options::no_gemm},
    {"no_audenc", "AVSE_NO_AUDENC", &Options::no_audenc},
    {"no_dechead", "AVSE_NO_DECHEAD", &Options::no_dechead},
    {"no_dectail", "AVSE_NO_DECTAIL", &Options::no_dectail},
    {"unfused_tail", "AVSE_UNFUSED_TAIL", &Options::unfused_tail},
    {"no_halo", "AVSE_NO_HALO", &Options::no_halo},
    {"mfma32", "AVSE_MFMA32", &Options::mfma32},
    {"serial", "AVSE_SERIAL", &Options::serial},
    {"graph", "AVSE_GRAPH", &Options::graph},
    {"gemm_ksplit_cap", "AVSE_GEMM_KSPLIT", &Options::gemm_ksplit_cap},
    {"dense_istft", "AVSE_DENSE_ISTFT", &Options::dense_istft},
    {"no_act_scale", "AVSE_NO_ACT_SCALE", &Options::no_act_scale},
    {"no_win", "AVSE_NO_WIN", &Options::no_win},
    {"no_v1p", "AVSE_NO_V1P", &Options::no_v1p},
    {"no_a1valu", "AVSE_NO_A1VALU", &Options::no_a1valu},
    {"side_prio", "AVSE_SIDE_PRIO", &Options::side_prio},
};

struct avse_weights {
    int dtype = 0;
    int device = 0;
    uint64_t serial = 0;                // unique per created weights object (graph-cache key: addresses get reused)
    NetPlan plan = kPlan25;             // the network shape these weights were built for (netplan.h)
    GpuLayer layers[kNumLayers - 1];  // all but d_deconv6
    float* d6_w = nullptr;
    float d6_bias = 0.f;
    // avse_forward with video == NULL (all-zero video input, BASELINE configs[2]): the video encoder's output is
    // then the same 2048-vector for every clip — computed once on first use and broadcast into the concat rows.
    // Published only after its stream has finished (another stream / thread may read it right away), under a lock.
    mutable std::atomic<void*> vzero_emb{nullptr};
    mutable std::mutex vzero_mu;
    mutable unsigned vzero_range = 0;   // split: range-guard bits the embedding's computation raised (sticky per forward)
    // AVSE_F32_SPLIT: per-layer power-of-two activation exponents (act_exponents: layer i stores the pairs of
    // x 2^act_exp[i]), the canonical blob (host copy) and, built from it on the first range-guard hit, the same network
    // on exact-fp32 MFMA that avse_forward_checked recomputes such a batch on
    int act_exp[kNumLayers] = {};
    std::vector<float> blob;
    mutable avse_weights* f32_twin = nullptr;
    mutable std::mutex twin_mu;
    std::vector<void*> allocs;
    ~avse_weights();
};

avse_weights::~avse_weights() {
    delete f32_twin;
    (void)hipFree(vzero_emb.load());
    for (void* p : allocs) (void)hipFree(p);
}

namespace {

template <typename T>
int upload(avse_weights* W, const std::vector<T>& h, T** out) {
    void* p = nullptr;
    if (hipMalloc(&p, sizeof(T) * (h.empty() ? 1 : h.size())) != hipSuccess) return fail(AVSE_ERR_OOM, "hipMalloc failed (weights)");
    W->allocs.push_back(p);
    if (!h.empty() && hipMemcpy(p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(AVSE_ERR_HIP, "hipMemcpy failed (weights)");
    *out = (T*)p;
    return 0;
}

// per-clip activation sizes (elements) of the forward scratch, in launch order
struct Arena {
    size_t off[32];
    size_t per_clip_bytes;
};
enum Buf { B_VIN, B_AIN, B_A1, B_A2, B_A3, B_A4, B_V1, B_V2, B_V3, B_V4, B_V5, B_CAT, B_E1, B_E2, B_E3,
           B_D1, B_D2, B_D3, B_D4, B_D5, B_COUNT };
size_t buf_elems(const NetPlan& p, int b) {
    const size_t T = p.T, w1 = (T + 1) / 2, w3 = p.W5;
    const size_t e[B_COUNT] = {128 * 128 * 8, 80 * T * 8, 40 * w1 * 64, 40 * w1 * 64, 20 * w3 * 128,
                               10 * w3 * 128, 64 * 64 * 128, 32 * 32 * 128, 16 * 16 * 256, 8 * 8 * 256,
                               4 * 4 * 512, (size_t)p.cat, (size_t)p.emb, (size_t)p.emb, (size_t)p.aemb,
                               10 * w3 * 128, 20 * w3 * 128, 40 * 2 * w3 * 128, 40 * 2 * w3 * 64, 80 * 4 * w3 * 64};
    return e[b];
}

// Split-K plan for a single-phase GEMM of M rows x Co columns x kpad on k_conv.
//  bf16: double the split while the grid stays <= ~1024 workgroups and every split keeps >= 16 k-slabs.
//  fp32 (AVSE_F32, and the generic layers of AVSE_F32_SPLIT): block-exact, as the training step's train_split —
//  every split is exactly one block of k_conv's blocked fp32 summation (kFp32Block 16-product slabs) and
//  k_splitk_reduce_tiles adds the splits in order, so each sum is the unsplit kernel's bit for bit.  Whether a launch
//  splits (short grids only) then changes no result: the fp32 forward of a clip is the same whatever batch it runs
//  in (the batched CLI predict reproduces the per-sample one exactly; tests/test_gpu_split.py).
//  AVSE_F32_SPLIT dense layers (one tap): groups of G blocks per split, G and the split count from K and Cout only
//  (never from M), so every batch size takes the same splits and the same ordered reduction — batch-invariant as
//  above, with G x fewer fp32 partials (enc_dense: 41 one-block splits moved 236 MB of partials per launch at B = 512;
//  11 four-block splits move 64 MB).  slabs_per_split (k_conv's ConvArgs::ksplit_slabs) = 8 G.
constexpr int64_t kSplitTileCap = 2048;   // fp32 tiles x splits per launch (128 x 128-float partials each)
int choose_ksplit(int64_t M, int Co, int kpad, int dtype, bool dense = false, int* slabs_per_split = nullptr) {
    const int BN = Co <= 64 ? 64 : 128;
    const int64_t tiles = ((M + 127) / 128) * ((Co + BN - 1) / BN);
    if (slabs_per_split) *slabs_per_split = 0;
    if (dtype == AVSE_F32_SPLIT && dense) {
        const int nblocks = (kpad / 16 + kFp32Block - 1) / kFp32Block, tiles_n = (Co + 127) / 128;
        const int G = std::max(1, (nblocks * tiles_n + 127) / 128);
        const int ks = (nblocks + G - 1) / G;
        if (ks < 2) return 1;
        if (slabs_per_split) *slabs_per_split = G * kFp32Block;
        return ks;
    }
    if (dtype != AVSE_BF16) {
        const int nslab = kpad / 16;
        const int ks = (nslab + kFp32Block - 1) / kFp32Block;
        if (tiles >= 256 || ks < 2 || (nslab + ks - 1) / ks != kFp32Block || tiles * ks > kSplitTileCap) return 1;
        return ks;
    }
    const int nslab = kpad / 32;
    int ks = 1;
    while (tiles * ks * 2 <= 1024 && nslab / (ks * 2) >= 16) ks *= 2;
    return ks;
}

// fp32 partial-sum workspace needed by the split-K layers (enc/dec dense, v_conv6) at batch N
size_t split_ws_bytes(int64_t N, int dtype, const Options& o, const NetPlan& p) {
    const struct { int64_t M; int Co, kpad; } g[4] = {{N, p.emb, (p.cat + 31) / 32 * 32}, {N, p.emb, (p.emb + 31) / 32 * 32},
                                                      {N, p.aemb, (p.emb + 31) / 32 * 32}, {N * 16, 512, 4608}};
    size_t mx = 0;
    for (const auto& x : g) {
        const int ks = choose_ksplit(x.M, x.Co, x.kpad, dtype, &x != &g[3]);
        // k_conv's partials cover whole 128 x BN tiles (MFMA-native order)
        const int bn = x.Co <= 64 ? 64 : 128;
        const size_t mp = (size_t)((x.M + 127) / 128) * 128, np = (size_t)((x.Co + bn - 1) / bn) * bn;
        if (ks > 1) mx = std::max(mx, (size_t)ks * mp * np * 4);
        if (dtype == AVSE_BF16) mx = std::max(mx, gemm_ws_bytes((int)x.M, x.Co, x.kpad, o.gemm_ksplit_cap));   // gemm.hip's split-K
        if (dtype == AVSE_F32_SPLIT && &x != &g[3]) {   // gemm.hip's split dense plan (v_conv6 takes k_conv's, above)
            const int gks = gemm_s16_ksplit(x.Co, x.kpad, nullptr);
            if (gks > 1) mx = std::max(mx, (size_t)((x.M + 127) / 128) * ((x.Co + 127) / 128) * gks * 128 * 128 * 4);
        }
    }
    return mx;
}

size_t arena_bytes(int64_t clips, int dtype, const Options& o, size_t* offs, const NetPlan& p) {
    const size_t es = dtype == AVSE_BF16 ? 2 : 4;
    size_t off = 0;
    for (int b = 0; b < B_COUNT; ++b) {
        if (offs) offs[b] = off;
        off += (buf_elems(p, b) * es * (size_t)clips + 255) & ~(size_t)255;
    }
    if (offs) offs[B_COUNT] = off;   // split-K partials
    off += (split_ws_bytes(clips, dtype, o, p) + 255) & ~(size_t)255;
    return off;
}

bool valid_dtype(int dtype) { return dtype == AVSE_F32 || dtype == AVSE_BF16 || dtype == AVSE_F32_SPLIT; }

// grows the forward scratch; never while `s` (nullable) is being captured into a graph: the caller must reserve first
int ensure_arena(avse_ctx* c, int64_t clips, int dtype, const NetPlan& p, hipStream_t s) {
    // at least the N = 1 layout: a video == NULL forward runs a one-clip video encoder (and its split-K) in it
    const size_t need = std::max(arena_bytes(clips, dtype, c->opt, nullptr, p), arena_bytes(1, dtype, c->opt, nullptr, p));
    if (need <= c->arena_bytes) return 0;
    if (s) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        AVSE_HIP_CHECK(hipStreamIsCapturing(s, &cs));
        if (cs != hipStreamCaptureStatusNone)
            return fail(AVSE_ERR_INVALID, "the forward scratch would grow while the stream is being captured: call "
                                          "avse_ctx_reserve_weights(ctx, weights, max_clips) before the capture");
    }
    if (c->arena) (void)hipFree(c->arena);
    c->arena = nullptr;
    c->arena_bytes = 0;
    if (hipMalloc((void**)&c->arena, need) != hipSuccess) return fail(AVSE_ERR_OOM, "hipMalloc failed (forward scratch)");
    c->arena_bytes = need;
    return 0;
}

int ensure_spec_tables(avse_ctx* c, int sr, int n_fft, int n_mels, double fmin, double fmax) {
    SpecTables& t = c->spec;
    if (t.sr == sr && t.n_fft == n_fft && t.n_mels == n_mels && t.fmin == fmin && t.fmax == fmax) return 0;
    (void)hipFree(t.twiddle); (void)hipFree(t.window); (void)hipFree(t.mel.start); (void)hipFree(t.mel.width); (void)hipFree(t.mel.weight);
    t = SpecTables();
    std::vector<float2> tw(n_fft);
    std::vector<float> win(n_fft);
    for (int k = 0; k < n_fft; ++k) {
        const double ang = -2.0 * M_PI * (double)k / (double)n_fft;
        tw[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
        win[k] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * (double)k / (double)n_fft));
    }
    const int nb = 1 + n_fft / 2;
    std::vector<double> fb = mel_filterbank(sr, n_fft, n_mels, fmin, fmax);
    std::vector<int> st(n_mels), wd(n_mels);
    int maxw = 1;
    for (int m = 0; m < n_mels; ++m) {
        int lo = -1, hi = -1;
        for (int k = 0; k < nb; ++k)
            if (fb[(size_t)m * nb + k] > 0) { if (lo < 0) lo = k; hi = k; }
        // bands start at an even bin (a leading zero weight when the first non-zero bin is odd): the STFT kernels
        // read a band's magnitudes as 8-B pairs (half the LDS instructions and bank-conflict cycles of 4-B reads)
        lo = lo < 0 ? -1 : (lo & ~1);
        st[m] = lo < 0 ? 0 : lo;
        wd[m] = lo < 0 ? 0 : hi - lo + 1;
        if (wd[m] > maxw) maxw = wd[m];
    }
    if (maxw <= 24) maxw = 24;   // rows padded to the STFT kernel's compile-time band width (16-B staging copies)
    std::vector<float> wt((size_t)n_mels * maxw, 0.f);
    for (int m = 0; m < n_mels; ++m)
        for (int j = 0; j < wd[m]; ++j) wt[(size_t)m * maxw + j] = (float)fb[(size_t)m * nb + st[m] + j];
    AVSE_HIP_CHECK(hipMalloc(&t.twiddle, sizeof(float2) * n_fft));
    AVSE_HIP_CHECK(hipMalloc(&t.window, sizeof(float) * n_fft));
    AVSE_HIP_CHECK(hipMalloc(&t.mel.start, sizeof(int) * n_mels));
    AVSE_HIP_CHECK(hipMalloc(&t.mel.width, sizeof(int) * n_mels));
    AVSE_HIP_CHECK(hipMalloc(&t.mel.weight, sizeof(float) * wt.size()));
    AVSE_HIP_CHECK(hipMemcpy(t.twiddle, tw.data(), sizeof(float2) * n_fft, hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.window, win.data(), sizeof(float) * n_fft, hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.mel.start, st.data(), sizeof(int) * n_mels, hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.mel.width, wd.data(), sizeof(int) * n_mels, hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.mel.weight, wt.data(), sizeof(float) * wt.size(), hipMemcpyHostToDevice));
    t.sr = sr; t.n_fft = n_fft; t.n_mels = n_mels; t.fmin = fmin; t.fmax = fmax;
    // k_spec_seg's mel pass j covers items 64 j .. 64 j + 63 = bands (item / 3): the widest of those bands (aligned
    // start) in 4-bin quads; the rows stay padded to maxw, so a pass reads only the quads its bands can use
    for (int j = 0; j < 4; ++j) {
        int w = 0;
        for (int it = 64 * j; it < 64 * j + 64 && it / 3 < n_mels; ++it) w = std::max(w, wd[it / 3]);
        t.mel.seg_nq[j] = std::min((w + 3) / 4, maxw / 4);
        // k_spec_seg reads 16-B quads from 4-aligned band starts (st & ~3: a further 0 or 2 leading zero weights)
        int w4 = 0;
        for (int it = 64 * j; it < 64 * j + 64 && it / 3 < n_mels; ++it) w4 = std::max(w4, (st[it / 3] & 3) + wd[it / 3]);
        t.mel.seg_nq4[j] = std::min((w4 + 3) / 4, (maxw + 4) / 4);
    }
    t.mel.n_mels = n_mels; t.mel.n_bins = nb; t.mel.max_width = maxw;
    return 0;
}

// pinv(mel) = M^T (M M^T)^{-1} in double (M is full row rank, cond ~4.5 for the reference's
// filterbanks; equal to np.linalg.pinv's SVD form to ~1e-13), plus the inverse-DFT tables.
int ensure_istft_tables(avse_ctx* c, int sr, int n_fft, int n_mels, double fmin, double fmax) {
    IstftTables& t = c->istft;
    if (t.sr == sr && t.n_fft == n_fft && t.n_mels == n_mels && t.fmin == fmin && t.fmax == fmax) return 0;
    (void)hipFree(t.pinvT); (void)hipFree(t.twiddle); (void)hipFree(t.window);
    (void)hipFree(t.bins); (void)hipFree(t.gram_inv);
    t = IstftTables();
    const int nb = 1 + n_fft / 2, N = 2 * (nb - 1);
    const std::vector<double> M = mel_filterbank(sr, n_fft, n_mels, fmin, fmax);
    // G = M M^T, then Gauss-Jordan inverse with partial pivoting
    std::vector<double> G((size_t)n_mels * n_mels), Gi((size_t)n_mels * n_mels, 0.0);
    for (int i = 0; i < n_mels; ++i)
        for (int j = 0; j < n_mels; ++j) {
            double s = 0;
            for (int k = 0; k < nb; ++k) s += M[(size_t)i * nb + k] * M[(size_t)j * nb + k];
            G[(size_t)i * n_mels + j] = s;
        }
    for (int i = 0; i < n_mels; ++i) Gi[(size_t)i * n_mels + i] = 1.0;
    for (int col = 0; col < n_mels; ++col) {
        int piv = col;
        for (int r = col + 1; r < n_mels; ++r)
            if (std::fabs(G[(size_t)r * n_mels + col]) > std::fabs(G[(size_t)piv * n_mels + col])) piv = r;
        if (std::fabs(G[(size_t)piv * n_mels + col]) < 1e-300) return fail(AVSE_ERR_UNSUPPORTED, "mel filterbank is rank deficient");
        if (piv != col)
            for (int j = 0; j < n_mels; ++j) {
                std::swap(G[(size_t)piv * n_mels + j], G[(size_t)col * n_mels + j]);
                std::swap(Gi[(size_t)piv * n_mels + j], Gi[(size_t)col * n_mels + j]);
            }
        const double d = G[(size_t)col * n_mels + col];
        for (int j = 0; j < n_mels; ++j) { G[(size_t)col * n_mels + j] /= d; Gi[(size_t)col * n_mels + j] /= d; }
        for (int r = 0; r < n_mels; ++r) {
            if (r == col) continue;
            const double f = G[(size_t)r * n_mels + col];
            if (f == 0) continue;
            for (int j = 0; j < n_mels; ++j) {
                G[(size_t)r * n_mels + j] -= f * G[(size_t)col * n_mels + j];
                Gi[(size_t)r * n_mels + j] -= f * Gi[(size_t)col * n_mels + j];
            }
        }
    }
    // pinv[k][m] = sum_j M[j][k] Gi[j][m]; stored transposed [m][k]
    std::vector<float> pinvT((size_t)n_mels * nb);
    for (int m = 0; m < n_mels; ++m)
        for (int k = 0; k < nb; ++k) {
            double s = 0;
            for (int j = 0; j < n_mels; ++j) s += M[(size_t)j * nb + k] * Gi[(size_t)j * n_mels + m];
            pinvT[(size_t)m * nb + k] = (float)s;
        }
    std::vector<float2> tw(N);
    std::vector<float> win(N);
    for (int k = 0; k < N; ++k) {
        const double ang = -2.0 * M_PI * (double)k / (double)N;
        tw[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
        win[k] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * (double)k / (double)N));
    }
    AVSE_HIP_CHECK(hipMalloc(&t.pinvT, sizeof(float) * pinvT.size()));
    AVSE_HIP_CHECK(hipMalloc(&t.twiddle, sizeof(float2) * N));
    AVSE_HIP_CHECK(hipMalloc(&t.window, sizeof(float) * N));
    AVSE_HIP_CHECK(hipMemcpy(t.pinvT, pinvT.data(), sizeof(float) * pinvT.size(), hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.twiddle, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice));
    AVSE_HIP_CHECK(hipMemcpy(t.window, win.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    // Tridiagonal form for the fused kernel: every bin covered by at most two filters j0, j0 + 1 => M M^T
    // has no entry beyond the first off-diagonals, and pinv(M) a = M^T y with (M M^T) y = a (Thomas, no
    // pivoting: the Gram matrix is symmetric positive definite).  Recomputed in double from G (Gi above
    // overwrote its working copy).
    {
        bool ok = true;
        std::vector<float4> bins(nb);
        for (int k = 0; k < nb && ok; ++k) {
            int j0 = -1, cnt = 0;
            for (int j = 0; j < n_mels; ++j)
                if (M[(size_t)j * nb + k] != 0.0) {
                    if (j0 < 0) j0 = j;
                    else if (j != j0 + 1) ok = false;
                    ++cnt;
                }
            if (cnt > 2) ok = false;
            const float w0 = j0 >= 0 ? (float)M[(size_t)j0 * nb + k] : 0.f;
            const float w1 = (j0 >= 0 && j0 + 1 < n_mels) ? (float)M[(size_t)(j0 + 1) * nb + k] : 0.f;
            int j0b = j0;
            float j0f;
            std::memcpy(&j0f, &j0b, 4);
            bins[k] = make_float4(w0, w1, j0f, 0.f);
        }
        if (ok) {
            auto gram = [&](int i, int j) {
                double acc = 0;
                for (int k = 0; k < nb; ++k) acc += M[(size_t)i * nb + k] * M[(size_t)j * nb + k];
                return acc;
            };
            // M M^T must be tridiagonal (adjacent Slaney triangles overlap, nothing else does) and its LU pivots
            // non-zero: the checks that make M^T (M M^T)^{-1} = pinv(M) computable from the band-local pieces
            double cprev = 0;
            for (int i = 0; i < n_mels && ok; ++i) {
                for (int j = 0; j < i - 1 && ok; ++j)
                    if (gram(i, j) != 0.0) ok = false;
                const double ai = i > 0 ? gram(i, i - 1) : 0.0, bi = gram(i, i);
                const double ci = i + 1 < n_mels ? gram(i, i + 1) : 0.0;
                const double piv = bi - ai * cprev;
                if (!(std::fabs(piv) > 1e-300)) { ok = false; break; }
                cprev = ci / piv;
            }
            if (ok) {
                AVSE_HIP_CHECK(hipMalloc(&t.bins, sizeof(float4) * nb));
                AVSE_HIP_CHECK(hipMemcpy(t.bins, bins.data(), sizeof(float4) * nb, hipMemcpyHostToDevice));
                if (n_mels == 80) {
                    // (M M^T)^{-1} by Gauss-Jordan in double (the Gram matrix is symmetric positive definite, cond ~20):
                    // the fused kernel solves all frames of a chunk at once as a [frames x 80] x [80 x 80] fp32 MFMA
                    // product (round 2: one Thomas recurrence per frame and lane)
                    const int n = n_mels;
                    std::vector<double> g((size_t)n * n), inv((size_t)n * n, 0.0);
                    for (int i = 0; i < n; ++i) {
                        inv[(size_t)i * n + i] = 1.0;
                        for (int j = std::max(0, i - 1); j <= std::min(n - 1, i + 1); ++j) g[(size_t)i * n + j] = gram(i, j);
                    }
                    for (int c = 0; c < n && ok; ++c) {
                        const double piv = g[(size_t)c * n + c];
                        if (!(std::fabs(piv) > 1e-300)) { ok = false; break; }
                        for (int j = 0; j < n; ++j) { g[(size_t)c * n + j] /= piv; inv[(size_t)c * n + j] /= piv; }
                        for (int r = 0; r < n; ++r) {
                            if (r == c) continue;
                            const double f = g[(size_t)r * n + c];
                            if (f == 0.0) continue;
                            for (int j = 0; j < n; ++j) {
                                g[(size_t)r * n + j] -= f * g[(size_t)c * n + j];
                                inv[(size_t)r * n + j] -= f * inv[(size_t)c * n + j];
                            }
                        }
                    }
                    if (ok) {
                        std::vector<float> fi(inv.begin(), inv.end());
                        AVSE_HIP_CHECK(hipMalloc(&t.gram_inv, sizeof(float) * n * n));
                        AVSE_HIP_CHECK(hipMemcpy(t.gram_inv, fi.data(), sizeof(float) * n * n, hipMemcpyHostToDevice));
                    }
                }
            }
        }
    }
    t.sr = sr; t.n_fft = n_fft; t.n_mels = n_mels; t.fmin = fmin; t.fmax = fmax;
    return 0;
}

// AVSE_F32_SPLIT activation exponents.  The split layers carry activations as f16 pairs, whose ~22 significant bits
// hold for |x| in [2^-3, 65504): below 2^-3 the lo piece is an f16 subnormal (absolute quantum 2^-24), from 65520 the
// hi piece overflows (the range guard then reports it).  A BatchNormalization layer's output per channel is
// gamma xhat + beta with xhat standardised by the moving statistics, so the layer's magnitude is ~ M = max_c (|beta_c| +
// |gamma_c|).  Layers with M in [2^-2, 2^8] keep exponent 0 (the common case: BN keeps activations O(1), and every
// stored value is then exactly the unscaled pair); any other layer stores the pairs of x 2^e with M 2^e in (4, 8], so a
// layer of tiny activations keeps its 22 bits and a layer of huge ones its headroom below 65504 (folded into the
// layer's own scale / shift and the next layer's scale, build_layer).  The two concat halves (a_conv5, v_conv6) share
// one exponent, the smaller (enc_dense reads them as one K); d_deconv5 feeds the fp32 d_deconv6 dot (exponent 0).
void act_exponents(const NetPlan& P, const float* blob, int* e) {
    const float* p = blob;
    for (int i = 0; i < kNumLayers; ++i) {
        const LayerDef& L = P.L[i];
        p += (size_t)L.kh * L.kw * L.cin * L.cout + L.cout;
        e[i] = 0;
        if (!L.bn) continue;
        const float* g = p;
        const float* b = p + L.bn_channels;
        p += 4 * (size_t)L.bn_channels;
        double m = 0.0;
        for (int c = 0; c < L.bn_channels; ++c) m = std::max(m, std::fabs((double)b[c]) + std::fabs((double)g[c]));
        if (!(m > 0.0) || !std::isfinite(m) || (m >= 0.25 && m <= 256.0)) continue;
        int e2 = 0;
        (void)std::frexp(m, &e2);                      // m <= 2^e2
        e[i] = std::max(-24, std::min(24, 3 - e2));    // m 2^e in (4, 8]
    }
    e[4] = e[10] = std::min(e[4], e[10]);
    e[18] = e[19] = 0;
}

// the exponent of the activations layer i reads (act_exponents; the network inputs: 0)
int act_exp_in(const int* e, int i) {
    if (i == 0 || i == 5) return 0;
    if (i == 11) return e[4];
    return e[i - 1];
}

// Build phase/tap tables + packed [Cout][Kpad] weights for one layer.
int build_layer(avse_weights* W, int li, const float* kernel, const float* bias, const float* bn,
                const Options& opt, int e_in = 0, int e_out = 0) {
    const LayerDef& L = W->plan.L[li];
    GpuLayer& G = W->layers[li];
    G.def = L;
    const int CHUNK_ELEMS = 8;   // channel padding so a 16-B chunk never straddles a tap (bf16: 8)
    G.cin_pad = (L.cin % CHUNK_ELEMS) ? ((L.cin + CHUNK_ELEMS - 1) / CHUNK_ELEMS) * CHUNK_ELEMS : L.cin;
    const int Cp = G.cin_pad;
    std::vector<int2> taps;
    std::vector<float> packed;
    std::vector<std::vector<std::pair<int, int>>> phase_taps;   // (ky, kx) per tap
    if (L.kind == DENSE) {
        G.hq = G.wq = G.ho = G.wo = 1;
        G.nphase = 1;
        phase_taps.push_back({{0, 0}});
        taps.push_back(make_int2(0, 0));
        G.ph[0] = ConvPhase{0, 0, 1, 0, 0, 0};
    } else if (L.kind == CONV) {
        const int pt = same_pad_before(L.hin, L.kh, L.sh), pl = same_pad_before(L.win, L.kw, L.sw);
        G.hq = same_out(L.hin, L.sh);
        G.wq = same_out(L.win, L.sw);
        G.ho = L.pool ? G.hq / 2 : G.hq;
        G.wo = L.pool ? G.wq / 2 : G.wq;
        G.nphase = 1;
        std::vector<std::pair<int, int>> pt_list;
        for (int ky = 0; ky < L.kh; ++ky)
            for (int kx = 0; kx < L.kw; ++kx) {
                pt_list.push_back({ky, kx});
                taps.push_back(make_int2(ky - pt, kx - pl));
            }
        phase_taps.push_back(pt_list);
        G.ph[0] = ConvPhase{0, 0, (int)pt_list.size(), 0, 0, 0};
    } else {  // DECONV: TF conv2d_transpose 'SAME' to in*s, crop at pad_before = max(k - s, 0) / 2
        const int pt = std::max(L.kh - L.sh, 0) / 2, pl = std::max(L.kw - L.sw, 0) / 2;
        G.hq = L.hin;
        G.wq = L.win;
        G.ho = L.hin * L.sh;
        G.wo = L.win * L.sw;
        G.nphase = L.sh * L.sw;
        if (G.nphase > MAX_PHASES) return fail(AVSE_ERR_UNSUPPORTED, "deconv stride too large");
        for (int py = 0; py < L.sh; ++py)
            for (int px = 0; px < L.sw; ++px) {
                std::vector<std::pair<int, int>> pt_list;
                const int toff = (int)taps.size();
                for (int ky = 0; ky < L.kh; ++ky) {
                    const int ry = py + pt - ky;
                    if (((ry % L.sh) + L.sh) % L.sh) continue;
                    for (int kx = 0; kx < L.kw; ++kx) {
                        const int rx = px + pl - kx;
                        if (((rx % L.sw) + L.sw) % L.sw) continue;
                        pt_list.push_back({ky, kx});
                        taps.push_back(make_int2(ry / L.sh, rx / L.sw));
                    }
                }
                const int p = py * L.sw + px;
                G.ph[p] = ConvPhase{py, px, (int)pt_list.size(), 0, 0, toff};
                phase_taps.push_back(pt_list);
            }
    }
    // pack weights per phase: W[n][j*Cp + c]
    long long woff = 0;
    for (int p = 0; p < G.nphase; ++p) {
        const auto& pl_ = phase_taps[p];
        const int kpad = (((int)pl_.size() * Cp + 31) / 32) * 32;
        G.ph[p].kpad = kpad;
        G.ph[p].w_off = woff;
        packed.resize((size_t)(woff + (long long)L.cout * kpad), 0.f);
        for (int n = 0; n < L.cout; ++n)
            for (size_t j = 0; j < pl_.size(); ++j) {
                const int ky = pl_[j].first, kx = pl_[j].second;
                for (int c = 0; c < L.cin; ++c) {
                    float v;
                    if (L.kind == DENSE) v = kernel[(size_t)c * L.cout + n];
                    else if (L.kind == CONV) v = kernel[(((size_t)ky * L.kw + kx) * L.cin + c) * L.cout + n];
                    else v = kernel[(((size_t)ky * L.kw + kx) * L.cout + n) * L.cin + c];
                    packed[(size_t)woff + (size_t)n * kpad + j * Cp + c] = v;
                }
            }
        woff += (long long)L.cout * kpad;
    }
    // fold bias + BN into scale/shift
    std::vector<float> scale(L.cout), shift(L.cout);
    for (int n = 0; n < L.cout; ++n) {
        if (L.bn) {
            const int c = n % L.bn_channels;
            const float* g = bn;
            const float* b = bn + L.bn_channels;
            const float* mu = bn + 2 * L.bn_channels;
            const float* var = bn + 3 * L.bn_channels;
            const double s = (double)g[c] / std::sqrt((double)var[c] + (double)kBnEps);
            scale[n] = (float)s;
            shift[n] = (float)(((double)bias[n] - (double)mu[c]) * s + (double)b[c]);
        } else {
            scale[n] = 1.f;
            shift[n] = bias[n];
        }
    }
    int rc;
    const bool split = W->dtype == AVSE_F32_SPLIT;
    if (split && (e_in || e_out)) {
        // activation exponents (act_exponents): this layer reads pairs of x 2^e_in and stores pairs of y 2^e_out, so
        // y 2^e_out = LReLU(acc 2^-e_in scale 2^e_out + shift 2^e_out) — powers of two: exact, and they commute with
        // LeakyReLU and max pooling
        for (int n = 0; n < L.cout; ++n) {
            scale[n] = std::ldexp(scale[n], e_out - e_in);
            shift[n] = std::ldexp(shift[n], e_out);
        }
    }
    std::vector<float> scale_g = scale;   // the generic kernel's epilogue scale (split: with the weight exponents undone)
    if (W->dtype == AVSE_BF16) {
        std::vector<uint16_t> pb(packed.size());
        for (size_t i = 0; i < packed.size(); ++i) pb[i] = f2bf(packed[i]);
        uint16_t* d;
        if ((rc = upload(W, pb, &d))) return rc;
        G.w = d;
    } else if (split) {
        // conv.hip k_conv<float, .., S16>: each 16-k slab row of [Cout][kpad] becomes [Bh(16) | Bl(16)] f16 (the same
        // bytes), output channel n scaled by 2^e_n (max |w| 2^e_n in [2^14, 2^15), as the video layers' packing)
        std::vector<int> ex(L.cout, 0);
        for (int n = 0; n < L.cout; ++n) {
            float mx = 0.f;
            for (int p = 0; p < G.nphase; ++p)
                for (int k = 0; k < G.ph[p].kpad; ++k)
                    mx = std::max(mx, std::fabs(packed[(size_t)G.ph[p].w_off + (size_t)n * G.ph[p].kpad + k]));
            int e2 = 0;
            if (mx > 0.f) (void)std::frexp(mx, &e2);
            ex[n] = mx > 0.f ? 15 - e2 : 0;
            scale_g[n] = std::ldexp(scale[n], -ex[n]);
        }
        if (L.kind == CONV && L.cin == 1) {   // a_conv1: f32 taps with the same per-channel power of two
            std::vector<float> wf((size_t)L.kh * L.kw * L.cout);
            for (int t = 0; t < L.kh * L.kw; ++t)
                for (int n = 0; n < L.cout; ++n) wf[(size_t)t * L.cout + n] = std::ldexp(kernel[(size_t)t * L.cout + n], ex[n]);
            if ((rc = upload(W, wf, &G.w_f32))) return rc;
        }
        std::vector<uint16_t> sp(2 * packed.size(), 0);
        for (int p = 0; p < G.nphase; ++p)
            for (int n = 0; n < L.cout; ++n)
                for (int k = 0; k < G.ph[p].kpad; ++k) {
                    const size_t src = (size_t)G.ph[p].w_off + (size_t)n * G.ph[p].kpad + k;
                    const size_t dst = 2 * ((size_t)G.ph[p].w_off + (size_t)n * G.ph[p].kpad) + (size_t)(k / 16) * 32 + k % 16;
                    const float v = std::ldexp(packed[src], ex[n]);
                    const uint16_t h = f2h(v);
                    sp[dst] = h;
                    sp[dst + 16] = f2h(v - h2f(h));
                }
        uint16_t* d;
        if ((rc = upload(W, sp, &d))) return rc;
        G.w = d;
    } else {
        float* d;
        if ((rc = upload(W, packed, &d))) return rc;
        G.w = d;
    }
    if (W->dtype == AVSE_BF16 && L.kind == CONV && L.cin == 1 && L.kh * L.kw <= 32) {
        // conv_aud.hip's a_conv1: the single input channel's taps as a dense 32-deep K (25 real)
        std::vector<uint16_t> dw((size_t)L.cout * 32, 0);
        for (int n = 0; n < L.cout; ++n)
            for (int t = 0; t < L.kh * L.kw; ++t) dw[(size_t)n * 32 + t] = f2bf(kernel[(size_t)t * L.cout + n]);
        uint16_t* d;
        if ((rc = upload(W, dw, &d))) return rc;
        G.w_dense = d;
    }
    if ((rc = upload(W, scale_g, &G.scale))) return rc;
    if ((rc = upload(W, shift, &G.shift))) return rc;
    if ((rc = upload(W, taps, &G.taps))) return rc;
    for (size_t t = 0; t < taps.size() && t < (size_t)(MAX_TAPS * MAX_PHASES); ++t) G.htaps[t] = taps[t];

    // packing for the bf16 video conv kernels: conv_stream.hip [slice][Cout][32], slice = (cg*4 + cc)*KS^2
    // + tap; conv_v1r.hip (v_conv1) [kernel row][Cout][32].  Options::no_halo keeps the generic k_conv.
    // Split dtype: the same kernels on split-f16 operands (see below).
    if ((W->dtype == AVSE_BF16 || split) && L.kind == CONV && L.pool && L.hin >= 8 && !opt.no_halo) {
        const int ntap = L.kh * L.kw;
        if ((L.cin == 5 || L.cin == 6) && L.kh == 5)   // conv_v1r.hip: 5 (25 / 29.97 fps) or 6 frames (30)
            G.halo = split && L.cin == 5 && L.kw == 5 && L.cout == 128 && !opt.no_v1p ? HALO_V1P : HALO_V1;
        else if (L.cin % 128) G.halo = HALO_NONE;
        else if (L.kh == 5) G.halo = HALO_K5;
        else if (L.hin >= 16) G.halo = HALO_K3_16;
        else G.halo = HALO_K3_8;
        // Sign fold: a channel whose folded BN scale is negative gets negated weights and |scale|, so
        // every epilogue scale is >= 0 and 2x2 max pooling commutes exactly with scale/shift (the kernels
        // pool the raw accumulators, then apply one FMA).  bf16 negation and fp32 sums are exact.
        std::vector<float> sgn(L.cout), scale_h(L.cout);
        for (int n = 0; n < L.cout; ++n) {
            sgn[n] = scale[n] < 0.f ? -1.f : 1.f;
            scale_h[n] = std::fabs(scale[n]);
        }
        if (G.halo == HALO_NONE) return 0;
        if (split) {
            // split-f16 operands: output channel n's (sign-folded) weights scaled by 2^e_n, e_n = 14 - ceil(log2 max|w|),
            // so that hi = f16(w 2^e) stays below 2^15 and lo = f16(w 2^e - hi) keeps full precision for every weight
            // above 2^-10 of the channel's largest; the BN scale takes 2^-e_n back (powers of two: exact)
            const int ntap = L.kh * L.kw;
            std::vector<int> ex(L.cout, 0);
            for (int n = 0; n < L.cout; ++n) {
                float mx = 0.f;
                for (int t = 0; t < ntap; ++t)
                    for (int c = 0; c < L.cin; ++c) mx = std::max(mx, std::fabs(kernel[((size_t)t * L.cin + c) * L.cout + n]));
                int e2 = 0;
                if (mx > 0.f) (void)std::frexp(mx, &e2);   // mx = f 2^e2, f in [0.5, 1)
                ex[n] = mx > 0.f ? 15 - e2 : 0;              // max|w| 2^e in [2^14, 2^15)
                scale_h[n] = std::ldexp(scale_h[n], -ex[n]);
            }
            auto wsc = [&](int n, float v) { return std::ldexp(sgn[n] * v, ex[n]); };
            std::vector<uint16_t> sp;
            if (G.halo == HALO_V1P) {
                // conv_v1r.hip k_conv_v1p: [piece h / l][K-slice s][Cout][32]; k-group g = 4 s + kg (8 k each):
                //   s = 0..2, kg = ky (0..3), and s = 3, kg = s' (0..2) for ky = 4, of type s' / s:
                //   0: kx 0, 1 x frames 0..3;  1: kx 2, 3 x frames 0..3;  2: kx 4 x frames 0..3, then kx 0..3 x frame 4;
                //   s = 3, kg = 3: (ky 0..4, kx 4) x frame 4, three zeros
                const size_t img = (size_t)4 * L.cout * 32;
                sp.assign(2 * img, 0);
                auto wt = [&](int n, int ky, int kx, int f) { return wsc(n, kernel[((size_t)(ky * 5 + kx) * 5 + f) * L.cout + n]); };
                for (int g = 0; g < 16; ++g)
                    for (int n = 0; n < L.cout; ++n)
                        for (int j = 0; j < 8; ++j) {
                            const int sl = g >> 2, kg = g & 3;
                            const int t = sl < 3 ? sl : kg, ky = sl < 3 ? kg : 4;
                            float v = 0.f;
                            if (t == 0) v = wt(n, ky, j >> 2, j & 3);
                            else if (t == 1) v = wt(n, ky, 2 + (j >> 2), j & 3);
                            else if (t == 2) v = j < 4 ? wt(n, ky, 4, j) : wt(n, ky, j - 4, 4);
                            else if (j < 5) v = wt(n, j, 4, 4);
                            const uint16_t h = f2h(v);
                            const size_t o = ((size_t)(g >> 2) * L.cout + n) * 32 + (g & 3) * 8 + j;
                            sp[o] = h;
                            sp[img + o] = f2h(v - h2f(h));
                        }
            } else if (G.halo == HALO_V1) {
                // conv_v1r.hip k_conv_v1s: [piece h / l][kernel row ky][Cout][32], k = kx * 6 + frame
                const size_t img = (size_t)L.kh * L.cout * 32;
                sp.assign(2 * img, 0);
                for (int ky = 0; ky < L.kh; ++ky)
                    for (int n = 0; n < L.cout; ++n)
                        for (int kx = 0; kx < L.kw; ++kx)
                            for (int f = 0; f < L.cin; ++f) {
                                const float v = wsc(n, kernel[((size_t)(ky * L.kw + kx) * L.cin + f) * L.cout + n]);
                                const uint16_t h = f2h(v);
                                const size_t o = ((size_t)ky * L.cout + n) * 32 + kx * 6 + f;
                                sp[o] = h;
                                sp[img + o] = f2h(v - h2f(h));
                            }
            } else {
                // conv_stream.hip (S16): slice = chunk * KS^2 + tap over 16-channel chunks; row n = [Bh(16) | Bl(16)]
                const int nsteps = (L.cin / 16) * ntap;
                sp.assign((size_t)nsteps * L.cout * 32, 0);
                for (int st = 0; st < nsteps; ++st)
                    for (int n = 0; n < L.cout; ++n)
                        for (int kk = 0; kk < 16; ++kk) {
                            const int tap = st % ntap, c = (st / ntap) * 16 + kk;
                            const float v = wsc(n, kernel[((size_t)tap * L.cin + c) * L.cout + n]);
                            const uint16_t h = f2h(v);
                            sp[((size_t)st * L.cout + n) * 32 + kk] = h;
                            sp[((size_t)st * L.cout + n) * 32 + 16 + kk] = f2h(v - h2f(h));
                        }
            }
            if ((rc = upload(W, scale_h, &G.scale_h))) return rc;
            uint16_t* d;
            if ((rc = upload(W, sp, &d))) return rc;
            G.w_halo = d;
            return 0;
        }
        if ((rc = upload(W, scale_h, &G.scale_h))) return rc;
        std::vector<uint16_t> hp;
        if (G.halo == HALO_V1) {
            // conv_v1r.hip: slice ky, k = kx * 6 + frame (k = 30, 31 zero; frame 5 too with 5 frames)
            hp.assign((size_t)L.kh * L.cout * 32, 0);
            for (int ky = 0; ky < L.kh; ++ky)
                for (int n = 0; n < L.cout; ++n)
                    for (int kx = 0; kx < L.kw; ++kx)
                        for (int f = 0; f < L.cin; ++f)
                            hp[((size_t)ky * L.cout + n) * 32 + kx * 6 + f] =
                                f2bf(sgn[n] * kernel[((size_t)(ky * L.kw + kx) * L.cin + f) * L.cout + n]);
        } else {
            const int nsteps = (L.cin / 128) * 4 * ntap;   // (4 chunks of 32 channels per 128) x taps
            hp.assign((size_t)nsteps * L.cout * 32, 0);
            for (int st = 0; st < nsteps; ++st)
                for (int n = 0; n < L.cout; ++n)
                    for (int kk = 0; kk < 32; ++kk) {
                        const int tap = st % ntap, chunk = st / ntap;   // chunk = cg*4 + cc
                        const int c = chunk * 32 + kk;
                        hp[((size_t)st * L.cout + n) * 32 + kk] =
                            f2bf(sgn[n] * kernel[((size_t)tap * L.cin + c) * L.cout + n]);
                    }
        }
        uint16_t* d;
        if ((rc = upload(W, hp, &d))) return rc;
        G.w_halo = d;
    }
    return 0;
}

HaloArgs halo_args(const GpuLayer& G, const void* in, const float* video, const float* vmean, const float* vstd,
                   void* out, long long out_clip_stride, int out_pix_stride, int out_c_off, int64_t N,
                   const Options& opt) {
    HaloArgs a;
    std::memset(&a, 0, sizeof(a));
    a.variant = G.halo;
    a.in = in;
    a.video = video;
    a.vmean = vmean;
    a.vstd = vstd;
    a.out = out;
    a.w = G.w_halo;
    a.mfma32 = opt.mfma32;
    a.scale = G.scale_h;
    a.shift = G.shift;
    a.N = (int)N;
    a.Hc = G.def.hin;
    a.Wc = G.def.win;
    a.Ci = G.def.cin;
    a.Co = G.def.cout;
    a.out_clip_stride = out_clip_stride;
    a.out_pix_stride = out_pix_stride;
    a.out_c_off = out_c_off;
    return a;
}

// fused d_deconv4 -> d_deconv5 -> d_deconv6 (conv_dec.hip): window geometry from the layers' tap extents
DecTailArgs dec_tail_args(const GpuLayer& G4, const GpuLayer& G5, const avse_weights* W, const void* in, float* out,
                          int64_t N) {
    DecTailArgs a;
    std::memset(&a, 0, sizeof(a));
    a.in = reinterpret_cast<const bf16_t*>(in);
    a.out = out;
    a.N = (int)N;
    auto extents = [](const GpuLayer& G, int p, int& dy0, int& dy1, int& dx0, int& dx1) {
        dy0 = dx0 = 1 << 20;
        dy1 = dx1 = -(1 << 20);
        for (int t = 0; t < G.ph[p].ntaps; ++t) {
            const int2 d = G.htaps[G.ph[p].tap_off + t];
            dy0 = std::min(dy0, d.x); dy1 = std::max(dy1, d.x);
            dx0 = std::min(dx0, d.y); dx1 = std::max(dx1, d.y);
        }
    };
    a.w4 = reinterpret_cast<const bf16_t*>(G4.w);
    a.sc4 = G4.scale;
    a.sh4 = G4.shift;
    a.nt4 = G4.ph[0].ntaps;
    a.kpad4 = G4.ph[0].kpad;
    int dy0, dy1, dx0, dx1;
    extents(G4, 0, dy0, dy1, dx0, dx1);
    a.pt4 = -dy0; a.pl4 = -dx0; a.rows4 = G4.hq + dy1 - dy0; a.pitch4 = G4.wq + dx1 - dx0;
    // the kernel walks a phase's taps as a (dy0 - a, dx0 - b) grid with nx columns: check that layout
    bool grid_ok = true;
    auto tap_grid = [&](const GpuLayer& G, int p, int& dy, int& dx, int& nx) {
        const int2* t = G.htaps + G.ph[p].tap_off;
        const int nt = G.ph[p].ntaps;
        dy = t[0].x;
        dx = t[0].y;
        nx = 1;
        while (nx < nt && t[nx].x == dy) ++nx;
        for (int k = 0; k < nt; ++k)
            if (t[k].x != dy - k / nx || t[k].y != dx - k % nx) grid_ok = false;
    };
    tap_grid(G4, 0, a.dy4, a.dx4, a.nx4);
    a.w5 = reinterpret_cast<const bf16_t*>(G5.w);
    a.sc5 = G5.scale;
    a.sh5 = G5.shift;
    int ey0 = 1 << 20, ey1 = -(1 << 20), ex0 = 1 << 20, ex1 = -(1 << 20);
    for (int p = 0; p < 4 && p < G5.nphase; ++p) {
        a.nt5[p] = G5.ph[p].ntaps;
        a.kpad5[p] = G5.ph[p].kpad;
        a.woff5[p] = G5.ph[p].w_off;
        tap_grid(G5, p, a.dy5[p], a.dx5[p], a.nx5[p]);
        extents(G5, p, dy0, dy1, dx0, dx1);
        ey0 = std::min(ey0, dy0); ey1 = std::max(ey1, dy1);
        ex0 = std::min(ex0, dx0); ex1 = std::max(ex1, dx1);
    }
    a.pt5 = -ey0; a.pl5 = -ex0; a.rows5 = G5.hq + ey1 - ey0; a.pitch5 = G5.wq + ex1 - ex0;
    a.w6 = W->d6_w;
    a.b6 = W->d6_bias;
    // shapes the kernel is written for (network.py:125-133 at the 200-ms segment); anything else: k_conv
    const bool shape_ok = G4.def.kind == DECONV && G5.def.kind == DECONV && G4.hq == 40 && G4.wq == 10 &&
                          G4.def.cin == 128 && G4.def.cout == 64 && G4.nphase == 1 && G5.hq == 40 && G5.wq == 10 &&
                          G5.def.cin == 64 && G5.def.cout == 64 && G5.nphase == 4 && G5.def.sh == 2 && G5.def.sw == 2 &&
                          grid_ok;
    if (!shape_ok) a.N = 0;   // dec_tail_supported() refuses
    return a;
}

ConvArgs conv_args(const GpuLayer& G, const void* in, long long in_clip_stride, void* out, long long out_clip_stride,
                   int out_pix_stride, int out_c_off, int64_t N) {
    const LayerDef& L = G.def;
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.in = in;
    a.out = out;
    a.w = G.w;
    a.scale = G.scale;
    a.shift = G.shift;
    a.taps = G.taps;
    a.N = (int)N;
    a.Hi = L.hin;
    a.Wi = L.win;
    a.Ci = (L.kind == DENSE) ? L.cin : G.cin_pad;
    a.in_clip_stride = in_clip_stride;
    a.Hq = G.hq;
    a.Wq = G.wq;
    a.sy = (L.kind == CONV) ? L.sh : 1;
    a.sx = (L.kind == CONV) ? L.sw : 1;
    a.oys = (L.kind == DECONV) ? L.sh : 1;
    a.oxs = (L.kind == DECONV) ? L.sw : 1;
    a.Ho = G.ho;
    a.Wo = G.wo;
    a.Co = L.cout;
    a.out_clip_stride = out_clip_stride;
    a.out_pix_stride = out_pix_stride;
    a.out_c_off = out_c_off;
    a.pool = L.pool ? 1 : 0;
    a.act = 1;
    a.nphase = G.nphase;
    a.ksplit = 1;
    for (int p = 0; p < G.nphase; ++p) a.ph[p] = G.ph[p];
    return a;
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

int avse_abi_version(void) { return AVSE_ABI_VERSION; }

int avse_build_flags(void) { return avse::kDebugBuild ? 1 : 0; }
const char* avse_last_error(void) { return g_err.c_str(); }

int avse_ctx_create(int device, avse_ctx** out) {
    if (!out) return fail(AVSE_ERR_INVALID, "out is NULL");
    int n = 0;
    AVSE_HIP_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(AVSE_ERR_INVALID, "bad device index");
    AVSE_HIP_CHECK(hipSetDevice(device));
    avse_ctx* c = new avse_ctx();
    c->device = device;
    for (const OptionName& o : kOptionNames) {
        const char* e = std::getenv(o.env);
        if (e && *e) c->opt.*(o.field) = std::atoi(e);
    }
    if (hipMalloc((void**)&c->mse_partial, sizeof(float) * 256) != hipSuccess ||
        hipMalloc((void**)&c->gemm_counters, sizeof(int) * 8192) != hipSuccess ||
        hipMemset(c->gemm_counters, 0, sizeof(int) * 8192) != hipSuccess ||
        hipMalloc((void**)&c->range, sizeof(unsigned) * 4) != hipSuccess ||
        hipMemset(c->range, 0, sizeof(unsigned) * 4) != hipSuccess ||
        hipHostMalloc((void**)&c->range_host, sizeof(unsigned) * 4, hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(c->mse_partial);
        (void)hipFree(c->gemm_counters);
        (void)hipFree(c->range);
        delete c;
        return fail(AVSE_ERR_OOM, "hipMalloc failed (ctx)");
    }
    *out = c;
    return 0;
}

void avse_ctx_destroy(avse_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipFree(c->spec.twiddle); (void)hipFree(c->spec.window);
    (void)hipFree(c->spec.mel.start); (void)hipFree(c->spec.mel.width); (void)hipFree(c->spec.mel.weight);
    (void)hipFree(c->istft.pinvT); (void)hipFree(c->istft.twiddle); (void)hipFree(c->istft.window);
    (void)hipFree(c->istft.bins); (void)hipFree(c->istft.gram_inv);
    (void)hipFree(c->frames);
    (void)hipFree(c->umax);
    (void)hipFree(c->mse_partial);
    (void)hipFree(c->gemm_counters);
    (void)hipFree(c->range);
    (void)hipHostFree(c->range_host);
    (void)hipFree(c->zero_video);
    (void)hipFree(c->arena);
    for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    if (c->cap) (void)hipStreamDestroy(c->cap);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->join) (void)hipEventDestroy(c->join);
    delete c;
}

int avse_ctx_set_option(avse_ctx* c, const char* name, int value) {
    if (!c || !name) return fail(AVSE_ERR_INVALID, "NULL argument");
    for (const OptionName& o : kOptionNames)
        if (std::strcmp(o.name, name) == 0) {
            c->opt.*(o.field) = value;
            return 0;
        }
    return fail(AVSE_ERR_INVALID, std::string("unknown option '") + name + "'");
}

int avse_ctx_get_option(avse_ctx* c, const char* name, int* value) {
    if (!c || !name || !value) return fail(AVSE_ERR_INVALID, "NULL argument");
    for (const OptionName& o : kOptionNames)
        if (std::strcmp(o.name, name) == 0) {
            *value = c->opt.*(o.field);
            return 0;
        }
    return fail(AVSE_ERR_INVALID, std::string("unknown option '") + name + "'");
}

int avse_ctx_reserve(avse_ctx* c, int64_t max_clips, int dtype) {
    if (!c || max_clips < 0 || !valid_dtype(dtype)) return fail(AVSE_ERR_INVALID, "bad reserve args");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    return ensure_arena(c, max_clips, dtype, kPlan25, nullptr);   // the 25-fps network's scratch
}

int avse_ctx_reserve_weights(avse_ctx* c, const avse_weights* w, int64_t max_clips) {
    if (!c || !w || max_clips < 0) return fail(AVSE_ERR_INVALID, "bad reserve args");
    if (w->device != c->device) return fail(AVSE_ERR_INVALID, "weights and context are on different devices");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    return ensure_arena(c, max_clips, w->dtype, w->plan, nullptr);   // the network shape these weights were built for
}

namespace avse {
// checked build: wait for the stream, then report the first device-side check that fired (avse_common.h DebugHit)
int debug_poll(void* stream) {
    if constexpr (!kDebugBuild) return 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    AVSE_HIP_CHECK(hipStreamIsCapturing((hipStream_t)stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return 0;   // no synchronisation inside a capture: checked on a later call
    AVSE_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    static const struct {
        int (*read)(DebugHit*);
        const char* what;
    } readers[] = {{debug_read_v1r, "k_conv_v1r"}, {debug_read_stft, "STFT"}, {debug_read_istft, "ISTFT"}};
    for (const auto& r : readers) {
        DebugHit h{};
        if (r.read(&h)) return fail(AVSE_ERR_HIP, "checked build: reading the device check record failed");
        if (h.hit)
            return fail(AVSE_ERR_CHECK, std::string("checked build: ") + r.what + " check " + std::to_string(h.code) +
                                            " failed (kernel id " + std::to_string(h.kernel) + ", block " +
                                            std::to_string(h.block) + ", thread " + std::to_string(h.thread) +
                                            ": value " + std::to_string(h.value) + ", expected " +
                                            std::to_string(h.expect) + ")");
    }
    return 0;
}
}  // namespace avse

int avse_spectrogram(avse_ctx* c, const float* sig, int64_t n_utt, int64_t n_samples, int sr, int n_fft, int hop,
                     int n_mels, float fmin, float fmax, float amin, float top_db, int pad_mode, int frames_per_slice,
                     float* mel_db, float* stft_ri, void* stream) {
    if (!c || !sig || !mel_db) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (n_utt < 0 || n_samples <= 0 || sr <= 0 || hop <= 0 || n_fft < 2)
        return fail(AVSE_ERR_INVALID, "bad spectrogram geometry");
    if (n_fft > 2048) return fail(AVSE_ERR_UNSUPPORTED, "n_fft > 2048 not supported");
    if (n_mels < 1 || n_mels > 80) return fail(AVSE_ERR_UNSUPPORTED, "n_mels must be in [1, 80]");
    if (pad_mode != AVSE_PAD_REFLECT && pad_mode != AVSE_PAD_CONSTANT) return fail(AVSE_ERR_INVALID, "bad pad_mode");
    if (pad_mode == AVSE_PAD_REFLECT && n_samples <= n_fft / 2)
        return fail(AVSE_ERR_INVALID, "reflect padding needs n_samples > n_fft/2");
    if (frames_per_slice < 0) return fail(AVSE_ERR_INVALID, "frames_per_slice < 0");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    int rc = ensure_spec_tables(c, sr, n_fft, n_mels, fmin, fmax);
    if (rc) return rc;
    if (n_utt > c->umax_cap) {
        (void)hipFree(c->umax);
        c->umax = nullptr;
        AVSE_HIP_CHECK(hipMalloc((void**)&c->umax, sizeof(unsigned) * n_utt));
        c->umax_cap = n_utt;
    }
    SpecArgs a;
    a.sig = sig;
    a.n_utt = n_utt;
    a.n_samples = n_samples;
    a.n_fft = n_fft;
    a.hop = hop;
    a.n_frames = (int)(1 + (n_samples + 2 * (n_fft / 2) - n_fft) / hop);   // centred frames (librosa.stft)
    a.n_mels = n_mels;
    a.amin = amin;
    a.db_floor = (float)(20.0 * std::log10((double)amin));   // exact value for clamped bins
    a.top_db = top_db;
    a.pad_mode = pad_mode;
    a.spf = frames_per_slice;
    a.n_slices = frames_per_slice > 0 ? a.n_frames / frames_per_slice : 0;
    a.mel_db = mel_db;
    a.stft_ri = stft_ri;
    a.twiddle = c->spec.twiddle;
    a.window = c->spec.window;
    a.mel_start = c->spec.mel.start;
    a.mel_width = c->spec.mel.width;
    a.mel_weight = c->spec.mel.weight;
    a.mel_max_width = c->spec.mel.max_width;
    std::memcpy(a.mel_seg_nq, c->spec.mel.seg_nq, sizeof(a.mel_seg_nq));
    std::memcpy(a.mel_seg_nq4, c->spec.mel.seg_nq4, sizeof(a.mel_seg_nq4));
    a.umax = c->umax;
    if (int lr = launch_spectrogram(a, (hipStream_t)stream)) return lr;
    return debug_poll(stream);
}

int avse_istft(avse_ctx* c, const float* mel_db, const float* stft_ri, int64_t n_utt, int n_frames, int stft_frames,
               int frames_per_slice, int sr, int n_fft, int hop, int n_mels, float fmin, float fmax, float* sig,
               void* stream) {
    if (!c || !mel_db || !stft_ri || !sig) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (n_utt < 0 || n_frames < 1 || stft_frames < n_frames || hop <= 0 || sr <= 0 || n_fft < 2)
        return fail(AVSE_ERR_INVALID, "bad istft geometry (need 1 <= n_frames <= stft_frames)");
    if (n_fft > 2048) return fail(AVSE_ERR_UNSUPPORTED, "n_fft > 2048 not supported");
    if (n_mels < 1 || n_mels > 80) return fail(AVSE_ERR_UNSUPPORTED, "n_mels must be in [1, 80]");
    if (frames_per_slice < 0 || (frames_per_slice > 0 && n_frames % frames_per_slice))
        return fail(AVSE_ERR_INVALID, "n_frames must be a multiple of frames_per_slice");
    if (n_utt == 0) return 0;
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    int rc = ensure_istft_tables(c, sr, n_fft, n_mels, fmin, fmax);
    if (rc) return rc;
    const int nb = 1 + n_fft / 2, N = 2 * (nb - 1);
    const size_t need = sizeof(float) * (size_t)n_utt * n_frames * N;
    if (need > c->frames_bytes) {
        (void)hipFree(c->frames);
        c->frames = nullptr;
        c->frames_bytes = 0;
        if (hipMalloc((void**)&c->frames, need) != hipSuccess) return fail(AVSE_ERR_OOM, "hipMalloc failed (istft scratch)");
        c->frames_bytes = need;
    }
    IstftArgs a;
    a.mel_db = mel_db;
    a.spf = frames_per_slice;
    a.n_slices = frames_per_slice > 0 ? n_frames / frames_per_slice : 0;
    a.stft = reinterpret_cast<const float2*>(stft_ri);
    a.stft_frames = stft_frames;
    a.n_utt = n_utt;
    a.T = n_frames;
    a.nb = nb;
    a.N = N;
    a.hop = hop;
    a.n_mels = n_mels;
    a.pinvT = c->istft.pinvT;
    a.twiddle = c->istft.twiddle;
    a.window = c->istft.window;
    a.frames = c->frames;
    a.sig = sig;
    a.bins = c->istft.bins;
    a.gram_inv = c->opt.dense_istft ? nullptr : c->istft.gram_inv;
    if (int lr = launch_istft(a, (hipStream_t)stream)) return lr;
    return debug_poll(stream);
}

int64_t avse_weights_blob_floats(void) { return blob_floats(kPlan25); }

int64_t avse_weights_blob_floats_shape(int spec_frames, int video_frames) {
    if (!plan_valid(spec_frames, video_frames)) return -1;
    return blob_floats(make_plan(spec_frames, video_frames));
}

int avse_weights_load(avse_ctx* c, const float* blob, int64_t n_floats, int dtype, avse_weights** out) {
    return avse_weights_load_shape(c, blob, n_floats, dtype, kPlan25.T, kPlan25.F, out);
}

int avse_weights_shape(const avse_weights* w, int* spec_frames, int* video_frames) {
    if (!w || !spec_frames || !video_frames) return fail(AVSE_ERR_INVALID, "NULL argument");
    *spec_frames = w->plan.T;
    *video_frames = w->plan.F;
    return 0;
}

int avse_weights_load_shape(avse_ctx* c, const float* blob, int64_t n_floats, int dtype, int spec_frames,
                            int video_frames, avse_weights** out) {
    if (!c || !blob || !out) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (!valid_dtype(dtype)) return fail(AVSE_ERR_INVALID, "bad compute dtype");
    if (!plan_valid(spec_frames, video_frames))
        return fail(AVSE_ERR_UNSUPPORTED, "network shape [80, " + std::to_string(spec_frames) + "] x [128, 128, " +
                                              std::to_string(video_frames) + "]: the decoder reproduces 80 x T only for "
                                              "T a multiple of 4; video frames must be 1..8");
    const NetPlan plan = make_plan(spec_frames, video_frames);
    if (n_floats != blob_floats(plan))
        return fail(AVSE_ERR_INVALID, "weight blob has " + std::to_string(n_floats) + " floats, expected " +
                                          std::to_string(blob_floats(plan)));
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    avse_weights* W = new avse_weights();
    static std::atomic<uint64_t> next_serial{1};
    W->serial = next_serial++;
    W->dtype = dtype;
    W->device = c->device;
    W->plan = plan;
    if (dtype == AVSE_F32_SPLIT) {
        if (!c->opt.no_act_scale) act_exponents(plan, blob, W->act_exp);
        W->blob.assign(blob, blob + n_floats);   // avse_forward_checked's exact-fp32 twin is built from it on demand
    }
    const float* p = blob;
    for (int i = 0; i < kNumLayers; ++i) {
        const LayerDef& L = plan.L[i];
        const float* kernel = p;
        p += (size_t)L.kh * L.kw * L.cin * L.cout;
        const float* bias = p;
        p += L.cout;
        const float* bn = nullptr;
        if (L.bn) {
            bn = p;
            p += 4 * (size_t)L.bn_channels;
        }
        if (i == kNumLayers - 1) {  // d_deconv6: 1x1, 64 -> 1
            std::vector<float> w64(kernel, kernel + 64);
            int rc = upload(W, w64, &W->d6_w);
            if (rc) { delete W; return rc; }
            W->d6_bias = bias[0];
            continue;
        }
        int rc = build_layer(W, i, kernel, bias, bn, c->opt, act_exp_in(W->act_exp, i), W->act_exp[i]);
        if (rc) { delete W; return rc; }
    }
    if (dtype == AVSE_F32_SPLIT) {
        // the split layers pass split-pair activations to each other: they must be a prefix v_conv1 .. of the video
        // encoder (a v_conv1 on the generic kernel makes every video layer generic; no_halo: all of them)
        bool prefix = true;
        for (int i = 5; i < 11; ++i) {
            if (W->layers[i].halo == HALO_NONE) prefix = false;
            if (!prefix) W->layers[i].halo = HALO_NONE;
        }
    }
    *out = W;
    return 0;
}

int avse_weights_act_exponents(const avse_weights* w, int* host_exp, int n) {
    if (!w || !host_exp || n < 0) return fail(AVSE_ERR_INVALID, "bad act_exponents args");
    for (int i = 0; i < n && i < kNumLayers; ++i) host_exp[i] = w->act_exp[i];
    return 0;
}

void avse_weights_destroy(avse_weights* w) {
    if (!w) return;
    (void)hipSetDevice(w->device);
    delete w;
}

}  // extern "C"

namespace {
// Stage order of avse_forward_profile (include/avse.h AVSE_NUM_STAGES).
// rflag: the split dtype's range-guard word the kernels report into (avse_ctx::range)
int forward_impl(avse_ctx* c, const avse_weights* W, const float* audio, const float* video, const float* vmean,
                 const float* vstd, int64_t N, float* out, hipStream_t s, hipEvent_t* ev, unsigned* rflag) {
    if (!c || !W || !audio || !out) return fail(AVSE_ERR_INVALID, "NULL argument");
    if ((vmean == nullptr) != (vstd == nullptr)) return fail(AVSE_ERR_INVALID, "vnorm_mean and vnorm_std must both be set or both NULL");
    if (!video && vmean) return fail(AVSE_ERR_INVALID, "video == NULL (all-zero video) takes no normaliser");
    if (N < 0 || N > (int64_t)(1 << 30) / (128 * 128)) return fail(AVSE_ERR_INVALID, "bad N");
    if (N == 0) return 0;
    if (W->device != c->device) return fail(AVSE_ERR_INVALID, "weights and context are on different devices");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    const NetPlan& P = W->plan;
    int rc = ensure_arena(c, N, W->dtype, P, s);
    if (rc) return rc;
    c->last_plan = P;
    const int dt = W->dtype;
    const bool split = dt == AVSE_F32_SPLIT;               // video convs on split-f16 operands, the rest fp32
    const int gdt = dt == AVSE_BF16 ? AVSE_BF16 : AVSE_F32;   // dtype of the generic kernels' buffers
    // launch_conv's arithmetic.  Split dtype: f16 split products; every generic layer writes its output as split pairs
    // (the next layer loads them as they are), except d_deconv5 (fused d_deconv6 -> float output, or fp32 unfused); the
    // layers fed by the fp32 preps (a_conv1, a generic v_conv1) split their fp32 input in the kernel
    const int cdt = split ? kConvSplit : gdt;
    // li: the layer's index in the plan (its range-guard bit)
    auto pairs = [&](ConvArgs& a, bool in_pairs, bool out_pairs, int li) -> int {
        if (!split) return gdt;
        a.range_flag = rflag;
        a.range_bit = 1u << li;
        a.range_in_bit = li == 0 ? kRangeAudioIn : kRangeVideoIn;   // the fp32 input split on load (a_conv1, v_conv1)
        if (in_pairs) {
            a.Ci *= 2;
            a.in_clip_stride *= 2;
            for (int p = 0; p < a.nphase; ++p) {
                a.ph[p].kpad *= 2;
                a.ph[p].w_off *= 2;
            }
        }
        if (out_pairs) {
            a.out_s16 = 1;
            a.out_clip_stride *= 2;
            a.out_pix_stride *= 2;
            a.out_c_off *= 2;
        }
        return in_pairs ? kConvSplitPairs : kConvSplit;
    };
    // a generic layer launch: split-pair stride-1 gather layers on the windowed kernel (conv_win.hip) when it takes
    // their shape (option no_win: always k_conv)
    auto conv = [&](const ConvArgs& a, int dti, const GpuLayer& G, hipStream_t st) -> int {
        if (split && dti == kConvSplitPairs && !c->opt.no_win) {
            const int rw = launch_conv_win(a, G.htaps, st);
            if (rw != -1) return rw;
        }
        return launch_conv(a, split ? dti : cdt, st);
    };
    size_t off[B_COUNT + 1];
    arena_bytes(N, dt, c->opt, off, P);
    const long long CAT = P.cat, AEMB = P.aemb, EMB = P.emb;
    const Options& opt = c->opt;
    auto buf = [&](int b) { return (void*)(c->arena + off[b]); };
    // dense layers and v_conv6 on gemm.hip (bf16, and split pairs: k_gemm S16; Options::no_gemm keeps k_conv + split-K
    // reduce)
    const bool use_gemm = (dt == AVSE_BF16 || split) && !opt.no_gemm;
    auto gemm = [&](const GpuLayer& G, const void* in, long long lda, void* outp, long long ldo, int out_off, int mode,
                    int64_t n, size_t part_off, int li) {
        GemmArgs g;
        std::memset(&g, 0, sizeof(g));
        g.a = reinterpret_cast<const bf16_t*>(in);
        g.lda = split ? 2 * lda : lda;
        g.w = reinterpret_cast<const bf16_t*>(G.w);
        g.M = (int)(mode == 1 ? n * 16 : n);
        g.N = G.def.cout;
        g.kpad = G.ph[0].kpad;
        g.scale = G.scale;
        g.shift = G.shift;
        g.act = 1;
        g.out = reinterpret_cast<bf16_t*>(outp);
        g.ldo = split ? 2 * ldo : ldo;
        g.out_off = split ? 2 * out_off : out_off;
        if (split) {
            // the k_conv path's plans: v_conv6 one block per split (or none), the dense layers from K and N only
            g.split = 1;
            if (mode == 1) {
                g.ksplit = choose_ksplit(g.M, g.N, g.kpad, dt);
                g.slabs_per_split = g.ksplit > 1 ? kFp32Block : 0;
            } else {
                g.ksplit = gemm_s16_ksplit(g.N, g.kpad, &g.slabs_per_split);
            }
            g.range_flag = rflag;
            g.range_bit = 1u << li;
        } else {
            g.ksplit = gemm_ksplit(g.M, g.N, g.kpad, opt.gemm_ksplit_cap);
        }
        g.partial = reinterpret_cast<float*>(c->arena + part_off);
        g.counters = c->gemm_counters;
        return launch_gemm(g, mode, s);
    };
    // dense layers / v_conv6: split-K when the grid is small, partials at the split-K offset of the arena layout the
    // launch's activations use (the N = 1 zero-video encoder has its own layout: its v_conv6 splits 36 ways)
    auto ksplit = [&](ConvArgs& a, size_t partial_off) {
        if (a.nphase != 1) return;
        const int64_t M = (int64_t)a.N * a.Hq * a.Wq;
        a.ksplit = choose_ksplit(M, a.Co, a.ph[0].kpad, dt, a.ph[0].ntaps == 1, &a.ksplit_slabs);
        a.partial = reinterpret_cast<float*>(c->arena + partial_off);
    };
    auto L = [&](int i) -> const GpuLayer& { return W->layers[i]; };
    int stage = 0;
    auto mark = [&]() -> int {
        if (ev) AVSE_HIP_CHECK(hipEventRecord(ev[stage], s));
        ++stage;
        return 0;
    };
    if ((rc = mark())) return rc;   // video_prep stage: now the video encoder's first launch (k_conv path only)
    if ((rc = mark())) return rc;
    // video encoder (network.py:138-175) over n clips, activations at the arena offsets o, embedding into cat
    auto video_encoder = [&](const float* vid, const float* vm, const float* vs, int64_t n, const size_t* o,
                             void* cat) -> int {
        auto vb = [&](int b) { return (void*)(c->arena + o[b]); };
        const int v_in[6] = {B_VIN, B_V1, B_V2, B_V3, B_V4, B_V5};
        if (L(5).halo == HALO_NONE && (rc = launch_video_prep(vid, vm, vs, vb(B_VIN), n, P.F, gdt, s))) return rc;
        for (int i = 0; i < 6; ++i) {
            const GpuLayer& G = L(5 + i);
            if (G.halo != HALO_NONE) {
                HaloArgs h = (i < 5) ? halo_args(G, vb(v_in[i]), vid, vm, vs, vb(v_in[i + 1]),
                                                 (long long)G.ho * G.wo * G.def.cout, G.def.cout, 0, n, opt)
                                     : halo_args(G, vb(v_in[i]), vid, vm, vs, cat, CAT, G.def.cout, AEMB, n, opt);
                if (split) {
                    // split-pair input (2 halves per channel) from the previous split layer; output split pairs for
                    // a next split layer, fp32 for a generic one (weights_load keeps the split layers a prefix)
                    // every consumer (the next split layer or the generic v_conv6) takes the pair layout
                    h.split = 1;
                    h.range_flag = rflag;
                    h.range_bit = 1u << (5 + i);
                    h.range_in_bit = kRangeVideoIn;
                    if (G.halo != HALO_V1 && G.halo != HALO_V1P) h.Ci = 2 * G.def.cin;
                    h.out_mode = OUT_S16;
                    h.out_clip_stride *= 2;
                    h.out_pix_stride *= 2;
                    h.out_c_off *= 2;
                }
                rc = G.halo == HALO_V1 || G.halo == HALO_V1P ? launch_conv_v1r(h, s) : launch_conv_stream(h, s);
                if (rc || (rc = mark())) return rc;
                continue;
            }
            const long long in_cs = (long long)G.def.hin * G.def.win * (i == 0 ? G.cin_pad : G.def.cin);
            if (i == 5 && use_gemm && G.def.hin == 4 && G.def.win == 4 && G.def.cin == 512 && G.def.kh == 3 && G.def.pool &&
                G.ph[0].kpad == 9 * 512) {
                if ((rc = gemm(G, vb(v_in[i]), in_cs, cat, CAT, AEMB, 1, n, o[B_COUNT], 10)) || (rc = mark())) return rc;   // concat[aemb:]
                continue;
            }
            ConvArgs a = (i < 5) ? conv_args(G, vb(v_in[i]), in_cs, vb(v_in[i + 1]), (long long)G.ho * G.wo * G.def.cout, G.def.cout, 0, n)
                                 : conv_args(G, vb(v_in[i]), in_cs, cat, CAT, G.def.cout, AEMB, n);  // concat[aemb:]
            if (i == 5) ksplit(a, o[B_COUNT]);
            const int dti = pairs(a, i > 0, true, 5 + i);   // v_conv1 generic: fp32 video-prep input
            if ((rc = launch_conv(a, split ? dti : cdt, s)) || (rc = mark())) return rc;
        }
        return 0;
    };
    // all-zero video: the embedding is one constant 2048-vector, computed once per weights object by an N = 1 video
    // encoder in the N = 1 arena layout.  It runs here, before the audio branch is launched: the per-layer audio
    // branch runs on the side stream and its N-clip buffers overlap the N = 1 layout (round 3: a race that broke
    // video == NULL forwards whenever the audio encoder was not the fused kernel, e.g. at 29.97 fps)
    if (!video) {
        const size_t es = dt == AVSE_BF16 ? 2 : 4;
        if (!W->vzero_emb.load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(W->vzero_mu);
            if (!W->vzero_emb.load(std::memory_order_relaxed)) {
                hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                AVSE_HIP_CHECK(hipStreamIsCapturing(s, &cs));
                if (cs != hipStreamCaptureStatusNone)
                    return fail(AVSE_ERR_INVALID, "the all-zero-video embedding must be computed before graph capture");
                if (!c->zero_video) {
                    AVSE_HIP_CHECK(hipMalloc((void**)&c->zero_video, sizeof(float) * 128 * 128 * 8));
                    AVSE_HIP_CHECK(hipMemsetAsync(c->zero_video, 0, sizeof(float) * 128 * 128 * 8, s));
                }
                void* emb = nullptr;
                AVSE_HIP_CHECK(hipMalloc(&emb, 2048 * es));
                size_t o1[B_COUNT + 1];
                arena_bytes(1, dt, opt, o1, P);
                hipEvent_t* keep = ev;
                unsigned* keep_flag = rflag;
                const int keep_stage = stage;
                ev = nullptr;   // the one-off N = 1 encoder is not a profiled stage
                rflag = c->range + 2;   // its own range word: the bits are kept with the cached embedding
                if (split) AVSE_HIP_CHECK(hipMemsetAsync(rflag, 0, sizeof(unsigned), s));
                rc = video_encoder(c->zero_video, nullptr, nullptr, 1, o1, c->arena + o1[B_CAT]);
                ev = keep;
                rflag = keep_flag;
                stage = keep_stage;
                if (rc) { (void)hipFree(emb); return rc; }
                AVSE_HIP_CHECK(hipMemcpyAsync(emb, c->arena + o1[B_CAT] + AEMB * es, 2048 * es, hipMemcpyDeviceToDevice, s));
                if (split) AVSE_HIP_CHECK(hipMemcpyAsync(c->range_host + 2, c->range + 2, sizeof(unsigned), hipMemcpyDeviceToHost, s));
                // one-time: the embedding is complete before any stream can see the pointer
                AVSE_HIP_CHECK(hipStreamSynchronize(s));
                W->vzero_range = split ? c->range_host[2] : 0u;
                W->vzero_emb.store(emb, std::memory_order_release);
            }
        }
    }
    // audio encoder (network.py:88-109): one fused kernel per clip (conv_aud.hip) when the layers have the network's
    // shapes (AVSE_NO_AUDENC=1: per-layer launches); profiled, its time shows as the audio_prep stage
    bool aud_fused = false;
    AudEncArgs aa;
    std::memset(&aa, 0, sizeof(aa));
    if (dt == AVSE_BF16) {
        aa.mel = audio;
        aa.out = reinterpret_cast<bf16_t*>(buf(B_CAT));
        aa.out_clip_stride = CAT;
        aa.N = (int)N;
        const void* ws[5] = {L(0).w_dense, L(1).w, L(2).w, L(3).w, L(4).w};
        const LayerDef* d = &L(0).def;
        const bool shapes = d[0].cin == 1 && L(0).hq == 40 && L(0).wq == 10 && L(1).def.cin == 64 && L(1).def.cout == 64 &&
                            L(1).def.kh == 4 && L(2).def.cout == 128 && L(2).hq == 20 && L(2).wq == 5 && L(3).hq == 10 &&
                            L(3).wq == 5 && L(4).hq == 5 && L(4).wq == 5 && L(3).ph[0].kpad == 512 && L(4).ph[0].kpad == 512 &&
                            L(1).ph[0].kpad == 1024 && L(2).ph[0].kpad == 1024;
        aa.w1 = (const bf16_t*)ws[0]; aa.w2 = (const bf16_t*)ws[1]; aa.w3 = (const bf16_t*)ws[2];
        aa.w4 = (const bf16_t*)ws[3]; aa.w5 = (const bf16_t*)ws[4];
        for (int i = 0; i < 5; ++i) { aa.sc[i] = L(i).scale; aa.sh[i] = L(i).shift; }
        aud_fused = shapes && !opt.no_audenc && aud_enc_supported(aa);
    }

    // The per-layer audio branch (prep + a_conv1..5 -> concat[0:3200]) shares no buffer with the video encoder until
    // the fusion dense: it runs on the context's side stream, forked from and joined back into s, so its short,
    // latency-bound kernels overlap the video encoder (the profiling path keeps one stream for per-stage events;
    // AVSE_SERIAL=1 forces it).  The fork waits for everything enqueued on s before this call.
    // The fused audio encoder runs on the caller's stream: beside the persistent video convolutions its 152-KB
    // workgroups hold whole CUs they wait for (measured: concurrent 2.377 ms vs serial 2.304 ms per step), and the
    // fork / join events alone cost ~25 us of idle GPU per step (rocprof trace).  (The side-stream option for it was
    // removed in round 3, as was tile_alt, v_conv2 / v_conv4 tiles walked last-first: both measured no gain.)
    const bool concurrent = ev == nullptr && !opt.serial && !aud_fused;
    hipStream_t sa = s;
    if (concurrent) {
        if (!c->side) {
            if (opt.side_prio) {
                int least = 0, greatest = 0;
                AVSE_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
                AVSE_HIP_CHECK(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, opt.side_prio == 1 ? least : greatest));
            } else {
                AVSE_HIP_CHECK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
            }
            AVSE_HIP_CHECK(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
            AVSE_HIP_CHECK(hipEventCreateWithFlags(&c->join, hipEventDisableTiming));
        }
        AVSE_HIP_CHECK(hipEventRecord(c->fork, s));
        AVSE_HIP_CHECK(hipStreamWaitEvent(c->side, c->fork, 0));
        sa = c->side;
    }
    if (aud_fused) {
        if ((rc = launch_aud_enc(aa, s))) return rc;
        for (int k = 0; k < 6; ++k)
            if ((rc = mark())) return rc;   // audio_prep (= the fused kernel), a_conv1..a_conv5
    }
    // split: a_conv1 on the vector ALUs from the audio input itself (conv.hip k_aconv1_split; no audio_prep copy)
    const bool a1_valu = split && !aud_fused && !opt.no_a1valu && L(0).w_f32 && L(0).def.cin == 1 && L(0).def.kind == CONV &&
                         L(0).def.cout == 64 && L(0).def.kh == 5 && L(0).def.kw == 5 && L(0).def.sh == L(0).def.sw;
    if (a1_valu) {
        const GpuLayer& G = L(0);
        const int pt = std::max((G.ho - 1) * G.def.sh + G.def.kh - G.def.hin, 0) / 2;
        const int pl = std::max((G.wo - 1) * G.def.sw + G.def.kw - G.def.win, 0) / 2;
        if ((rc = mark()) ||
            (rc = launch_aconv1_split(audio, G.w_f32, G.scale, G.shift, buf(B_A1), N, G.def.hin, G.def.win, G.ho, G.wo,
                                      G.def.kh, G.def.kw, G.def.sh, pt, pl, G.def.cout, rflag, 1u, kRangeAudioIn, sa)) ||
            (rc = mark()))
            return rc;
    }
    if (!aud_fused && !a1_valu && ((rc = launch_audio_prep(audio, buf(B_AIN), N * kMels * P.T, gdt, sa)) || (rc = mark()))) return rc;
    const int a_in[5] = {B_AIN, B_A1, B_A2, B_A3, B_A4};
    for (int i = a1_valu ? 1 : 0; i < 5 && !aud_fused; ++i) {
        const GpuLayer& G = L(i);
        const long long in_cs = (long long)G.def.hin * G.def.win * (i == 0 ? G.cin_pad : G.def.cin);
        ConvArgs a = (i < 4) ? conv_args(G, buf(a_in[i]), in_cs, buf(a_in[i + 1]), (long long)G.ho * G.wo * G.def.cout, G.def.cout, 0, N)
                             : conv_args(G, buf(a_in[i]), in_cs, buf(B_CAT), CAT, G.def.cout, 0, N);   // Flatten -> concat[0:aemb]
        const int dti = pairs(a, i > 0, true, i);   // a_conv1: fp32 audio-prep input
        if ((rc = conv(a, dti, G, sa)) || (rc = mark())) return rc;
    }
    if (concurrent) AVSE_HIP_CHECK(hipEventRecord(c->join, sa));
    if (video) {
        if ((rc = video_encoder(video, vmean, vstd, N, off, buf(B_CAT)))) return rc;
    } else {
        // all-zero video: broadcast the constant embedding computed above
        const size_t es = dt == AVSE_BF16 ? 2 : 4;
        if ((rc = launch_broadcast_row(W->vzero_emb.load(std::memory_order_acquire), (char*)buf(B_CAT) + AEMB * es, N, 2048 * es, CAT * es, s))) return rc;
        // an embedding that left the pair range reports it in every forward that broadcasts it
        if (split && W->vzero_range && rflag && (rc = launch_flag_or(rflag, W->vzero_range, s))) return rc;
        for (int k = 0; k < 6; ++k)
            if ((rc = mark())) return rc;   // v_conv1..v_conv6 stages (the broadcast shows as v_conv1)
    }
    if (concurrent) AVSE_HIP_CHECK(hipStreamWaitEvent(s, c->join, 0));
    // fusion + decoder dense (network.py:53-58, :66-78)
    if (use_gemm) {
        if ((rc = gemm(L(11), buf(B_CAT), CAT, buf(B_E1), EMB, 0, 0, N, off[B_COUNT], 11)) || (rc = mark())) return rc;
        if ((rc = gemm(L(12), buf(B_E1), EMB, buf(B_E2), EMB, 0, 0, N, off[B_COUNT], 12)) || (rc = mark())) return rc;
        if ((rc = gemm(L(13), buf(B_E2), EMB, buf(B_E3), AEMB, 0, 0, N, off[B_COUNT], 13)) || (rc = mark())) return rc;
    } else {
        ConvArgs a = conv_args(L(11), buf(B_CAT), CAT, buf(B_E1), EMB, EMB, 0, N);
        ksplit(a, off[B_COUNT]);
        int dti = pairs(a, true, true, 11);
        if ((rc = launch_conv(a, split ? dti : cdt, s)) || (rc = mark())) return rc;
        a = conv_args(L(12), buf(B_E1), EMB, buf(B_E2), EMB, EMB, 0, N);
        ksplit(a, off[B_COUNT]);
        dti = pairs(a, true, true, 12);
        if ((rc = launch_conv(a, split ? dti : cdt, s)) || (rc = mark())) return rc;
        a = conv_args(L(13), buf(B_E2), EMB, buf(B_E3), AEMB, AEMB, 0, N);
        ksplit(a, off[B_COUNT]);
        dti = pairs(a, true, true, 13);
        if ((rc = launch_conv(a, split ? dti : cdt, s)) || (rc = mark())) return rc;
    }
    // audio decoder (network.py:112-135)
    const int d_in[6] = {B_E3, B_D1, B_D2, B_D3, B_D4, B_D5};
    for (int i = 0; i < 5; ++i) {
        const GpuLayer& G = L(14 + i);
        const long long in_cs = (long long)G.def.hin * G.def.win * G.def.cin;
        if (i == 0 && dt == AVSE_BF16) {
            // d_deconv1 + d_deconv2 + d_deconv3 in one kernel, one workgroup per clip (conv_dech.hip): the layers
            // must have the network's shapes and sub-pixel tap grids (checked here)
            auto taps_ok = [&](const GpuLayer& D, int np, int nt, bool wide) {
                if (D.nphase != np || D.def.cin != 128 || D.def.cout != 128) return false;
                for (int p = 0; p < np; ++p) {
                    if (D.ph[p].ntaps != nt || D.ph[p].kpad != nt * 128 || D.ph[p].w_off != (long long)p * 128 * nt * 128) return false;
                    for (int t = 0; t < nt; ++t) {
                        const int2 d = D.htaps[D.ph[p].tap_off + t];
                        const int dy = wide ? (p >> 1) - (t >> 1) : 0, dx = wide ? (p & 1) - (t & 1) : -t;
                        if (d.x != dy || d.y != dx) return false;
                    }
                }
                return true;
            };
            const bool shapes = L(14).hq == 5 && L(14).wq == 5 && L(15).hq == 10 && L(15).wq == 5 && L(16).hq == 20 &&
                                L(16).wq == 5 && taps_ok(L(14), 2, 2, false) && taps_ok(L(15), 2, 2, false) &&
                                taps_ok(L(16), 4, 4, true);
            DecHeadArgs ha;
            std::memset(&ha, 0, sizeof(ha));
            ha.in = reinterpret_cast<const bf16_t*>(buf(B_E3));
            ha.in_clip_stride = AEMB;
            ha.out = reinterpret_cast<bf16_t*>(buf(B_D3));
            ha.out_clip_stride = 40 * 10 * 128;
            ha.N = (int)N;
            ha.w1 = (const bf16_t*)L(14).w; ha.w2 = (const bf16_t*)L(15).w; ha.w3 = (const bf16_t*)L(16).w;
            for (int k = 0; k < 3; ++k) { ha.sc[k] = L(14 + k).scale; ha.sh[k] = L(14 + k).shift; }
            if (shapes && !opt.no_dechead && dec_head_supported(ha)) {
                if ((rc = launch_dec_head(ha, s)) || (rc = mark()) || (rc = mark()) || (rc = mark())) return rc;
                i = 2;   // continue with d_deconv4
                continue;
            }
        }
        if (i == 3 && split && !opt.unfused_tail && !opt.no_dectail) {
            // d_deconv4 + d_deconv5 + d_deconv6 on split pairs, one workgroup per half clip (conv_dects.hip)
            DecTailArgs da = dec_tail_args(L(17), L(18), W, buf(d_in[3]), out, N);
            da.range_flag = rflag;
            da.range_bit = 1u << 17;
            if (dec_tail_s16_supported(da)) {
                if ((rc = launch_dec_tail_s16(da, s)) || (rc = mark()) || (rc = mark())) return rc;   // d4, d5 stages
                break;
            }
        }
        if (i == 3 && dt == AVSE_BF16 && !opt.unfused_tail && !opt.no_dectail) {
            // d_deconv4 + d_deconv5 + d_deconv6 in one kernel, one workgroup per clip (conv_dec.hip)
            const DecTailArgs da = dec_tail_args(L(17), L(18), W, buf(d_in[3]), out, N);
            if (dec_tail_supported(da)) {
                if ((rc = launch_dec_tail(da, s)) || (rc = mark()) || (rc = mark())) return rc;   // d4, d5 stages
                break;
            }
        }
        if (i == 4 && !opt.unfused_tail) {
            // d_deconv5 with d_deconv6 (1x1, 64 -> 1, network.py:133) fused into its epilogue: the 64-channel
            // [N, 80, 20] activation is never written; orow addresses the float output pixel directly
            ConvArgs a = conv_args(G, buf(d_in[i]), in_cs, nullptr, (long long)G.ho * G.wo, 1, 0, N);
            a.fuse_w = W->d6_w;
            a.fuse_bias = W->d6_bias;
            a.fuse_out = out;
            const int dti = pairs(a, true, false, 14 + i);
            if ((rc = conv(a, dti, G, s)) || (rc = mark())) return rc;
            continue;
        }
        ConvArgs a = conv_args(G, buf(d_in[i]), in_cs, buf(d_in[i + 1]), (long long)G.ho * G.wo * G.def.cout, G.def.cout, 0, N);
        const int dti = pairs(a, true, i < 4 || !opt.unfused_tail, 14 + i);   // an unfused d_deconv5 feeds launch_out_conv fp32
        if ((rc = conv(a, dti, G, s)) || (rc = mark())) return rc;
    }
    if (opt.unfused_tail) {
        if ((rc = launch_out_conv(buf(B_D5), W->d6_w, W->d6_bias, out, N * kMels * P.T, gdt, s)) || (rc = mark())) return rc;
    } else if ((rc = mark())) {   // d_deconv6: fused into d_deconv5 above
        return rc;
    }
    return 0;
}
}  // namespace

extern "C" {

// avse_forward replays a hipGraph of the forward once the same arguments (weights, input / output pointers, N, the
// context's scratch arena and its Options) come a second time: the first call launches directly,
// the second captures and launches the graph, later ones replay it — the ~15 kernels then run without the per-kernel
// dispatch gaps of stream launches.  The graph bakes the pointers in; every argument set has its own entry (at most 8
// are kept).  Opt-in (AVSE_GRAPH=1): a torch graph of the whole bench step (spectrogram + forward) measured 2.20 ->
// 2.14 ms (tools/graph_probe.py), but replaying the forward alone inside the same step measured 2.234 vs 2.24-2.26 ms
// direct (bench.py A/B, same box), so direct launches stay the default.
static int forward_dispatch(avse_ctx* c, const avse_weights* W, const float* audio, const float* video,
                            const float* vmean, const float* vstd, int64_t N, float* out, void* stream,
                            unsigned* rflag);

int avse_forward(avse_ctx* c, const avse_weights* W, const float* audio, const float* video, const float* vmean,
                 const float* vstd, int64_t N, float* out, void* stream) {
    if (int rc = forward_dispatch(c, W, audio, video, vmean, vstd, N, out, stream, c ? c->range : nullptr)) return rc;
    return avse::debug_poll(stream);
}

int avse_range_status(avse_ctx* c, void* stream, uint32_t* host_bits) {
    if (!c || !host_bits) return fail(AVSE_ERR_INVALID, "NULL argument");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    AVSE_HIP_CHECK(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) return fail(AVSE_ERR_INVALID, "avse_range_status waits for its stream: not inside a capture");
    AVSE_HIP_CHECK(hipMemcpyAsync(c->range_host, c->range, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    AVSE_HIP_CHECK(hipMemsetAsync(c->range, 0, sizeof(unsigned), s));
    AVSE_HIP_CHECK(hipStreamSynchronize(s));
    *host_bits = c->range_host[0];
    return 0;
}

int avse_range_snapshot(avse_ctx* c, void* stream, uint32_t* host_word) {
    if (!c || !host_word) return fail(AVSE_ERR_INVALID, "NULL argument");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    AVSE_HIP_CHECK(hipMemcpyAsync(host_word, c->range, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    AVSE_HIP_CHECK(hipMemsetAsync(c->range, 0, sizeof(unsigned), s));
    return 0;
}

int avse_forward_checked(avse_ctx* c, const avse_weights* W, const float* audio, const float* video, const float* vmean,
                         const float* vstd, int64_t N, float* out, void* stream, int mode, uint32_t* host_bits) {
    if (host_bits) *host_bits = 0;
    if (!c || !W) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (mode != AVSE_RANGE_RECOMPUTE && mode != AVSE_RANGE_ERROR) return fail(AVSE_ERR_INVALID, "bad range mode");
    if (W->dtype != AVSE_F32_SPLIT || N <= 0) return avse_forward(c, W, audio, video, vmean, vstd, N, out, stream);
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    AVSE_HIP_CHECK(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone)
        return fail(AVSE_ERR_INVALID, "avse_forward_checked waits for its stream: capture avse_forward instead");
    unsigned* flag = c->range + 1;
    AVSE_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(unsigned), s));
    // (option graph: the forward itself replays its hipGraph, so the launches after each wait are one graph launch)
    if (int rc = forward_dispatch(c, W, audio, video, vmean, vstd, N, out, stream, flag)) return rc;
    AVSE_HIP_CHECK(hipMemcpyAsync(c->range_host + 1, flag, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    AVSE_HIP_CHECK(hipStreamSynchronize(s));
    const unsigned bits = c->range_host[1];
    if (host_bits) *host_bits = bits;
    if (!bits) return avse::debug_poll(stream);
    if (mode == AVSE_RANGE_ERROR)
        return fail(AVSE_ERR_RANGE, "AVSE_F32_SPLIT: an activation left the f16 pair range (range bits 0x" +
                                        [](unsigned b) { char t[16]; std::snprintf(t, sizeof(t), "%x", b); return std::string(t); }(bits) +
                                        "): the outputs are not float32-accurate");
    // recompute the batch on the exact-fp32 network (the same kernels as AVSE_F32 weights), built once from the blob
    const avse_weights* twin = nullptr;
    {
        std::lock_guard<std::mutex> lk(W->twin_mu);
        if (!W->f32_twin) {
            avse_weights* t = nullptr;
            if (int rc = avse_weights_load_shape(c, W->blob.data(), (int64_t)W->blob.size(), AVSE_F32, W->plan.T, W->plan.F, &t))
                return rc;
            W->f32_twin = t;
        }
        twin = W->f32_twin;
    }
    if (int rc = forward_impl(c, twin, audio, video, vmean, vstd, N, out, s, nullptr, nullptr)) return rc;
    return avse::debug_poll(stream);
}

static int forward_dispatch(avse_ctx* c, const avse_weights* W, const float* audio, const float* video,
                            const float* vmean, const float* vstd, int64_t N, float* out, void* stream,
                            unsigned* rflag) {
    if (!c || !W || N <= 0 || !c->opt.graph)
        return forward_impl(c, W, audio, video, vmean, vstd, N, out, (hipStream_t)stream, nullptr, rflag);
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    if (W->device != c->device) return fail(AVSE_ERR_INVALID, "weights and context are on different devices");
    int rc = ensure_arena(c, N, W->dtype, W->plan, (hipStream_t)stream);   // no allocation inside the capture
    if (rc) return rc;
    const void* key[9] = {(const void*)W->serial, audio, video, vmean, vstd, out, c->arena, (const void*)c->arena_bytes,
                          rflag};
    avse_ctx::Graph* hit = nullptr;
    for (auto& g : c->graphs)
        if (g.n == N && std::memcmp(&g.opt, &c->opt, sizeof(Options)) == 0 && std::memcmp(g.key, key, sizeof(key)) == 0)
            hit = &g;
    if (hit && hit->exec) {
        AVSE_HIP_CHECK(hipGraphLaunch(hit->exec, (hipStream_t)stream));
        return 0;
    }
    auto evict = [&] {
        if (c->graphs.size() < 8) return;
        if (c->graphs.front().exec) (void)hipGraphExecDestroy(c->graphs.front().exec);
        c->graphs.erase(c->graphs.begin());
    };
    if (!hit) {   // first sighting of this argument set: launch directly (a one-off call pays no capture)
        evict();
        avse_ctx::Graph g;
        std::memcpy(g.key, key, sizeof(key));
        g.n = N;
        g.opt = c->opt;
        g.exec = nullptr;
        c->graphs.push_back(g);
        return forward_impl(c, W, audio, video, vmean, vstd, N, out, (hipStream_t)stream, nullptr, rflag);
    }
    if (!c->cap) AVSE_HIP_CHECK(hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking));
    AVSE_HIP_CHECK(hipStreamBeginCapture(c->cap, hipStreamCaptureModeRelaxed));
    rc = forward_impl(c, W, audio, video, vmean, vstd, N, out, c->cap, nullptr, rflag);
    hipGraph_t graph = nullptr;
    const hipError_t ce = hipStreamEndCapture(c->cap, &graph);
    if (rc || ce != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc ? rc : fail(AVSE_ERR_HIP, std::string("forward capture: ") + hipGetErrorString(ce));
    }
    hipGraphExec_t exec = nullptr;
    const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ie != hipSuccess) return fail(AVSE_ERR_HIP, std::string("forward graph instantiate: ") + hipGetErrorString(ie));
    hit->exec = exec;
    AVSE_HIP_CHECK(hipGraphLaunch(exec, (hipStream_t)stream));
    return 0;
}

int avse_forward_profile(avse_ctx* c, const avse_weights* W, const float* audio, const float* video,
                         const float* vmean, const float* vstd, int64_t N, float* out, void* stream, float* host_ms) {
    if (!host_ms) return fail(AVSE_ERR_INVALID, "host_ms is NULL");
    if (c) AVSE_HIP_CHECK(hipSetDevice(c->device));
    hipEvent_t ev[AVSE_NUM_STAGES + 1];
    for (int i = 0; i <= AVSE_NUM_STAGES; ++i) AVSE_HIP_CHECK(hipEventCreate(&ev[i]));
    int rc = forward_impl(c, W, audio, video, vmean, vstd, N, out, (hipStream_t)stream, ev, c ? c->range : nullptr);
    if (!rc) {
        AVSE_HIP_CHECK(hipEventSynchronize(ev[AVSE_NUM_STAGES]));
        for (int i = 0; i < AVSE_NUM_STAGES; ++i) {
            float ms = 0.f;
            AVSE_HIP_CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            host_ms[i] = ms;
        }
    }
    for (int i = 0; i <= AVSE_NUM_STAGES; ++i) (void)hipEventDestroy(ev[i]);
    return rc;
}

int avse_video_normalize(avse_ctx* c, float* video, int64_t S, int H, int W, int F, const float* mean,
                         const float* stdv, void* stream) {
    if (!c || !video || !mean || !stdv) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (S < 0 || H <= 0 || W <= 0 || F <= 0) return fail(AVSE_ERR_INVALID, "bad video shape");
    if (S == 0) return 0;
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    return launch_video_normalize(video, S, H, W, F, mean, stdv, (hipStream_t)stream);
}

int avse_mse(avse_ctx* c, const float* pred, const float* target, int64_t n, float* loss, void* stream) {
    if (!c || !pred || !target || !loss) return fail(AVSE_ERR_INVALID, "NULL argument");
    if (n <= 0) return fail(AVSE_ERR_INVALID, "n must be positive");
    AVSE_HIP_CHECK(hipSetDevice(c->device));
    return launch_mse(pred, target, n, loss, c->mse_partial, (hipStream_t)stream);
}

int avse_debug_scratch(avse_ctx* c, int64_t N, int dtype, void** base, int64_t* offsets) {
    if (!c || !base || !offsets || N <= 0) return fail(AVSE_ERR_INVALID, "bad debug_scratch args");
    size_t off[B_COUNT + 1];
    const size_t need = arena_bytes(N, dtype, c->opt, off, c->last_plan);
    if (!c->arena || need > c->arena_bytes) return fail(AVSE_ERR_INVALID, "no forward scratch of that size yet");
    *base = c->arena;
    for (int b = 0; b < B_COUNT; ++b) offsets[b] = (int64_t)off[b];
    return 0;
}

}  // extern "C"
