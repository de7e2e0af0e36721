// Fused audio encoder, one workgroup per clip (bf16, gfx950): network.py:88-109
//   a_conv1  Conv2D(64, 5x5, strides 2, 'same')      80 x 20 x 1  -> 40 x 10 x 64
//   a_conv2  Conv2D(64, 4x4, 'same')                  40 x 10 x 64 -> 40 x 10 x 64
//   a_conv3  Conv2D(128, 4x4, strides 2, 'same')      40 x 10 x 64 -> 20 x 5 x 128
//   a_conv4  Conv2D(128, 2x2, strides (2, 1), 'same') 20 x 5 x 128 -> 10 x 5 x 128
//   a_conv5  Conv2D(128, 2x2, strides (2, 1), 'same') 10 x 5 x 128 ->  5 x 5 x 128 -> Flatten -> concat[0:3200]
// each followed by BatchNormalization + LeakyReLU(0.3); activations rounded to bf16 between layers exactly as the
// layer-by-layer path stores them.
//
// Why: layer by layer these are six short launches (~0.18 ms per 512 clips: a_conv1 0.65 GFLOP in 32 us, a_conv4 /
// a_conv5 ~21 us each for 1.7-3.4 GFLOP) and, run on the side stream next to the video encoder, they hold CUs the
// persistent video convolutions wait for.  The recipe of the fused decoder tail (conv_dec.hip): a clip's activations
// stay in LDS, weights stream through an LDS ring of slab groups (one barrier per group), geometry is
// compile-time so every fragment read is a ds_read_b128 at a per-lane base + immediate.
//   * a_conv1 (one input channel): the 400 x 32 im2col tile (25 taps + 7 zeros) is built in LDS from the f32
//     mel input (the audio_prep kernel disappears); one K slab;
//   * a_conv2: input image = two 43 x 14-pixel chunk buffers of 96-B rows with 8 x 2-pixel M fragments
//     (bank-conflict free, as d_deconv4); 32 slabs, 16 MFMAs per wave per slab;
//   * a_conv3..a_conv5: zero-padded images of 160-B (64 channels) / 288-B (128 channels) rows, 16-pixel M
//     fragments; waves split the 128 output channels;
//   * 8 waves (two per SIMD).
#include <cstdlib>
#include <utility>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr int NW = 8, NT = 64 * NW;
// a_conv2 input: 2 chunk buffers, 43 rows x 14 pixels x 96 B; pixel (y + ky, x + kx) for output (y, x), tap (ky, kx)
constexpr int P2 = 14, S2 = 96, W2BUF = 43 * P2 * S2;                 // 57,792
// a_conv3 input: 42 x 13 x 144 B (64 channels + pad); pixel (2 y + ky, 2 x + kx).  a_conv3..a_conv5 gather their
// 16-pixel M fragments from a 5-wide grid (stride 2 rows / columns): the pixel and row pitches are the ones with the
// fewest ds_read_b128 bank conflicts over every tap (searched exhaustively, 16-lane groups of 16-B units; a_conv3
// 2.9-way at 160 B x 14 -> 1.1-way at 144 B x 13, a_conv4 2.8 -> 1.8-way at 7 pixels per row)
constexpr int P3 = 13, S3 = 144, IMG3B = 42 * P3 * S3;                // 78,624
// a_conv4 / a_conv5 inputs: 20 (10) rows x 7 pixels x 288 B (128 channels + pad); pixel (2 y + ky, x + kx)
constexpr int P4 = 7, S4 = 288, IMG4B = 20 * P4 * S4;                 // 40,320
constexpr int IMG5 = 40960, IMG5B = 10 * P4 * S4;                     // 20,160
constexpr int BOFF = 2 * W2BUF;                                       // weight ring (2 x 16 KB); a_conv1's im2col
constexpr int PAR = BOFF + 2 * 16384;                                 // folded bias / BN of the five layers (f32)
constexpr int PSC[5] = {PAR, PAR + 512, PAR + 1024, PAR + 2048, PAR + 3072};   // scale of layer l; shift at + 4 * Cout
constexpr int MEL = PAR + 4096, MP = 24;                              // a_conv1 input: zero-padded 83 x 24 bf16
constexpr int LDS_BYTES = MEL + 83 * MP * 2;                          // 156,432
constexpr int DA = 6;                                                 // a_conv3..5 weight pieces in flight (registers)
static_assert(IMG3B <= BOFF && IMG4B <= IMG5 && IMG5 + IMG5B <= BOFF && 400 * 64 <= 32768, "LDS map");

typedef int i32x2 __attribute__((ext_vector_type(2)));
struct Pre { i32x4 w[DA + 2]; };   // a layer's first DA + 2 weight pieces (see prefetch)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int wsw(int row) { return 2 * ((row >> 2) & 1); }
__device__ __forceinline__ i32x4 lds16(const char* base, int off) { return *reinterpret_cast<const i32x4*>(base + off); }
template <int... I, typename F>
__device__ __forceinline__ void unroll(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}
__device__ __forceinline__ float bn_lrelu(float acc, float sc, float sh) {
    const float v = fmaf(acc, sc, sh);
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(LRELU * v));   // LeakyReLU, no canonicalise
    return r;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// BN + LeakyReLU of an accumulator quad (4 consecutive channels) -> 4 bf16 (RNE, as (bf16_t) casts)
__device__ __forceinline__ i32x2 bn_pack4(f32x4 v, f32x4 sc, f32x4 sh) {
    const float a = bn_lrelu(v[0], sc[0], sh[0]), b = bn_lrelu(v[1], sc[1], sh[1]);
    const float c = bn_lrelu(v[2], sc[2], sh[2]), d = bn_lrelu(v[3], sc[3], sh[3]);
    const bf16x2 lo = __builtin_convertvector((f32x2){a, b}, bf16x2), hi = __builtin_convertvector((f32x2){c, d}, bf16x2);
    return (i32x2){__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi)};
}
__device__ __forceinline__ f32x4 mfma(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// STAMP (tools/aud_stamp.hip only; 0 in the library): thread 0 records s_memtime at the phase boundaries into
// g_stamps[block][k] (k = 0 start, 1 im2col, 2 a_conv1, 3 a_conv2 prologue, 4 a_conv2 loop, 5 its epilogue, 6 a_conv3
// loop, 7 its epilogue, 8 a_conv4, 9 a_conv5; 10 / 11 the end of the a_conv4 / a_conv5 slab loops)
[[maybe_unused]] __device__ unsigned long long* g_stamps;
template <int STAMP = 0>
__global__ __launch_bounds__(NT, 1) void k_aud_enc(AudEncArgs a) {
#define STAMP_AT(k) \
    do { if constexpr (STAMP != 0) { if (threadIdx.x == 0) g_stamps[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
    STAMP_AT(0);
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int clip = blockIdx.x;
    auto st16 = [&](int addr, i32x4 v) { *reinterpret_cast<i32x4*>(lds + addr) = v; };
    auto zero = [&](int from, int to) {
        for (int o = from + tid * 16; o < to; o += NT * 16) st16(o, (i32x4){0, 0, 0, 0});
    };

    // every layer's folded bias / BN -> LDS (read as f32x4 quads in the epilogues: lanes of a row group kg share
    // an address, so the reads broadcast)
    {
        constexpr int co[5] = {64, 64, 128, 128, 128};
#pragma unroll
        for (int l = 0; l < 5; ++l)
            if (tid < 2 * co[l])
                reinterpret_cast<float*>(lds + PSC[l])[tid] = tid < co[l] ? a.sc[l][tid] : a.sh[l][tid - co[l]];
    }
    // scale / shift quad of layer l for channels n .. n + 3
    auto bnq = [&](int l, int n, f32x4& sc, f32x4& sh) {
        constexpr int co[5] = {64, 64, 128, 128, 128};
        sc = *reinterpret_cast<const f32x4*>(lds + PSC[l] + n * 4);
        sh = *reinterpret_cast<const f32x4*>(lds + PSC[l] + (co[l] + n) * 4);
    };
    auto st8l = [&](int addr, i32x2 v) { *reinterpret_cast<i32x2*>(lds + addr) = v; };

    // ================= a_conv1: 5x5 stride 2 on the single mel channel =================
    // weights (global) first; the mel clip -> a zero-padded 83 x 24 bf16 image in LDS (TF 'SAME': 1 row / column
    // before, 2 after); each lane gathers its A fragment rows (k = ky * 5 + kx, 25 of 32) straight from the image
    // (the first version built a 400 x 32 im2col tile with 32 scalar global loads per lane: 11K cycles)
    i32x4 fb1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb1[j] = *reinterpret_cast<const i32x4*>(reinterpret_cast<const char*>(a.w1) + ((16 * j + r16) * 32 + kg * 8) * 2);
    const f32x4 mv = tid < 400 ? *reinterpret_cast<const f32x4*>(a.mel + (long long)clip * 1600 + 4 * tid) : (f32x4){};
    zero(0, BOFF);   // a_conv2's input image: its padding ring reads as zero
    zero(MEL, MEL + 83 * MP * 2);
    __syncthreads();
    if (tid < 400) {
        const int iy = tid / 5, ix = 4 * (tid - 5 * iy);
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16_t*>(lds + MEL + ((iy + 1) * MP + ix + 1 + q) * 2) = (bf16_t)mv[q];
    }
    __syncthreads();
    STAMP_AT(1);
    {
        int toff[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int tap = 8 * kg + e, ky = tap / 5, kx = tap - 5 * ky;
            toff[e] = tap < 25 ? (ky * MP + kx) * 2 : -1;
        }
        // M fragment f = rows 16 f .. 16 f + 15 of the 40 x 10 grid; slot i = fragment w + 8 i
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = (w + 8 * i < 25) ? w + 8 * i : 0;
            const int m = 16 * f + r16, oy = m / 10, ox = m - oy * 10;
            const char* const base = lds + MEL + (2 * oy * MP + 2 * ox) * 2;
            unsigned v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = toff[e] >= 0 ? *reinterpret_cast<const unsigned short*>(base + toff[e]) : 0u;
            const i32x4 fa = {(int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)), (int)(v[4] | (v[5] << 16)),
                              (int)(v[6] | (v[7] << 16))};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fb1[j], fa, (f32x4){0.f, 0.f, 0.f, 0.f});   // W x A
        }
        // -> a_conv2's input: chunk (n / 32) buffer, padded pixel (oy + 1, ox + 1); lane = pixel row r16,
        // channels 16 j + 4 kg .. + 3 (scale / shift quads read once per j: the stores in between are LDS stores,
        // so the compiler could not reuse the reads)
        f32x4 sc[4], sh[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bnq(0, 16 * j + 4 * kg, sc[j], sh[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = w + 8 * i;
            if (f >= 25) continue;
            const int m = 16 * f + r16, oy = m / 10, ox = m - oy * 10;
            const int px = ((oy + 1) * P2 + ox + 1) * S2 + kg * 8;
#pragma unroll
            for (int j = 0; j < 4; ++j) st8l(px + (j >> 1) * W2BUF + (j & 1) * 32, bn_pack4(acc[i][j], sc[j], sh[j]));
        }
    }
    __syncthreads();
    STAMP_AT(2);

    // ================= a_conv3..a_conv5: 128 output channels, one 16-channel slice per wave =================
    // A wave owns output channels 16 w .. 16 w + 15 and every M fragment of the layer, so no two waves use the same
    // weights: each wave loads its B fragments (16 rows x 64 B per 32-deep slab) straight from global memory DA + 2
    // slabs ahead, and the loop has no LDS weight ring and no barrier.  A fragments come from the LDS image, read
    // two slabs ahead.  (With an LDS ring shared by waves that split M and N, a_conv3..a_conv5 ran at 20-40 % of
    // the MFMA rate: 2-8 MFMAs per slab could not cover a barrier every two slabs.)
    const __amdgpu_buffer_rsrc_t rsW3 = make_rsrc(a.w3, 128 * 1024 * 2), rsW4 = make_rsrc(a.w4, 128 * 512 * 2),
                                 rsW5 = make_rsrc(a.w5, 128 * 512 * 2);
    auto bsoff3 = [](auto ss) { constexpr int S = decltype(ss)::value; return (S % 16) * 128 + (S / 16) * 64; };
    auto bsoff45 = [](auto ss) { constexpr int S = decltype(ss)::value; return (S % 4) * 256 + (S / 4) * 64; };
    // a layer's first DA + 2 B fragments of this wave (weight row 16 w + r16 of rowb bytes, k-group kg)
    auto prefetch_direct = [&](const __amdgpu_buffer_rsrc_t& rsW, int rowb, auto bsoff) {
        const int vbw = (16 * w + r16) * rowb + kg * 16;
        Pre p;
        unroll(std::make_integer_sequence<int, DA + 2>{}, [&](auto k) {
            p.w[decltype(k)::value] = __builtin_amdgcn_raw_buffer_load_b128(rsW, vbw + bsoff(k), 0, 0);
        });
        return p;
    };
    // the slab loop: NFR M fragments at LDS bases vb[i] + aimm(slab); acc = the 16 x (16 NFR) tile (W x A)
    auto direct = [&](auto nff, auto nss, const __amdgpu_buffer_rsrc_t& rsW, int rowb, auto bsoff, auto aimm, const int* vb,
                      const Pre& pre, f32x4* acc) {
        constexpr int NFR = decltype(nff)::value, NS = decltype(nss)::value, DB = DA + 2, RA = NFR >= 7 ? 3 : 4;
        const int vbw = (16 * w + r16) * rowb + kg * 16;
        i32x4 fa[RA][NFR], pb[DB];
#pragma unroll
        for (int k = 0; k < DB; ++k) pb[k] = pre.w[k];
        auto read_a = [&](auto ss) {
            constexpr int S = decltype(ss)::value;
            if constexpr (S < NS) {
                const int imm = aimm(ss);
#pragma unroll
                for (int i = 0; i < NFR; ++i) fa[S % RA][i] = lds16(lds + imm, vb[i]);
            }
        };
        unroll(std::make_integer_sequence<int, RA - 1>{}, [&](auto k) { read_a(k); });
        unroll(std::make_integer_sequence<int, NS>{}, [&](auto ss) {
            constexpr int S = decltype(ss)::value;
            __builtin_amdgcn_sched_barrier(0);   // the reads of slab S + RA - 1 go out ahead of slab S's MFMAs
            const i32x4 fb = pb[S % DB];
            if constexpr (S + DB < NS)
                pb[S % DB] = __builtin_amdgcn_raw_buffer_load_b128(rsW, vbw + bsoff(std::integral_constant<int, S + DB>{}), 0, 0);
            read_a(std::integral_constant<int, S + RA - 1>{});
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < NFR; ++i) acc[i] = mfma(fb, fa[S % RA][i], S == 0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i]);
        });
    };
    Pre pre3{}, pre4{}, pre5{};

    // ================= a_conv2: 4x4, 64 -> 64 on 40 x 10 (slab = chunk * 16 + tap) =================
    {
        // weight slabs (64 rows x 64 B = 4 KB) through the ring in groups of 4: lane moves 8 B per slab
        const int brow = tid >> 3, kq = (tid >> 1) & 3, kh = tid & 1;
        const int bst = BOFF + brow * 64 + ((kq ^ wsw(brow)) << 4) + kh * 8;   // + slot 16384 + pos 4096
        const int bfr = BOFF + r16 * 64 + ((kg ^ wsw(r16)) << 4);              // + slot 16384 + pos 4096 + 1024 j
        const __amdgpu_buffer_rsrc_t rsW = make_rsrc(a.w2, 64 * 1024 * 2);
        const int vbl = brow * 2048 + kq * 16 + kh * 8;
        auto bpiece = [&](auto tt, int csoff) {   // slab (chunk, tap t): k = t * 64 + chunk * 32
            return __builtin_amdgcn_raw_buffer_load_b64(rsW, vbl + decltype(tt)::value * 128, csoff, 0);
        };
        auto st8 = [&](int addr, i32x2 v) { *reinterpret_cast<i32x2*>(lds + addr) = v; };
        // fragment slots: 0..2 = fragments w, w + 8, w + 16 x all 64 channels; 3 = fragment 24 x channels 16 w .. + 15
        // on waves 0..3 (100 fragment pairs, 13 / 12 per wave, instead of 4 x 4 slots with 28 pairs dropped)
        const bool xw = w < 4;
        int vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = i < 3 ? w + 8 * i : 24;
            const int y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
            vb[i] = (y * P2 + x) * S2 + kg * 16;
        }
        i32x2 pb[4];
        {
            i32x2 w0[4];
            unroll(std::make_integer_sequence<int, 4>{}, [&](auto tt) {
                constexpr int t = decltype(tt)::value;
                w0[t] = bpiece(tt, 0);
                pb[t] = bpiece(std::integral_constant<int, t + 4>{}, 0);
            });
#pragma unroll
            for (int t = 0; t < 4; ++t) st8(bst + t * 4096, w0[t]);
        }
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        STAMP_AT(3);
        i32x4 fa[2][4], fb[2][4], fbx[2];
        int vq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) vq[i] = vb[i];
        auto read_a = [&](auto tt, i32x4 (&f)[4]) {
            constexpr int t = decltype(tt)::value % 16;
            constexpr int imm = ((t / 4) * P2 + t % 4) * S2;
#pragma unroll
            for (int i = 0; i < 3; ++i) f[i] = lds16(lds + imm, vq[i]);
            if (xw) f[3] = lds16(lds + imm, vq[3]);
        };
        auto read_b = [&](int base, i32x4 (&f)[4], i32x4& fx) {
#pragma unroll
            for (int j = 0; j < 4; ++j) f[j] = lds16(lds, base + 1024 * j);
            if (xw) fx = lds16(lds, base + 1024 * w);
        };
        read_a(std::integral_constant<int, 0>{}, fa[0]);
        read_b(bfr, fb[0], fbx[0]);
        for (int c = 0; c < 2; ++c) {
            const int cs = c * 64, cn = (c + 1 < 2 ? c + 1 : 0) * 64;
            unroll(std::make_integer_sequence<int, 16>{}, [&](auto tt) {
                constexpr int t = decltype(tt)::value;
                __builtin_amdgcn_sched_barrier(0);
                st8(bst + (((t / 4) + 1) & 1) * 16384 + (t % 4) * 4096, pb[t & 3]);   // slab S + 4
                if constexpr (t + 8 < 16) pb[t & 3] = bpiece(std::integral_constant<int, t + 8>{}, cs);   // slab S + 8
                else pb[t & 3] = bpiece(std::integral_constant<int, t + 8 - 16>{}, cn);
                if constexpr (t % 4 == 3) __syncthreads();
                if constexpr (t == 15) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) vq[i] = vb[i] + (c + 1) * W2BUF;   // past the last chunk: unused reads
                }
                read_a(std::integral_constant<int, t + 1>{}, fa[(t + 1) & 1]);
                read_b(bfr + (((t + 1) / 4) & 1) * 16384 + ((t + 1) % 4) * 4096, fb[(t + 1) & 1], fbx[(t + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fb[t & 1][j], fa[t & 1][i], acc[i][j]);   // W x A
                if (xw) acc[3][0] = mfma(fbx[t & 1], fa[t & 1][3], acc[3][0]);
            });
        }
        __syncthreads();   // every read of a_conv2's input done: a_conv3's image goes over it
        STAMP_AT(4);
        pre3 = prefetch_direct(rsW3, 2048, bsoff3);   // a_conv3's first weight fragments load under this epilogue
        zero(0, IMG3B);
        __syncthreads();
        // -> a_conv3's input, padded pixel (oy + 1, ox + 1), 8 x 2 fragment rows; lane = fragment row r16
        f32x4 sc[4], sh[4], scx, shx;   // per channel block (read once; see a_conv1)
#pragma unroll
        for (int j = 0; j < 4; ++j) bnq(1, 16 * j + 4 * kg, sc[j], sh[j]);
        bnq(1, 16 * (w & 3) + 4 * kg, scx, shx);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i == 3 && !xw) continue;
            const int f = i < 3 ? w + 8 * i : 24;
            const int y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
            const int px = ((y + 1) * P3 + x + 1) * S3 + kg * 8;
            if (i < 3) {
#pragma unroll
                for (int j = 0; j < 4; ++j) st8l(px + 32 * j, bn_pack4(acc[i][j], sc[j], sh[j]));
            } else {
                st8l(px + 32 * w, bn_pack4(acc[3][0], scx, shx));   // channel block w
            }
        }
        __syncthreads();
        STAMP_AT(5);
    }

    // ---- a_conv3: 4x4 stride 2, 64 -> 128, 40 x 10 -> 20 x 5 (100 rows, 7 fragments); slab = chunk * 16 + tap ----
    {
        int vb[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int m = (16 * i + r16 < 100) ? 16 * i + r16 : 0;
            const int oy = m / 5, ox = m - oy * 5;
            vb[i] = (2 * oy * P3 + 2 * ox) * S3 + kg * 16;
        }
        f32x4 acc[7];
        direct(std::integral_constant<int, 7>{}, std::integral_constant<int, 32>{}, rsW3, 2048, bsoff3, [](auto ss) {
            constexpr int S = decltype(ss)::value, t = S % 16, c = S / 16;
            return ((t / 4) * P3 + t % 4) * S3 + c * 64;
        }, vb, pre3, acc);
        __syncthreads();   // every read of a_conv3's input done: a_conv4's image goes over it
        STAMP_AT(6);
        pre4 = prefetch_direct(rsW4, 1024, bsoff45);   // a_conv4's first weight fragments load under this epilogue
        zero(0, IMG4B);   // a_conv4's input: column 5 reads as zero
        __syncthreads();
        const int n = 16 * w + 4 * kg;   // lane channels n .. n + 3
        f32x4 sc, sh;
        bnq(2, n, sc, sh);
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int m = 16 * i + r16;
            if (m >= 100) continue;
            const int oy = m / 5, ox = m - oy * 5;
            st8l((oy * P4 + ox) * S4 + n * 2, bn_pack4(acc[i], sc, sh));
        }
        __syncthreads();
        STAMP_AT(7);
    }

    // ---- a_conv4 / a_conv5: 2x2 stride (2, 1), 128 -> 128; slab = chunk * 4 + tap ----
    auto small = [&](auto nff, int img, const __amdgpu_buffer_rsrc_t& rsW, const Pre& pre, int layer, auto store,
                     auto next) {
        constexpr int NFR = decltype(nff)::value;   // M fragments (4: 50 rows, 2: 25 rows)
        constexpr int MR = NFR == 4 ? 50 : 25;
        // fragment row m -> output (oy, ox): column-major on a_conv4's 10 x 5 grid (1.5-way bank conflicts
        // against 1.75 row-major), row-major on a_conv5's 5 x 5
        auto grid = [](int m, int& oy, int& ox) {
            if constexpr (NFR == 4) { ox = m / 10; oy = m - ox * 10; } else { oy = m / 5; ox = m - oy * 5; }
        };
        int vb[NFR];
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            const int m = (16 * i + r16 < MR) ? 16 * i + r16 : 0;
            int oy, ox;
            grid(m, oy, ox);
            vb[i] = img + (2 * oy * P4 + ox) * S4 + kg * 16;
        }
        f32x4 acc[NFR];
        direct(nff, std::integral_constant<int, 16>{}, rsW, 1024, bsoff45, [](auto ss) {
            constexpr int S = decltype(ss)::value, t = S % 4, c = S / 4;
            return ((t / 2) * P4 + t % 2) * S4 + c * 64;
        }, vb, pre, acc);
        STAMP_AT(10 + (NFR == 2));
        next();   // the next layer's first weight fragments load under this epilogue
        const int n = 16 * w + 4 * kg;   // lane channels n .. n + 3
        f32x4 sc, sh;
        bnq(layer, n, sc, sh);
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            const int m = 16 * i + r16;
            int oy, ox;
            grid(m, oy, ox);
            if (m < MR) store(oy, ox, n, bn_pack4(acc[i], sc, sh));
        }
        __syncthreads();
        STAMP_AT(8 + (NFR == 2));
    };
    zero(IMG5, IMG5 + IMG5B);   // a_conv5's input: column 5 reads as zero (ordered by the barriers in `small`)
    small(std::integral_constant<int, 4>{}, 0, rsW4, pre4, 3, [&](int oy, int ox, int n, i32x2 v) {
        st8l(IMG5 + (oy * P4 + ox) * S4 + n * 2, v);
    }, [&] { pre5 = prefetch_direct(rsW5, 1024, bsoff45); });
    bf16_t* const outc = a.out + (long long)clip * a.out_clip_stride;
    small(std::integral_constant<int, 2>{}, IMG5, rsW5, pre5, 4, [&](int oy, int ox, int n, i32x2 v) {
        *reinterpret_cast<i32x2*>(outc + (oy * 5 + ox) * 128 + n) = v;   // Flatten (HWC) -> concat[0:3200]
    }, [] {});
}

}  // namespace

#undef STAMP_AT

bool aud_enc_supported(const AudEncArgs& a) {
    return a.N > 0 && a.w1 && a.w2 && a.w3 && a.w4 && a.w5;
}

int launch_aud_enc(const AudEncArgs& a, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_aud_enc<0>, LDS_BYTES)) return rc;
    hipLaunchKernelGGL(k_aud_enc<0>, dim3(a.N), dim3(NT), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
