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
// a_conv3 input: 42 x 14 x 160 B (64 channels + pad); pixel (2 y + ky, 2 x + kx)
constexpr int P3 = 14, S3 = 160, IMG3B = 42 * P3 * S3;                // 94,080
// a_conv4 / a_conv5 inputs: 20 (10) rows x 6 pixels x 288 B (128 channels + pad); pixel (2 y + ky, x + kx)
constexpr int P4 = 6, S4 = 288, IMG4B = 20 * P4 * S4;                 // 34,560
constexpr int IMG5 = 40960, IMG5B = 10 * P4 * S4;                     // 17,280
constexpr int BOFF = 2 * W2BUF;                                       // weight ring (2 x 16 KB); a_conv1's im2col
constexpr int PAR = BOFF + 2 * 16384;                                 // folded bias / BN of the five layers (f32)
constexpr int PSC[5] = {PAR, PAR + 512, PAR + 1024, PAR + 2048, PAR + 3072};   // scale of layer l; shift at + 4 * Cout
constexpr int LDS_BYTES = PAR + 4096;                                 // 152,448
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

__global__ __launch_bounds__(NT, 1) void k_aud_enc(AudEncArgs a) {
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
    const int mh = w >> 2, nq = w & 3;   // a_conv3: fragments 4 mh .. 4 mh + 3, channels 32 nq .. 32 nq + 31
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

    // ================= a_conv1: im2col of the mel input (k = ky * 5 + kx, 25 of 32) =================
    zero(0, BOFF);   // a_conv2's input image: its padding ring reads as zero
    {
        const float* mel = a.mel + (long long)clip * 1600;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = tid + NT * k;   // (row m, 8-tap group)
            if (u < 1600) {
                const int m = u >> 2, g = u & 3, oy = m / 10, ox = m - oy * 10;
                unsigned short v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int tap = 8 * g + e, ky = tap / 5, kx = tap - ky * 5;
                    const int iy = 2 * oy + ky - 1, ix = 2 * ox + kx - 1;
                    const float f = (tap < 25 && iy >= 0 && iy < 80 && ix >= 0 && ix < 20) ? mel[iy * 20 + ix] : 0.f;
                    v[e] = __builtin_bit_cast(unsigned short, (bf16_t)f);
                }
                i32x4 p;
#pragma unroll
                for (int e = 0; e < 4; ++e) p[e] = (int)v[2 * e] | ((int)v[2 * e + 1] << 16);
                st16(BOFF + m * 64 + g * 16, p);
            }
        }
    }
    __syncthreads();
    {
        // M fragment f = rows 16 f .. 16 f + 15 of the 40 x 10 grid; slot i = fragment w + 8 i
        f32x4 acc[4][4];
        i32x4 fb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const i32x4*>(reinterpret_cast<const char*>(a.w1) + ((16 * j + r16) * 32 + kg * 8) * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = (w + 8 * i < 25) ? w + 8 * i : 0;
            const i32x4 fa = lds16(lds, BOFF + (16 * f + r16) * 64 + kg * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fb[j], fa, (f32x4){0.f, 0.f, 0.f, 0.f});   // W x A
        }
        // -> a_conv2's input: chunk (n / 32) buffer, padded pixel (oy + 1, ox + 1); lane = pixel row r16,
        // channels 16 j + 4 kg .. + 3
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = w + 8 * i;
            if (f >= 25) continue;
            const int m = 16 * f + r16, oy = m / 10, ox = m - oy * 10;
            const int px = ((oy + 1) * P2 + ox + 1) * S2 + kg * 8;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f32x4 sc, sh;
                bnq(0, 16 * j + 4 * kg, sc, sh);
                st8l(px + (j >> 1) * W2BUF + (j & 1) * 32, bn_pack4(acc[i][j], sc, sh));
            }
        }
    }
    __syncthreads();

    // ================= a_conv3..a_conv5: 128 output channels, weight slabs of 8 KB in groups of 2 =================
    const int brow3 = tid >> 2, kq3 = tid & 3;
    const int bst3 = BOFF + brow3 * 64 + ((kq3 ^ wsw(brow3)) << 4);   // + slot 16384 + pos 8192
    auto st16b = [&](int addr, i32x4 v) { st16(addr, v); };
    // generic slab loop over NS compile-time slabs: bsoff(s) = weight byte offset of slab s (+ lane part),
    // aread(s, f) / mm(f, b) supplied per layer
    auto run = [&](auto nss, const __amdgpu_buffer_rsrc_t& rsW, int vbl, auto bsoff, const Pre& pre, auto read_a,
                   auto read_b, auto mm) {
        constexpr int NS = decltype(nss)::value;
        i32x4 pb[DA];   // pb[S % DA] holds slab S + 2 at step S
#pragma unroll
        for (int k = 0; k < DA; ++k) pb[k] = pre.w[k + 2];
        st16b(bst3, pre.w[0]);
        st16b(bst3 + 8192, pre.w[1]);
        __syncthreads();
        read_a(std::integral_constant<int, 0>{}, 0);
        read_b(std::integral_constant<int, 0>{}, 0);
        unroll(std::make_integer_sequence<int, NS>{}, [&](auto ss) {
            constexpr int S = decltype(ss)::value;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (S + 2 < NS) {
                st16b(bst3 + (((S / 2) + 1) & 1) * 16384 + (S % 2) * 8192, pb[S % DA]);   // slab S + 2
                if constexpr (S + 2 + DA < NS)
                    pb[S % DA] = __builtin_amdgcn_raw_buffer_load_b128(rsW, vbl + bsoff(std::integral_constant<int, S + 2 + DA>{}), 0, 0);
            }
            if constexpr (S % 2 == 1) __syncthreads();
            if constexpr (S + 1 < NS) {
                read_a(std::integral_constant<int, S + 1>{}, (S + 1) & 1);
                read_b(std::integral_constant<int, S + 1>{}, (S + 1) & 1);
            }
            __builtin_amdgcn_sched_barrier(0);
            mm(S & 1);
        });
    };
    // a layer's first DA + 2 weight slabs (two to the ring, DA in flight), issued before the previous layer's epilogue
    auto prefetch = [&](const __amdgpu_buffer_rsrc_t& rsW, int vbl, auto bsoff) {
        Pre p;
        unroll(std::make_integer_sequence<int, DA + 2>{}, [&](auto k) {
            p.w[decltype(k)::value] = __builtin_amdgcn_raw_buffer_load_b128(rsW, vbl + bsoff(k), 0, 0);
        });
        return p;
    };
    const __amdgpu_buffer_rsrc_t rsW3 = make_rsrc(a.w3, 128 * 1024 * 2), rsW4 = make_rsrc(a.w4, 128 * 512 * 2),
                                 rsW5 = make_rsrc(a.w5, 128 * 512 * 2);
    const int vbl34 = brow3 * 2048 + kq3 * 32;   // a_conv3 (1024-deep rows): vbl34; a_conv4/5 (512): vbl34 / 2
    auto bsoff3 = [](auto ss) { constexpr int S = decltype(ss)::value; return (S % 16) * 128 + (S / 16) * 64; };
    auto bsoff45 = [](auto ss) { constexpr int S = decltype(ss)::value; return (S % 4) * 256 + (S / 4) * 64; };
    auto b_read = [&](int row0, auto ss, int nfr, i32x4* dst) {   // B fragments of rows row0 + 16 j + r16
        constexpr int S = decltype(ss)::value;
        for (int j = 0; j < nfr; ++j)
            dst[j] = lds16(lds, BOFF + ((S / 2) & 1) * 16384 + (S % 2) * 8192 + (row0 + 16 * j + r16) * 64 + ((kg ^ wsw(r16)) << 4));
    };

    const int vbl3 = brow3 * 2048 + kq3 * 16;
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
        int vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = (w + 8 * i < 25) ? w + 8 * i : 0;
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
        i32x4 fa[2][4], fb[2][4];
        int vq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) vq[i] = vb[i];
        auto read_a = [&](auto tt, i32x4 (&f)[4]) {
            constexpr int t = decltype(tt)::value % 16;
            constexpr int imm = ((t / 4) * P2 + t % 4) * S2;
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = lds16(lds + imm, vq[i]);
        };
        auto read_b = [&](int base, i32x4 (&f)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) f[j] = lds16(lds, base + 1024 * j);
        };
        read_a(std::integral_constant<int, 0>{}, fa[0]);
        read_b(bfr, fb[0]);
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
                read_b(bfr + (((t + 1) / 4) & 1) * 16384 + ((t + 1) % 4) * 4096, fb[(t + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fb[t & 1][j], fa[t & 1][i], acc[i][j]);   // W x A
            });
        }
        __syncthreads();   // every read of a_conv2's input done: a_conv3's image goes over it
        pre3 = prefetch(rsW3, vbl3, bsoff3);   // a_conv3's first slabs load under this epilogue
        zero(0, IMG3B);
        __syncthreads();
        // -> a_conv3's input, padded pixel (oy + 1, ox + 1), 8 x 2 fragment rows; lane = fragment row r16
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = w + 8 * i;
            if (f >= 25) continue;
            const int y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
            const int px = ((y + 1) * P3 + x + 1) * S3 + kg * 8;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f32x4 sc, sh;
                bnq(1, 16 * j + 4 * kg, sc, sh);
                st8l(px + 32 * j, bn_pack4(acc[i][j], sc, sh));
            }
        }
        __syncthreads();
    }

    // ---- a_conv3: 4x4 stride 2, 64 -> 128, 40 x 10 -> 20 x 5 (100 rows, 7 fragments); slab = chunk * 16 + tap ----
    {
        int vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = 4 * mh + i, m = (16 * f + r16 < 100) ? 16 * f + r16 : 0;
            const int oy = m / 5, ox = m - oy * 5;
            vb[i] = (2 * oy * P3 + 2 * ox) * S3 + kg * 16;
        }
        f32x4 acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        i32x4 fa[2][4], fb[2][2];
        run(std::integral_constant<int, 32>{}, rsW3, vbl3, bsoff3, pre3,
            [&](auto ss, int buf) {
                constexpr int S = decltype(ss)::value, t = S % 16, c = S / 16;
                constexpr int imm = ((t / 4) * P3 + t % 4) * S3 + c * 64;
#pragma unroll
                for (int i = 0; i < 4; ++i) fa[buf][i] = lds16(lds + imm, vb[i]);
            },
            [&](auto ss, int buf) { b_read(32 * nq, ss, 2, fb[buf]); },
            [&](int buf) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fb[buf][j], fa[buf][i], acc[i][j]);   // W x A
            });
        __syncthreads();
        pre4 = prefetch(rsW4, vbl34 / 2, bsoff45);   // a_conv4's first slabs load under this epilogue
        zero(0, IMG4B);   // a_conv4's input: column 5 reads as zero
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = 16 * (4 * mh + i) + r16;
            if (m >= 100) continue;
            const int oy = m / 5, ox = m - oy * 5;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = 32 * nq + 16 * j + 4 * kg;
                f32x4 sc, sh;
                bnq(2, n, sc, sh);
                st8l((oy * P4 + ox) * S4 + n * 2, bn_pack4(acc[i][j], sc, sh));
            }
        }
        __syncthreads();
    }

    // ---- a_conv4 / a_conv5: 2x2 stride (2, 1), 128 -> 128; slab = chunk * 4 + tap; wave w: channels 16 w .. 16 w + 15 ----
    auto small = [&](auto nff, int img, const __amdgpu_buffer_rsrc_t& rsW, const Pre& pre, int layer, auto store,
                     auto next) {
        constexpr int NFR = decltype(nff)::value;   // M fragments (4: 50 rows, 2: 25 rows)
        constexpr int MR = NFR == 4 ? 50 : 25;
        int vb[NFR];
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            const int m = (16 * i + r16 < MR) ? 16 * i + r16 : 0;
            const int oy = m / 5, ox = m - oy * 5;
            vb[i] = img + (2 * oy * P4 + ox) * S4 + kg * 16;
        }
        f32x4 acc[NFR];
#pragma unroll
        for (int i = 0; i < NFR; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
        i32x4 fa[2][NFR], fb[2][1];
        run(std::integral_constant<int, 16>{}, rsW, vbl34 / 2, bsoff45, pre,
            [&](auto ss, int buf) {
                constexpr int S = decltype(ss)::value, t = S % 4, c = S / 4;
                constexpr int imm = ((t / 2) * P4 + t % 2) * S4 + c * 64;
#pragma unroll
                for (int i = 0; i < NFR; ++i) fa[buf][i] = lds16(lds + imm, vb[i]);
            },
            [&](auto ss, int buf) { b_read(16 * w, ss, 1, fb[buf]); },
            [&](int buf) {
#pragma unroll
                for (int i = 0; i < NFR; ++i) acc[i] = mfma(fb[buf][0], fa[buf][i], acc[i]);   // W x A
            });
        const int n = 16 * w + 4 * kg;   // lane channels n .. n + 3
        __syncthreads();
        next();   // the next layer's first weight slabs load under this epilogue
        f32x4 sc, sh;
        bnq(layer, n, sc, sh);
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            const int m = 16 * i + r16;
            if (m < MR) store(m / 5, m % 5, n, bn_pack4(acc[i], sc, sh));
        }
        __syncthreads();
    };
    zero(IMG5, IMG5 + IMG5B);   // a_conv5's input: column 5 reads as zero (ordered by the barriers in `small`)
    small(std::integral_constant<int, 4>{}, 0, rsW4, pre4, 3, [&](int oy, int ox, int n, i32x2 v) {
        st8l(IMG5 + (oy * P4 + ox) * S4 + n * 2, v);
    }, [&] { pre5 = prefetch(rsW5, vbl34 / 2, bsoff45); });
    bf16_t* const outc = a.out + (long long)clip * a.out_clip_stride;
    small(std::integral_constant<int, 2>{}, IMG5, rsW5, pre5, 4, [&](int oy, int ox, int n, i32x2 v) {
        *reinterpret_cast<i32x2*>(outc + (oy * 5 + ox) * 128 + n) = v;   // Flatten (HWC) -> concat[0:3200]
    }, [] {});
}

}  // namespace

bool aud_enc_supported(const AudEncArgs& a) {
    const char* e = std::getenv("AVSE_NO_AUDENC");
    if (e && e[0] == '1') return false;
    return a.N > 0 && a.w1 && a.w2 && a.w3 && a.w4 && a.w5;
}

int launch_aud_enc(const AudEncArgs& a, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_aud_enc, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
        attr = true;
    }
    hipLaunchKernelGGL(k_aud_enc, dim3(a.N), dim3(NT), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
