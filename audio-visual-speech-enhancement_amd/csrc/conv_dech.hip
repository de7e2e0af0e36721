// Fused decoder head, two clips per workgroup (bf16, gfx950): network.py:112-123
//   d_deconv1  Conv2DTranspose(128, 2x2, strides (2, 1), 'same')   5 x 5 x 128 -> 10 x 5 x 128
//   d_deconv2  Conv2DTranspose(128, 2x2, strides (2, 1), 'same')  10 x 5 x 128 -> 20 x 5 x 128
//   d_deconv3  Conv2DTranspose(128, 4x4, strides (2, 2), 'same')  20 x 5 x 128 -> 40 x 10 x 128 (-> HBM, k_dec_tail)
// each + BatchNormalization + LeakyReLU(0.3); input = dec_dense2's [5, 5, 128] reshape.
//
// Why: three k_conv launches (~0.105 ms per 512 clips; d_deconv1 / d_deconv2 ~17-20 us each for 1-2 GFLOP,
// d_deconv3 26.8 GFLOP at ~400 TFLOP/s).  The recipe of conv_aud.hip / conv_dec.hip: activations in zero-padded LDS
// images (288-B rows: 128 channels + pad), weights through the LDS slab ring (8 KB slabs, groups of 2, the next
// layer's first slabs prefetched under each epilogue), the sub-pixel phases of each transposed conv as in k_conv
// (only the taps that hit a phase: phase (py, px) tap (a, b) = input offset (py - a, px - b)), the whole slab
// schedule compile-time.
// The head's layers are small (M = 25 / 50 / 100 pixels per phase and clip) against 768 KB of weights per clip: with
// one clip per workgroup a slab carried 2-8 MFMAs per wave and the weight stream (L2 latency, 8 KB per slab, two
// slabs of look-ahead) bounded the kernel.  Here:
//   * two clips share every weight slab (twice the MFMAs per slab, half the weight traffic per clip);
//   * the weight pieces run DA slabs ahead in registers;
//   * the MFMA computes D = W x A (channels x pixels): a lane's 4 accumulator rows are 4 consecutive channels of one
//     pixel, so the epilogue stores 8 B per lane and fragment (ds_write_b64 / buffer 8-B stores) instead of four
//     2-byte stores;
//   * d_deconv1 / d_deconv2: wave w owns output channels 16 w .. 16 w + 15 and all M fragments of both clips;
//     d_deconv3 (7 M fragments per phase and clip): wave (c, nq) owns clip c's fragments x channels 32 nq .. + 31.
#include <cstdlib>
#include <utility>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr int NW = 8, NT = 64 * NW;
constexpr int NC = 2;                                        // clips per workgroup
constexpr int S = 288;                                       // image pixel stride (128 bf16 channels + 32 B)
// per-clip LDS region: d_deconv3's input image, d_deconv1's input aliased into its first 30 pixels (dead once
// d_deconv1 is done; the border pixels it covered are re-zeroed before d_deconv3 reads them), d_deconv2's input
constexpr int IMG3 = 0, P3 = 7, IMG3B = 22 * P3 * S;         // d_deconv3 input: 20 x 5 padded by 1 -> 22 x 7
constexpr int IMG1 = 0, P1 = 6, IMG1B = 5 * P1 * S;          // d_deconv1 input: 5 x 5, left pad 1 -> 5 x 6
constexpr int IMG2 = IMG3B, P2 = 6, IMG2B = 10 * P2 * S;     // d_deconv2 input: 10 x 5, left pad 1 -> 10 x 6
constexpr int CLB = IMG2 + IMG2B;                            // 61,632 B per clip
constexpr int BOFF = NC * CLB;                               // weight ring: 2 slots x 2 slabs x 8 KB
constexpr int LDS_BYTES = BOFF + 32768;                      // 156,032
constexpr int DA = 6;                                        // weight pieces in flight in registers
static_assert(NC == 2 && IMG1B <= IMG3B && CLB % 64 == 0 && LDS_BYTES <= 160 * 1024, "LDS map");
// IMG3 border pixels among IMG1's 30: row 0, columns 0 / 6 of rows 1..3, (4, 0)
constexpr int NBZ = 14;
__device__ __forceinline__ int border_px(int i) {
    return i < 7 ? i : i < 13 ? ((i - 7) / 2 + 1) * P3 + ((i - 7) & 1) * 6 : 4 * P3;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
struct Pre { i32x4 w[DA + 2]; };   // a layer's first DA + 2 weight pieces

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int wsw(int row) { return 2 * ((row >> 2) & 1); }
__device__ __forceinline__ i32x4 lds16(const char* base, int off) { return *reinterpret_cast<const i32x4*>(base + off); }
template <int... I, typename F>
__device__ __forceinline__ void unroll(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}
__device__ __forceinline__ f32x4 mfma(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ float bn_lrelu(float acc, float sc, float sh) {
    const float v = fmaf(acc, sc, sh);
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(LRELU * v));   // LeakyReLU, no canonicalise
    return r;
}
__device__ __forceinline__ i32x2 pack4(float a, float b, float c, float d) {   // 4 bf16 (RNE, as (bf16_t) casts)
    const bf16x2 lo = __builtin_convertvector((f32x2){a, b}, bf16x2), hi = __builtin_convertvector((f32x2){c, d}, bf16x2);
    return (i32x2){__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi)};
}

// Layer geometry.  L = 1, 2: phases py in {0, 1} (px = 0), taps b in {0, 1}: input (yq, xq - b); grid HQ x 5.
// L = 3: phases (py, px), taps (a, b) in {0, 1}^2: input (yq + py - a, xq + px - b); grid 20 x 5.
template <int L> struct Geo {
    static constexpr int NP = L == 3 ? 4 : 2, NTAP = L == 3 ? 4 : 2, HQ = L == 1 ? 5 : L == 2 ? 10 : 20, WQ = 5;
    static constexpr int M = HQ * WQ, NFR = (M + 15) / 16;            // M fragments per phase and clip
    static constexpr int NSL = NTAP * 4;                               // slabs per phase: tap * 4 + chunk
    static constexpr int KPAD = NTAP * 128;
    static constexpr int IMG = L == 1 ? IMG1 : L == 2 ? IMG2 : IMG3, P = L == 3 ? P3 : P1, PT = L == 3 ? 1 : 0, PL = 1;
    // smallest tap offset: (dy, dx) = (-1, -1) for L = 3, (0, -1) otherwise
    static constexpr int DY0 = L == 3 ? -1 : 0, DX0 = -1;
    static constexpr int tap_dy(int p, int t) { return L == 3 ? (p >> 1) - (t >> 1) : 0; }
    static constexpr int tap_dx(int p, int t) { return L == 3 ? (p & 1) - (t & 1) : -t; }
    // fragment row m -> grid (yq, xq): column-major for d_deconv2 / d_deconv3 (16 consecutive rows of a column: the
    // ds_read_b128 fragment gathers are 1.5 / 1.4-way bank-conflicted instead of 1.75 / 2.0 row-major, exhaustive
    // check over every tap), row-major for d_deconv1
    static constexpr bool CM = L >= 2;
    __device__ static void grid(int m, int& yq, int& xq) {
        if constexpr (CM) { xq = m / HQ; yq = m - xq * HQ; } else { yq = m / WQ; xq = m - yq * WQ; }
    }
};

// ABL: ablation mask for tools/dech_ablate.hip only (0 in the library): 1 = no MFMAs, 2 = no epilogue stores,
// 4 = no barriers in the slab loop (2: the stores are skipped by a runtime test, so the MFMAs stay live), 8 = no weight-piece loads (timing only: results are meaningless)
template <int ABL = 0>
__global__ __launch_bounds__(NT, 1) void k_dec_head(DecHeadArgs a) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int clip0 = NC * blockIdx.x;
    const int mh = w >> 2, nq = w & 3;   // d_deconv3's wave split: clip mh, channels 32 nq .. + 31
    auto st16 = [&](int addr, i32x4 v) { *reinterpret_cast<i32x4*>(lds + addr) = v; };

    // ---- weight ring: lane tid moves 16 B (kq = tid & 3) of row tid >> 2 of an 8-KB slab ----
    const int brow = tid >> 2, kq = tid & 3;
    const int bst = BOFF + brow * 64 + ((kq ^ wsw(brow)) << 4);   // + slot 16384 + pos 8192
    const __amdgpu_buffer_rsrc_t rsW1 = make_rsrc(a.w1, 2 * 128 * 256 * 2), rsW2 = make_rsrc(a.w2, 2 * 128 * 256 * 2),
                                 rsW3 = make_rsrc(a.w3, 4 * 128 * 512 * 2);
    // ring piece of slab s of layer L (phase s / NSL, slab within phase s % NSL): k = tap * 128 + chunk * 32
    auto piece = [&](auto ll, auto ss) -> i32x4 {
        constexpr int LL = decltype(ll)::value, s = decltype(ss)::value;
        using G = Geo<LL>;
        constexpr int sv = s < G::NP * G::NSL ? s : 0, p = sv / G::NSL, sl = sv % G::NSL;
        const __amdgpu_buffer_rsrc_t& rs = LL == 1 ? rsW1 : LL == 2 ? rsW2 : rsW3;
        if constexpr ((ABL & 8) != 0) return (i32x4){s, 0, 0, 0};
        return __builtin_amdgcn_raw_buffer_load_b128(rs, brow * (G::KPAD * 2) + kq * 16, (p * 128 * G::KPAD + sl * 32) * 2, 0);
    };
    // d_deconv1 / d_deconv2: wave w's own B fragment of slab s (rows 16 w + r16, k-group kg), straight from global
    // memory — no wave shares it, so these layers skip the LDS ring and its barrier every two slabs
    auto dpiece = [&](auto ll, auto ss) -> i32x4 {
        constexpr int LL = decltype(ll)::value, s = decltype(ss)::value;
        using G = Geo<LL>;
        constexpr int sv = s < G::NP * G::NSL ? s : 0, p = sv / G::NSL, sl = sv % G::NSL;
        const __amdgpu_buffer_rsrc_t& rs = LL == 1 ? rsW1 : rsW2;
        return __builtin_amdgcn_raw_buffer_load_b128(rs, (16 * w + r16) * (G::KPAD * 2) + kg * 16,
                                                     (p * 128 * G::KPAD + sl * 32) * 2, 0);
    };
    auto prefetch = [&](auto ll) {
        Pre pr;
        unroll(std::make_integer_sequence<int, DA + 2>{}, [&](auto k) {
            if constexpr (decltype(ll)::value <= 2) pr.w[decltype(k)::value] = dpiece(ll, k);
            else pr.w[decltype(k)::value] = piece(ll, k);
        });
        return pr;
    };

    // ---- d_deconv1 input: dec_dense2's 5 x 5 x 128 (HWC) -> image pixel (y, x + 1) ----
    for (int o = tid * 16; o < BOFF; o += NT * 16) st16(o, (i32x4){0, 0, 0, 0});   // zero padding rings
    Pre pre = prefetch(std::integral_constant<int, 1>{});
    __syncthreads();
    for (int q = tid; q < NC * 400; q += NT) {
        const int c = q >= 400, r = q - 400 * c;
        const int px = r >> 4, part = r & 15, y = px / 5, x = px - y * 5;
        const int clip = clip0 + c < a.N ? clip0 + c : a.N - 1;   // a missing second clip computes on a copy
        const i32x4 v = *reinterpret_cast<const i32x4*>(reinterpret_cast<const char*>(a.in) + (long long)clip * a.in_clip_stride * 2 + px * 256 + part * 16);
        st16(c * CLB + IMG1 + (y * P1 + x + 1) * S + part * 16, v);
    }

    auto layer = [&](auto ll, const float* scp, const float* shp, auto store, auto next) {
        constexpr int LL = decltype(ll)::value;
        using G = Geo<LL>;
        constexpr bool WIDE = LL == 3;                 // waves split clips and N (d_deconv3) or N only
        constexpr bool DIRECT = !WIDE;                 // B fragments per wave from global memory (see dpiece)
        constexpr int NI = WIDE ? G::NFR : NC * G::NFR, NJ = WIDE ? 2 : 1;
        const int row0 = WIDE ? 32 * nq : 16 * w;      // this wave's first output channel
        // fragment slot i: clip (WIDE ? mh : i / NFR), M fragment (WIDE ? i : i % NFR); lane row r16 -> grid
        // (yq, xq) -> image base at tap (DY0, DX0)
        int vb[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = WIDE ? mh : i / G::NFR, f = WIDE ? i : i % G::NFR;
            const int m = (16 * f + r16 < G::M) ? 16 * f + r16 : 0;
            int yq, xq;
            G::grid(m, yq, xq);
            vb[i] = c * CLB + G::IMG + ((yq + G::PT + G::DY0) * G::P + (xq + G::PL + G::DX0)) * S + kg * 16;
        }
        // accumulator row e of channel fragment j = channel row0 + 16 j + 4 kg + e
        float sc[NJ][4], sh[NJ][4];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                sc[j][e] = scp[row0 + 16 * j + 4 * kg + e];
                sh[j][e] = shp[row0 + 16 * j + 4 * kg + e];
            }
        f32x4 acc[NI][NJ];
        auto zero_acc = [&] {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        };
        i32x4 fa[2][NI], fb[2][NJ];
        auto read = [&](auto ss, int buf) {
            constexpr int s = decltype(ss)::value, p = s / G::NSL, sl = s % G::NSL, t = sl / 4, c = sl % 4;
            constexpr int imm = ((G::tap_dy(p, t) - G::DY0) * G::P + (G::tap_dx(p, t) - G::DX0)) * S + c * 64;
#pragma unroll
            for (int i = 0; i < NI; ++i) fa[buf][i] = lds16(lds + imm, vb[i]);
            if constexpr (!DIRECT)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                fb[buf][j] = lds16(lds, BOFF + (((s / 2) & 1) * 16384 + (s % 2) * 8192) + (row0 + 16 * j + r16) * 64 +
                                            ((kg ^ wsw(r16)) << 4));
        };
        constexpr int NS = G::NP * G::NSL;
        // register ring: pb[s % DA] holds slab s + 2 at step s (LDS ring); pd[s % (DA + 2)] holds slab s (DIRECT)
        i32x4 pb[DA], pd[DA + 2];
        if constexpr (DIRECT) {
#pragma unroll
            for (int k = 0; k < DA + 2; ++k) pd[k] = pre.w[k];
        } else {
#pragma unroll
            for (int k = 0; k < DA; ++k) pb[k] = pre.w[k + 2];
            st16(bst, pre.w[0]);
            st16(bst + 8192, pre.w[1]);
        }
        zero_acc();
        __syncthreads();
        read(std::integral_constant<int, 0>{}, 0);
        unroll(std::make_integer_sequence<int, NS>{}, [&](auto ss) {
            constexpr int s = decltype(ss)::value, p = s / G::NSL;
            constexpr bool last = (s + 1) % G::NSL == 0;
            __builtin_amdgcn_sched_barrier(0);
            i32x4 fbd;
            if constexpr (DIRECT) {
                fbd = pd[s % (DA + 2)];
                if constexpr (s + DA + 2 < NS) pd[s % (DA + 2)] = dpiece(ll, std::integral_constant<int, s + DA + 2>{});
            } else {
                if constexpr (s + 2 < NS) {
                    st16(bst + (((s / 2) + 1) & 1) * 16384 + (s % 2) * 8192, pb[s % DA]);    // slab s + 2
                    if constexpr (s + 2 + DA < NS) pb[s % DA] = piece(ll, std::integral_constant<int, s + 2 + DA>{});
                }
                if constexpr (s % 2 == 1 && !(ABL & 4)) __syncthreads();
            }
            if constexpr (s + 1 < NS && !last) read(std::integral_constant<int, s + 1>{}, (s + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    if constexpr (!(ABL & 1)) acc[i][j] = mfma(DIRECT ? fbd : fb[s & 1][j], fa[s & 1][i], acc[i][j]);   // W x A
                    else acc[i][j][0] += __builtin_bit_cast(float, fa[s & 1][i][0] ^ fb[s & 1][j][0]);
            if constexpr (last) {
                if constexpr (p + 1 == G::NP) {   // layer done: the next layer's first slabs load under this epilogue
                    __syncthreads();
                    next();
                }
                // epilogue of phase p: lane pixel m = 16 f + r16 of the grid (yq, xq) -> output (2 yq + py, OXS xq + px)
                constexpr int py = LL == 3 ? p >> 1 : p, px = LL == 3 ? p & 1 : 0;
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const int c = WIDE ? mh : i / G::NFR, f = WIDE ? i : i % G::NFR;
                    const int m = 16 * f + r16;
                    if (((ABL & 2) != 0 && a.N != -1) || (16 * f + 15 >= G::M && m >= G::M)) continue;
                    int yq, xq;
                    G::grid(m, yq, xq);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const f32x4 v = acc[i][j];
                        store(c, 2 * yq + py, (LL == 3 ? 2 : 1) * xq + px, row0 + 16 * j + 4 * kg,
                              pack4(bn_lrelu(v[0], sc[j][0], sh[j][0]), bn_lrelu(v[1], sc[j][1], sh[j][1]),
                                    bn_lrelu(v[2], sc[j][2], sh[j][2]), bn_lrelu(v[3], sc[j][3], sh[j][3])));
                    }
                }
                if constexpr (p + 1 < G::NP) {
                    zero_acc();
                    read(std::integral_constant<int, s + 1>{}, (s + 1) & 1);
                }
            }
        });
        __syncthreads();
    };

    layer(std::integral_constant<int, 1>{}, a.sc[0], a.sh[0], [&](int c, int y, int x, int n, i32x2 v) {
        *reinterpret_cast<i32x2*>(lds + c * CLB + IMG2 + (y * P2 + x + 1) * S + n * 2) = v;
    }, [&] { pre = prefetch(std::integral_constant<int, 2>{}); });
    // d_deconv1's input is dead: restore the zero border of d_deconv3's image it overlapped
    if (tid < NC * NBZ * 16) {
        const int c = tid >= NBZ * 16, r = tid - NBZ * 16 * c;
        st16(c * CLB + IMG3 + border_px(r >> 4) * S + (r & 15) * 16, (i32x4){0, 0, 0, 0});
    }
    layer(std::integral_constant<int, 2>{}, a.sc[1], a.sh[1], [&](int c, int y, int x, int n, i32x2 v) {
        *reinterpret_cast<i32x2*>(lds + c * CLB + IMG3 + ((y + 1) * P3 + x + 1) * S + n * 2) = v;
    }, [&] { pre = prefetch(std::integral_constant<int, 3>{}); });
    // d_deconv3: wave clip mh -> HBM [clip][40][10][128]; a missing last clip of the grid stores nothing
    const __amdgpu_buffer_rsrc_t ors =
        make_rsrc(a.out + (long long)(clip0 + mh) * a.out_clip_stride, clip0 + mh < a.N ? 400 * 128 * 2 : 0);
    layer(std::integral_constant<int, 3>{}, a.sc[2], a.sh[2], [&](int, int y, int x, int n, i32x2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(v, ors, ((y * 10 + x) * 128 + n) * 2, 0, 0);
    }, [] {});
}

}  // namespace

bool dec_head_supported(const DecHeadArgs& a) {
    return a.N > 0 && a.w1 && a.w2 && a.w3;
}

int launch_dec_head(const DecHeadArgs& a, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_dec_head<0>, LDS_BYTES)) return rc;
    hipLaunchKernelGGL(k_dec_head<0>, dim3((a.N + NC - 1) / NC), dim3(NT), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
