// Batched-clip GEMMs of the fusion / decoder MLP and v_conv6 (bf16, gfx950):
//   enc_dense   Dense(1312) on concat [N][5248]   network.py:56-58     (MODE 0)
//   dec_dense1  Dense(1312)                        network.py:69-71     (MODE 0)
//   dec_dense2  Dense(3200) -> Reshape(5, 5, 128)  network.py:75-78     (MODE 0)
//   v_conv6     Conv2D(512, 3x3, 'same') on 4 x 4 x 512 + BN + LeakyReLU + MaxPool(2x2) -> concat[3200:5248]
//               network.py:169-175 (MODE 1: implicit GEMM, M = 16 pixels per clip)
// all with the folded bias / BatchNorm + LeakyReLU(0.3) epilogue.
//
// Why: on k_conv these ran at 200-500 TFLOP/s (enc_dense 7 GFLOP in ~27 us + a split-K reduce launch, v_conv6
// 38.6 GFLOP in ~61 us + reduce): a barrier per 64-byte slab and a second kernel for every split-K sum.  Here:
//   * 128 x 128 output tile per workgroup, 8 waves (two per SIMD), wave (wm, wn) = 64 rows x 32 columns:
//     4 x 2 v_mfma_f32_16x16x32_bf16 per 32-deep K slab;
//   * A and W slabs (8 KB each) stream through an LDS ring of 4-slab groups (2 x 64 KB): every lane moves 16 B
//     of A and 16 B of W per slab, 8 slabs ahead in registers, 4 ahead into LDS; one barrier per group;
//   * split-K over blockIdx.z with the reduction in the LAST-ARRIVING workgroup of a tile (atomic ticket):
//     fp32 partial tiles in MFMA-native lane order (16-B coalesced stores), no second launch;
//   * v_conv6: tile rows are 8 clips x 16 pixels ordered so that a lane's 4 accumulator rows are one 2x2 pool
//     window; the A row of slab (tap, 32-channel chunk) is gathered per lane (zero outside the 4 x 4 image).
#include <cstdlib>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;
constexpr int NT = 512;
constexpr int SLAB = 16384;                     // A (8 KB) + W (8 KB) per 32-deep slab
constexpr int GRP = 4 * SLAB;                   // one ring slot: 4 slabs
constexpr int LDS_BYTES = 2 * GRP;              // 128 KB

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ int wsw(int row) { return 2 * ((row >> 2) & 1); }
__device__ __forceinline__ i32x4 lds16(const char* p) { return *reinterpret_cast<const i32x4*>(p); }

// ABL: timing ablations for tools/gemm_ablate.hip only (0 in the library): 1 = the tile's last workgroup skips
// reading the other partials (outputs meaningless)
template <int MODE, int ABL = 0>
__global__ __launch_bounds__(NT, 1) void k_gemm(GemmArgs g) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    __shared__ int last_flag;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int wm = w >> 2, wn = w & 3;
    const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 128, z = blockIdx.z;
    const int nslab_all = g.kpad / 32;
    const int sps = (nslab_all + g.ksplit - 1) / g.ksplit;
    const int s_begin = z * sps, nsl = min(nslab_all, s_begin + sps) - s_begin;

    // ---- loader lane: row = tid / 4 of the A and W tiles, 16-B part tid % 4 of a 64-B slab row ----
    const int lrow = tid >> 2, part = tid & 3;
    const int ldst = lrow * 64 + ((part ^ wsw(lrow)) << 4);   // + slot GRP + pos SLAB (+ 8192 for W)
    const __amdgpu_buffer_rsrc_t rsW = make_rsrc(g.w, (long long)g.N * g.kpad * 2);
    const int wvoff = (n0 + lrow < g.N) ? (n0 + lrow) * g.kpad * 2 + part * 16 : kOOB;
    __amdgpu_buffer_rsrc_t rsA;
    int avoff = kOOB, py = 0, px = 0;
    if constexpr (MODE == 0) {
        rsA = make_rsrc(g.a, (long long)g.M * g.lda * 2);
        if (m0 + lrow < g.M) avoff = (m0 + lrow) * (int)g.lda * 2 + part * 16;
    } else {
        // row m: clip m / 16, pixel p = m % 16, pool window q = p / 4, e = p % 4 -> (y, x) of the 4 x 4 image
        const int m = m0 + lrow, clip = m >> 4, p = m & 15, q = p >> 2, e = p & 3;
        py = 2 * (q >> 1) + (e >> 1);
        px = 2 * (q & 1) + (e & 1);
        rsA = make_rsrc(g.a, (long long)(g.M >> 4) * g.lda * 2);
        if (m < g.M) avoff = clip * (int)g.lda * 2 + (py * 4 + px) * 1024 + part * 16;
    }
    // slab s of this split (absolute k slab s_begin + s): A / W pieces
    auto load = [&](int s, i32x4& va, i32x4& vw) {
        const int sa = s_begin + (s < nsl ? s : 0);
        vw = __builtin_amdgcn_raw_buffer_load_b128(rsW, wvoff, sa * 64, 0);
        if constexpr (MODE == 0) {
            va = __builtin_amdgcn_raw_buffer_load_b128(rsA, avoff, sa * 64, 0);
        } else {
            // k = tap * 512 + chunk * 32: tap = sa / 16 (dy = tap / 3 - 1, dx = tap % 3 - 1), chunk = sa % 16
            const int tap = sa >> 4, c = sa & 15, dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
            const bool ok = (unsigned)(py + dy) < 4u && (unsigned)(px + dx) < 4u && avoff != kOOB;
            va = __builtin_amdgcn_raw_buffer_load_b128(rsA, ok ? avoff + (dy * 4 + dx) * 1024 : kOOB, c * 64, 0);
        }
    };
    auto store = [&](int s, const i32x4& va, const i32x4& vw) {   // slab s -> slot (s / 4) & 1, position s % 4
        char* const d = lds + ((s >> 2) & 1) * GRP + (s & 3) * SLAB + ldst;
        *reinterpret_cast<i32x4*>(d) = va;
        *reinterpret_cast<i32x4*>(d + 8192) = vw;
    };
    // ---- fragments: A rows 64 wm + 16 i + r16, W rows 32 wn + 16 j + r16 (16-B k-group kg, swizzled) ----
    const int afr = (64 * wm + r16) * 64 + ((kg ^ wsw(r16)) << 4);
    const int bfr = 8192 + (32 * wn + r16) * 64 + ((kg ^ wsw(r16)) << 4);
    i32x4 fa[2][4], fb[2][2];
    auto read = [&](int s, int buf) {
        const char* const b = lds + ((s >> 2) & 1) * GRP + (s & 3) * SLAB;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[buf][i] = lds16(b + afr + 1024 * i);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[buf][j] = lds16(b + bfr + 1024 * j);
    };
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // epilogue scale / shift of this lane's two columns, loaded now (in the epilogue their latency was exposed)
    float esc[2], esh[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + 32 * wn + 16 * j + r16;
        esc[j] = n < g.N ? g.scale[n] : 0.f;
        esh[j] = n < g.N ? g.shift[n] : 0.f;
    }

    // prologue: slabs 0..3 -> slot 0, slabs 4..7 in registers
    i32x4 ra[4], rw[4];
    {
        i32x4 a0[4], w0[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) load(s, a0[s], w0[s]);
#pragma unroll
        for (int s = 0; s < 4; ++s) load(s + 4, ra[s], rw[s]);
#pragma unroll
        for (int s = 0; s < 4; ++s) store(s, a0[s], w0[s]);
    }
    __syncthreads();
    read(0, 0);
    // slab S: store S + 4 (loaded 4 slabs ago), load S + 8, a barrier every 4 slabs publishes the next group;
    // every step runs (the padding past nsl only moves data) so the outstanding-load count is static
    const int npad = (nsl + 3) & ~3;
    for (int s0 = 0; s0 < npad; s0 += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int s = s0 + q;
            __builtin_amdgcn_sched_barrier(0);
            store(s + 4, ra[q], rw[q]);
            load(s + 8, ra[q], rw[q]);
            if (q == 3) __syncthreads();
            if (s + 1 < nsl) read(s + 1, (q + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
            if (s < nsl) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[q & 1][i]),
                                                                             __builtin_bit_cast(bf16x8, fb[q & 1][j]),
                                                                             acc[i][j], 0, 0, 0);
            }
        }
    }

    // ---- split-K: partial tile -> workspace; the last workgroup of the tile sums and runs the epilogue ----
    // Cross-XCD hand-off without __threadfence() (an L2 write-back + invalidate per workgroup: it made the dense
    // layers 3-4x slower): partials are stored and re-read with sc1 (L2 write-through / L1 bypass), every wave
    // waits for its stores, one lane takes an agent-scope ticket, the tile's last workgroup reads after a barrier
    // (MI355X_MICROARCH.md, inter-workgroup visibility).
    if (g.ksplit > 1) {
        const int tile = blockIdx.y * gridDim.x + blockIdx.x;
        const __amdgpu_buffer_rsrc_t rsP = make_rsrc(g.partial + (size_t)tile * g.ksplit * 8 * NT * 4,
                                                     (long long)g.ksplit * 8 * NT * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, acc[i][j]), rsP,
                                                       ((z * 8 + i * 2 + j) * NT + tid) * 16, 0, 16 /* sc1 */);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            last_flag = __hip_atomic_fetch_add(g.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g.ksplit - 1;
        __syncthreads();
        if (!last_flag) return;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        for (int zz = 0; zz < ((ABL & 1) ? 0 : g.ksplit); ++zz)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                               rsP, ((zz * 8 + i * 2 + j) * NT + tid) * 16, 0, 16 /* sc1 */));
        if (tid == 0) g.counters[tile] = 0;   // ready for the next launch (stream order)
    }

    // ---- epilogue: lane holds rows 4 kg .. 4 kg + 3 of fragment i, column n0 + 32 wn + 16 j + r16 ----
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + 32 * wn + 16 * j + r16;
        if (n >= g.N) continue;
        const float sc = esc[j], sh = esh[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int mb = m0 + 64 * wm + 16 * i + 4 * kg;
            if (mb >= g.M) continue;
            if constexpr (MODE == 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (mb + e >= g.M) continue;
                    float v = acc[i][j][e] * sc + sh;
                    if (g.act) v = v >= 0.f ? v : LRELU * v;
                    g.out[(long long)(mb + e) * g.ldo + g.out_off + n] = (bf16_t)v;
                }
            } else {
                float v = fmaxf(fmaxf(acc[i][j][0] * sc + sh, acc[i][j][1] * sc + sh),
                                fmaxf(acc[i][j][2] * sc + sh, acc[i][j][3] * sc + sh));
                if (g.act) v = v >= 0.f ? v : LRELU * v;
                const int clip = mb >> 4, q = (mb & 15) >> 2;   // pooled pixel q of the 2 x 2 output (HWC)
                g.out[(long long)clip * g.ldo + g.out_off + q * g.N + n] = (bf16_t)v;
            }
        }
    }
}

}  // namespace

// split-K factor: as many workgroups as fit one round on the 256 CUs (one 128-KB workgroup per CU: 264
// workgroups took two rounds), at least 8 slabs each
int gemm_ksplit(int M, int N, int kpad, int cap) {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128), nslab = kpad / 32;
    int ks = 256 / tiles;
    ks = ks > nslab / 8 ? nslab / 8 : ks;
    if (cap > 0 && cap < ks) ks = cap;   // A/B: cap the split (timing experiments, ksplit == 1 parity test)
    return ks < 1 ? 1 : ks;
}

size_t gemm_ws_bytes(int M, int N, int kpad, int cap) {
    const int ks = gemm_ksplit(M, N, kpad, cap);
    const size_t tiles = (size_t)((M + 127) / 128) * ((N + 127) / 128);
    return ks > 1 ? tiles * ks * 128 * 128 * 4 : 0;
}

int launch_gemm(const GemmArgs& g, int mode, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_gemm<0>, LDS_BYTES)) return rc;
    if (int rc = ensure_lds_attr((const void*)k_gemm<1>, LDS_BYTES)) return rc;
    if (g.kpad % 32 || g.M <= 0 || g.N <= 0 || g.ksplit < 1 || (g.ksplit > 1 && (!g.partial || !g.counters)) ||
        (mode == 1 && (g.M % 16 || g.kpad != 9 * 512))) {
        set_error("gemm: bad arguments");
        return 3;
    }
    const dim3 grid((g.M + 127) / 128, (g.N + 127) / 128, g.ksplit);
    if (mode == 0) hipLaunchKernelGGL(k_gemm<0>, grid, dim3(NT), LDS_BYTES, s, g);
    else hipLaunchKernelGGL(k_gemm<1>, grid, dim3(NT), LDS_BYTES, s, g);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
