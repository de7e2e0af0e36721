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
#include <algorithm>
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

// ABL: timing ablations (0 in the library; tools/gemm_ablate.hip, AVSE_GEMM_ABL variant libraries): 1 = the tile's
// last workgroup skips reading the other partials, 2 = S16: no global loads, 4 = S16: no MFMAs (outputs meaningless)
// S16: AVSE_F32_SPLIT operands (DESIGN.md §3 split-f16).  A slab row is 16 k as [h(16) | l(16)] f16 (the same 64 B
// as 32 bf16 k), activations in the split-pair layout and weights packed [Wh(16) | Wl(16)] per 16 k (capi.hip
// build_layer, k_conv's packing); per slab two v_mfma_f32_16x16x32_f16, [Ah | Al] x [Wh | Wh] and [Ah | Al] x [Wl | Wl]
// (every lane of a W fragment reads k-group kg & 1 of the h or the l half): all four products.  Sums are blocked as
// k_conv's (kFp32Block slabs summed from zero, then added to the running sum in order) and split-K splits hold
// whole blocks (GemmArgs::slabs_per_split), so a split plan fixed by K and N (dense) or one block per split (v_conv6)
// gives every batch size the same bits.  Outputs are stored as pairs (range guard: GemmArgs::range_flag).
template <int MODE, int ABL = 0, bool S16 = false>
__global__ __launch_bounds__(NT, 1) void k_gemm(GemmArgs g) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    __shared__ int last_flag;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int wm = w >> 2, wn = w & 3;
    const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 128, z = blockIdx.z;
    constexpr int KB = S16 ? 4 : 2;                 // bytes per k in A and W rows
    const int nslab_all = g.kpad * KB / 64;
    const int sps = S16 && g.slabs_per_split > 0 ? g.slabs_per_split : (nslab_all + g.ksplit - 1) / g.ksplit;
    const int s_begin = z * sps, nsl = min(nslab_all, s_begin + sps) - s_begin;

    // ---- loader lane: row = tid / 4 of the A and W tiles, 16-B part tid % 4 of a 64-B slab row ----
    const int lrow = tid >> 2, part = tid & 3;
    const int ldst = lrow * 64 + ((part ^ wsw(lrow)) << 4);   // + slot GRP + pos SLAB (+ 8192 for W)
    const __amdgpu_buffer_rsrc_t rsW = make_rsrc(g.w, (long long)g.N * g.kpad * KB);
    const int wvoff = (n0 + lrow < g.N) ? (n0 + lrow) * g.kpad * KB + part * 16 : kOOB;
    constexpr int PIXB = 512 * KB, CPT = PIXB / 64;   // mode 1: bytes per input pixel, 64-B chunks per tap
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
        if (m < g.M) avoff = clip * (int)g.lda * 2 + (py * 4 + px) * PIXB + part * 16;
    }
    // slab s of this split (absolute k slab s_begin + s): A / W pieces
    // (S16: slabs past nsl read zeros, so the padded steps of the main loop add exact zeros and need no branches)
    auto load = [&](int s, i32x4& va, i32x4& vw) {
        if constexpr ((ABL & 2) != 0) {   // ablation: no global loads (zeros)
            va = vw = (i32x4){s, 0, 0, 0};
            return;
        }
        const int sa = s_begin + (s < nsl ? s : 0);
        const bool pad = S16 && s >= nsl;
        vw = __builtin_amdgcn_raw_buffer_load_b128(rsW, pad ? kOOB : wvoff, sa * 64, 0);
        if constexpr (MODE == 0) {
            va = __builtin_amdgcn_raw_buffer_load_b128(rsA, pad ? kOOB : avoff, sa * 64, 0);
        } else {
            // k = tap * 512 + chunk * (64 / KB): tap = sa / CPT (dy = tap / 3 - 1, dx = tap % 3 - 1), chunk = sa % CPT
            const int tap = sa / CPT, c = sa % CPT, dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
            const bool ok = (unsigned)(py + dy) < 4u && (unsigned)(px + dx) < 4u && avoff != kOOB && !pad;
            va = __builtin_amdgcn_raw_buffer_load_b128(rsA, ok ? avoff + (dy * 4 + dx) * PIXB : kOOB, c * 64, 0);
        }
    };
    auto store = [&](int s, const i32x4& va, const i32x4& vw) {   // slab s -> slot (s / 4) & 1, position s % 4
        char* const d = lds + ((s >> 2) & 1) * GRP + (s & 3) * SLAB + ldst;
        *reinterpret_cast<i32x4*>(d) = va;
        *reinterpret_cast<i32x4*>(d + 8192) = vw;
    };
    // ---- fragments: A rows 64 wm + 16 i + r16, W rows 32 wn + 16 j + r16 (16-B k-group kg, swizzled) ----
    const int afr = (64 * wm + r16) * 64 + ((kg ^ wsw(r16)) << 4);
    // S16: the h half of W read by every lane (k-group kg & 1) and the l half (2 + (kg & 1))
    const int bfr = 8192 + (32 * wn + r16) * 64 + (((S16 ? kg & 1 : kg) ^ wsw(r16)) << 4);
    const int bfl = 8192 + (32 * wn + r16) * 64 + (((2 + (kg & 1)) ^ wsw(r16)) << 4);
    i32x4 fa[2][4], fb[2][2], fl[2][2];
    auto read = [&](int s, int buf) {
        const char* const b = lds + ((s >> 2) & 1) * GRP + (s & 3) * SLAB;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[buf][i] = lds16(b + afr + 1024 * i);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[buf][j] = lds16(b + bfr + 1024 * j);
        if constexpr (S16) {
#pragma unroll
            for (int j = 0; j < 2; ++j) fl[buf][j] = lds16(b + bfl + 1024 * j);
        }
    };
    f32x4 acc[4][2], blk[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = blk[i][0] = blk[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
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
    if constexpr (S16) {
        // one fp32 summation block per iteration: the block's MFMAs into blk (the h-weight products of all eight
        // fragment blocks, then the l-weight ones: no MFMA waits on the one just issued; per accumulator k_conv's
        // order), then into the running sum.  Padded slabs read zeros (load) and add exact zeros: no branch in the
        // loop, so the wait counts stay exact.
        const int npad8 = (nsl + kFp32Block - 1) & ~(kFp32Block - 1);
        for (int s0 = 0; s0 < npad8; s0 += kFp32Block) {
#pragma unroll
            for (int q = 0; q < kFp32Block; ++q) {
                const int s = s0 + q;
                __builtin_amdgcn_sched_barrier(0);
                store(s + 4, ra[q & 3], rw[q & 3]);
                load(s + 8, ra[q & 3], rw[q & 3]);
                if ((q & 3) == 3) __syncthreads();
                read(s + 1, (q + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr ((ABL & 4) != 0) {   // ablation: no MFMAs (fragments kept live)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        blk[i][0][0] += __builtin_bit_cast(float, fa[q & 1][i][0] ^ fb[q & 1][i & 1][1] ^ fl[q & 1][i & 1][2]);
                    continue;
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            blk[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                __builtin_bit_cast(f16x8, fa[q & 1][i]), __builtin_bit_cast(f16x8, h ? fl[q & 1][j] : fb[q & 1][j]),
                                blk[i][j], 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] += blk[i][j];
                    blk[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
                }
        }
    }
    const int npad = S16 ? 0 : (nsl + 3) & ~3;
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
    // S16: out in halves, value (row, n) as the pair at (n / 16) * 32 + n % 16 and + 16 of the row's channel run
    bool bad = false;
    auto put = [&](long long base, int n, float v) {
        if constexpr (S16) {
            const _Float16 h = (_Float16)v, l = (_Float16)(v - (float)h);
            bad |= pair_out_of_range(v);
            unsigned short* o = reinterpret_cast<unsigned short*>(g.out) + base + (n >> 4) * 32 + (n & 15);
            o[0] = __builtin_bit_cast(unsigned short, h);
            o[16] = __builtin_bit_cast(unsigned short, l);
        } else {
            g.out[base + n] = (bf16_t)v;
        }
    };
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
                    put((long long)(mb + e) * g.ldo + g.out_off, n, v);
                }
            } else {
                float v = fmaxf(fmaxf(acc[i][j][0] * sc + sh, acc[i][j][1] * sc + sh),
                                fmaxf(acc[i][j][2] * sc + sh, acc[i][j][3] * sc + sh));
                if (g.act) v = v >= 0.f ? v : LRELU * v;
                const int clip = mb >> 4, q = (mb & 15) >> 2;   // pooled pixel q of the 2 x 2 output (HWC)
                put((long long)clip * g.ldo + g.out_off + q * g.N * (S16 ? 2 : 1), n, v);
            }
        }
    }
    if constexpr (S16) range_report(g.range_flag, g.range_bit, bad);
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

// AVSE_F32_SPLIT dense layers: splits of whole kFp32Block-slab blocks, the plan from K and N only (never M, so every
// batch takes the same splits and the same ordered reduction): as many splits as fill the 256 CUs at the bench
// batch's 4 row tiles
int gemm_s16_ksplit(int N, int kpad, int* slabs_per_split) {
    const int nblocks = (kpad / 16 + kFp32Block - 1) / kFp32Block, tiles_n = (N + 127) / 128;
    int ks = std::max(1, std::min(nblocks, 256 / (4 * tiles_n)));
    const int G = (nblocks + ks - 1) / ks;
    ks = (nblocks + G - 1) / G;
    if (slabs_per_split) *slabs_per_split = G * kFp32Block;
    return ks;
}

int launch_gemm(const GemmArgs& g, int mode, hipStream_t s) {
    const bool s16 = g.split != 0;
#ifndef AVSE_GEMM_ABL
#define AVSE_GEMM_ABL 0
#endif
    const void* kf = mode == 0 ? (s16 ? (const void*)k_gemm<0, AVSE_GEMM_ABL, true> : (const void*)k_gemm<0>)
                               : (s16 ? (const void*)k_gemm<1, AVSE_GEMM_ABL, true> : (const void*)k_gemm<1>);
    if (int rc = ensure_lds_attr(kf, LDS_BYTES)) return rc;
    const int kq = s16 ? 16 : 32;   // k per 64-B slab
    const int nslab = g.kpad / kq;
    // split: every split but the last holds whole blocks, and the splits cover the slabs exactly
    const bool s16_bad = s16 && (g.N % 16 || (g.ksplit > 1 && (g.slabs_per_split <= 0 || g.slabs_per_split % kFp32Block ||
                                                               (nslab + g.slabs_per_split - 1) / g.slabs_per_split != g.ksplit)));
    if (g.kpad % kq || g.M <= 0 || g.N <= 0 || g.ksplit < 1 || (g.ksplit > 1 && (!g.partial || !g.counters)) ||
        (mode == 1 && (g.M % 16 || g.kpad != 9 * 512)) || s16_bad) {
        set_error("gemm: bad arguments");
        return 3;
    }
    const dim3 grid((g.M + 127) / 128, (g.N + 127) / 128, g.ksplit);
    hipLaunchKernelGGL(reinterpret_cast<void (*)(GemmArgs)>(const_cast<void*>(kf)), grid, dim3(NT), LDS_BYTES, s, g);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
