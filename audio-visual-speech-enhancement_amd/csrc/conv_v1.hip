// v_conv1 (network.py:139-143: Conv2D(128, 5x5, 'same') on the normalised 5-frame mouth crops ->
// BatchNorm -> LeakyReLU(0.3) -> MaxPooling2D(2x2)) fused with VideoNormalizer.normalize
// (data_processor.py:208-212) and the f32 -> bf16 cast, gfx950.
//
// With 5 input channels a tap-major K wastes most of every MFMA (the previous kernel padded each tap to
// 8 channels and 28 taps: K = 224 for 125 real products).  Here the K axis is the dense im2col order
// k = tap * 5 + frame (125, padded to 128 = 4 K-slices of 32), so v_conv1 costs 4 slices of MFMAs per
// tile instead of 7.  Structure as in conv_stream.hip (persistent, 4 compute + 4 loader waves, one of
// each per SIMD, v_mfma_f32_32x32x16_bf16, one barrier per K-slice):
//   * weights: all 128 x 128 bf16 (32 KB) stay resident in LDS;
//   * loader waves fetch the 20 x 20-pixel f32 input window of a tile two steps ahead, normalise it
//     with the per-pixel mean / std images, and store it as bf16 (16 B per pixel: frames 0..4, zeros)
//     in a 2-tile halo ring;
//   * each step, loader lane L assembles the 64-byte im2col row of tile row L for the K-slice two steps
//     ahead from 7 halo pixels (compile-time dword shuffles) into a 3-slot slice ring;
//   * compute waves read A fragments from the slice ring and B fragments from the resident weights.
// M order and epilogue as in conv_stream.hip (32-row blocks of 4 x 8 pixels, pool windows in registers).
//
// LDS images (bank-conflict free for the compute waves' ds_read_b128 lane groups):
//   slice slot: row L (0..255) 64 B, 16-B chunk j at position j ^ ((L >> 2) & 3);
//   weights:    row co (0..127) 256 B, 16-B chunk j (k = 8j .. 8j+7) at position j ^ (co & 15).
#include "avse_common.h"

namespace avse {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }

constexpr int TH = 16, TW = 16, KS = 5, PAD = 2, NF = 5;       // tile, kernel, padding, frames
constexpr int HH = TH + KS - 1, HW = TW + KS - 1, HPIX = HH * HW;   // 20 x 20 window
constexpr int KP = 128;                                          // padded K (125 real)
constexpr int NSL = KP / 32;                                     // K-slices per tile
constexpr int BPR = TW / 8;                                      // 4x8-pixel blocks per tile row
constexpr int WIMG = 128 * KP * 2;                               // 32 KB resident weights
constexpr int SSLOT = 256 * 64;                                  // 16 KB slice slot
constexpr int HSLOT = HPIX * 16;                                 // 6.4 KB halo slot
constexpr int LDS_BYTES = WIMG + 3 * SSLOT + 2 * HSLOT;
constexpr int PPL = (HPIX + 255) / 256;                          // window pixels per loader lane (2)
static_assert(LDS_BYTES > 80 * 1024 && LDS_BYTES <= 160 * 1024, "one persistent workgroup per CU");

// ABL: ablation mask for tools/v1_ablate.hip only (0 in the library): 1 = no epilogue, 2 = loaders do
// not build im2col slices, 4 = loaders do not load / store input windows, 8 = no MFMAs
template <int ABL = 0>
__global__ __launch_bounds__(512, 1) void k_conv_v1(HaloArgs a) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const wimg = lds;
    char* const ring = lds + WIMG;                 // [3][SSLOT]
    char* const halo = ring + 3 * SSLOT;           // [2][HSLOT]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;

    const int tiles_x = a.Wc / TW, tiles_per_clip = tiles_x * (a.Hc / TH);
    const int ntiles = a.N * tiles_per_clip;
    // XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (XCD = linear id % 8), so
    // slot bx % 8 * (gx / 8) + bx / 8 gives each XCD a contiguous run of tiles per round (whole clips): the
    // halo rows neighbouring tiles share are then fetched into that XCD's L2 once
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    const int total = nmine * NSL;
    auto tile_origin = [&](int k, int& clip, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip = t / tiles_per_clip;
        const int tt = t - clip * tiles_per_clip;
        oy0 = (tt / tiles_x) * TH;
        ox0 = (tt % tiles_x) * TW;
    };

    if (wave >= 4) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;   // tile row this lane assembles
        // resident weights: 128 rows x 16 chunks, chunk (co, j) at co*256 + ((j ^ (co & 15)) << 4)
        {
            const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, (long long)WIMG);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int C = L + 256 * i, co = C >> 4, j = C & 15;
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, C * 16, 0, 0);
                *reinterpret_cast<i32x4*>(wimg + co * 256 + ((j ^ (co & 15)) << 4)) = v;
            }
        }
        // this row's window pixel (tap (0,0)) and its slice-slot byte offsets
        int hrow;
        {
            const int b = L >> 5, r = L & 31, q = r >> 2;
            const int y = 4 * (b / BPR) + 2 * (q >> 2) + ((r >> 1) & 1);
            const int x = 8 * (b % BPR) + 2 * (q & 3) + (r & 1);
            hrow = (y * HW + x) * 16;
        }
        const int sw = (L >> 2) & 3;
        // window pixel loads of a tile: pixel P = L + 256 e (e < PPL), 5 frames + mean + std each
        const long long clip_bytes = (long long)a.Hc * a.Wc * NF * 4;
        const bool norm = a.vmean != nullptr;
        const __amdgpu_buffer_rsrc_t mrs = make_rsrc(norm ? a.vmean : a.video, (long long)a.Hc * a.Wc * 4);
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(norm ? a.vstd : a.video, (long long)a.Hc * a.Wc * 4);
        // two register sets: tile j's window is loaded into set j & 1 seven steps before it is stored
        float px[2][PPL][NF], pm[2][PPL], ps[2][PPL];
        int pok[2][PPL];
        auto halo_load = [&](auto set, int k) {
            constexpr int Q = decltype(set)::value;
            int clip, oy0, ox0;
            tile_origin(k < nmine ? k : nmine - 1, clip, oy0, ox0);
            const __amdgpu_buffer_rsrc_t vrs =
                make_rsrc(reinterpret_cast<const char*>(a.video) + (long long)clip * clip_bytes, clip_bytes);
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                const int wy = P / HW, wx = P - wy * HW;
                const int iy = oy0 + wy - PAD, ix = ox0 + wx - PAD;
                const int ok = (int)(P < HPIX) & (int)((unsigned)iy < (unsigned)a.Hc) & (int)((unsigned)ix < (unsigned)a.Wc);
                const int pix = iy * a.Wc + ix, mask = -ok;
                const int voff = ((pix * NF * 4) & mask) | (kOOB & ~mask);
                const int moff = ((pix * 4) & mask) | (kOOB & ~mask);
#pragma unroll
                for (int f = 0; f < NF; ++f)
                    px[Q][e][f] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff + 4 * f, 0, 0));
                pm[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mrs, moff, 0, 0));
                ps[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, moff, 0, 0));
                pok[Q][e] = ok;
            }
        };
        // normalise (VideoNormalizer: (v - mean) / std; 'same' padding is zero AFTER normalisation) and
        // store the window as bf16 pixels of 16 B
        // (one reciprocal per pixel: within 1 ulp of the division, far below the bf16 rounding that follows)
        auto halo_store = [&](auto set, int slot) {
            constexpr int Q = decltype(set)::value;
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                const float rs = 1.f / ps[Q][e];
                bf16x8 v;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const float n = norm ? (px[Q][e][f] - pm[Q][e]) * rs : px[Q][e][f];
                    v[f] = (bf16_t)(pok[Q][e] ? n : 0.f);
                }
                v[5] = v[6] = v[7] = (bf16_t)0.f;
                if (P < HPIX) *reinterpret_cast<bf16x8*>(halo + slot * HSLOT + P * 16) = v;
            }
        };
        // im2col row L of K-slice S (k = 32 S .. 32 S + 31, k = tap * 5 + frame) from halo slot hs
        auto build = [&](auto sidx, int hs, int rslot) {
            constexpr int S = decltype(sidx)::value;
            constexpr int T0 = (32 * S) / NF, T1 = (32 * S + 31) / NF < 24 ? (32 * S + 31) / NF : 24;
            i32x4 d[T1 - T0 + 2];
#pragma unroll
            for (int t = T0; t <= T1; ++t) {
                const int off = ((t / KS) * HW + (t % KS)) * 16;
                d[t - T0] = *reinterpret_cast<const i32x4*>(halo + hs * HSLOT + hrow + off);
            }
            d[T1 - T0 + 1] = (i32x4){0, 0, 0, 0};
            int o[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int k = 32 * S + 2 * i;
                if (k >= 125) {
                    o[i] = 0;
                    continue;
                }
                const int t = k / NF - T0, c = k % NF;
                const unsigned lo = (unsigned)d[t][c >> 1], hi2 = (unsigned)d[t + (c == 4)][((c + 1) % NF) >> 1];
                if (c == 0 || c == 2) o[i] = (int)lo;                                    // (c, c+1) of one tap
                else if (c == 4) o[i] = (int)((lo & 0xffffu) | (hi2 << 16));             // (4 of t, 0 of t+1)
                else o[i] = (int)__builtin_amdgcn_alignbit(hi2, lo, 16);                 // (c, c+1) across dwords
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<i32x4*>(ring + rslot * SSLOT + L * 64 + ((j ^ sw) << 4)) =
                    (i32x4){o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]};
        };

        using Q0 = std::integral_constant<int, 0>;
        using Q1 = std::integral_constant<int, 1>;
        constexpr int NLD = PPL * (NF + 2);   // loads per window set
        // prologue: tile 0's window to halo slot 0, slices 0 and 1 to ring slots 0 and 1; windows of
        // tiles 1 and 2 in flight (stored at step 1 of tiles 0 and 1)
        halo_load(Q0{}, 0);
        wait_vm_lgkm0<0>();
        halo_store(Q0{}, 0);
        wait_vm_lgkm0<0>();
        barrier_raw();   // loader-internal: halo visible to all loader lanes (compute waves join too)
        build(std::integral_constant<int, 0>{}, 0, 0);
        build(std::integral_constant<int, 1>{}, 0, 1);
        halo_load(Q1{}, 1);
        halo_load(Q0{}, 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();

        // step t of tile k (S = t % 4): build slice S+2 (this tile) or S-2 (next tile) into ring slot
        // (t+2)%3; S == 1: store tile k+1's window (set (k+1)&1, loaded at step 2 of tile k-2) into halo
        // slot (k+1)&1, free since tile k-1's last build; S == 2: issue tile k+3's window loads into the
        // set just stored (vmcnt retires in order: at S == 1 the loads of tile k+2 may stay in flight)
        int rs = 2;   // ring slot (t + 2) % 3
        auto tile = [&](auto par, int k) {
            constexpr int hk = decltype(par)::value;     // k & 1
            auto lstep = [&](auto sidx) {
                constexpr int S = decltype(sidx)::value;
                if constexpr (S == 1 && !(ABL & 4)) {
                    wait_vm_lgkm0<NLD>();
                    halo_store(std::integral_constant<int, hk ^ 1>{}, hk ^ 1);
                }
                if constexpr (!(ABL & 2)) {
                    if constexpr (S < 2) build(std::integral_constant<int, S + 2>{}, hk, rs);
                    else build(std::integral_constant<int, S - 2>{}, hk ^ 1, rs);
                }
                if constexpr (S == 2 && !(ABL & 4)) halo_load(std::integral_constant<int, hk ^ 1>{}, k + 3);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                barrier_raw();
                rs = rs == 2 ? 0 : rs + 1;
            };
            lstep(std::integral_constant<int, 0>{});
            lstep(std::integral_constant<int, 1>{});
            lstep(std::integral_constant<int, 2>{});
            lstep(std::integral_constant<int, 3>{});
        };
        int k = 0;
        for (; k + 1 < nmine; k += 2) {
            tile(Q0{}, k);
            tile(Q1{}, k + 1);
        }
        if (k < nmine) tile(Q0{}, k);
        wait_vm_lgkm0<0>();
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    const int r32 = lane & 31, hi = lane >> 5;
    const int arow = (64 * w + r32) * 64;                 // block 2w row r32 in a slice slot (+ 2048 for block 2w+1)
    const int asw = (r32 >> 2) & 3;
    const int bsw = r32 & 15;
    auto frags = [&](int slot, int S, i32x4 (&fa)[4], i32x4 (&fb)[8]) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int ca = 2 * m + hi;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                fa[2 * i + m] = *reinterpret_cast<const i32x4*>(ring + slot * SSLOT + arow + i * 2048 + ((ca ^ asw) << 4));
            const int j = 4 * S + 2 * m + hi;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                fb[2 * jb + m] = *reinterpret_cast<const i32x4*>(wimg + (32 * jb + r32) * 256 + ((j ^ bsw) << 4));
        }
    };
    float sc[4], sh[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        sc[jb] = a.scale[32 * jb + r32];
        sh[jb] = a.shift[32 * jb + r32];
    }
    barrier_raw();   // loader prologue: halo of tile 0
    barrier_raw();   // loader prologue: slices 0, 1

    f32x16 acc[2][4];
    const int Wp = a.Wc / 2;
    // scale >= 0 (host sign fold), so pooling the raw accumulators then one FMA equals BN-then-pool exactly;
    // LeakyReLU(0.3) = max(x, 0.3 x); 32-bit offsets into a per-clip buffer resource.  (Transposing the
    // wave's pooled pixels through LDS for 16-B stores measured 6% slower: the epilogue is VALU-bound.)
    auto epilogue = [&](int clip, int oy0, int ox0) {
        const __amdgpu_buffer_rsrc_t ors =
            make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip * a.out_clip_stride * 2, a.out_clip_stride * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int b = 2 * w + i;
            const int py0 = (oy0 + 4 * (b / BPR)) / 2, px0 = (ox0 + 8 * (b % BPR)) / 2;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const int co = 32 * jb + r32;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int q = 2 * g + hi;
                    const int py = py0 + (q >> 2), pxx = px0 + (q & 3);
                    const float mx = fmaxf(fmaxf(acc[i][jb][4 * g], acc[i][jb][4 * g + 1]),
                                           fmaxf(acc[i][jb][4 * g + 2], acc[i][jb][4 * g + 3]));
                    float x = fmaf(mx, sc[jb], sh[jb]);
                    x = fmaxf(x, LRELU * x);
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)x), ors,
                                                          ((py * Wp + pxx) * a.out_pix_stride + a.out_c_off + co) * 2, 0, 0);
                }
            }
        }
    };
    i32x4 fa[4], fb[8], na[4], nb[8];
    frags(0, 0, fa, fb);
    int slot1 = 1;   // ring slot of the next slice ((t + 1) % 3)
    auto cstep = [&](auto first, auto sidx, i32x4 (&ca)[4], i32x4 (&cb)[8], i32x4 (&xa)[4], i32x4 (&xb)[8]) {
        constexpr int S = decltype(sidx)::value;
        frags(slot1, (S + 1) & 3, xa, xb);
        if constexpr (!(ABL & 8))
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, ca[2 * i + m]), __builtin_bit_cast(bf16x8, cb[2 * jb + m]),
                        (decltype(first)::value && m == 0) ? (f32x16){} : acc[i][jb], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_barrier(0);
        // LDS reads only: the epilogue's global stores (vmcnt on gfx9) are never waited for
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();
        slot1 = slot1 == 2 ? 0 : slot1 + 1;
    };
    for (int k = 0; k < nmine; ++k) {
        cstep(std::true_type{}, std::integral_constant<int, 0>{}, fa, fb, na, nb);
        cstep(std::false_type{}, std::integral_constant<int, 1>{}, na, nb, fa, fb);
        cstep(std::false_type{}, std::integral_constant<int, 2>{}, fa, fb, na, nb);
        cstep(std::false_type{}, std::integral_constant<int, 3>{}, na, nb, fa, fb);
        int clip, oy0, ox0;
        tile_origin(k, clip, oy0, ox0);
        if constexpr (!(ABL & 1)) epilogue(clip, oy0, ox0);
    }
    (void)total;
}

}  // namespace

int launch_conv_v1(const HaloArgs& a, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_v1<0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
        attr = true;
    }
    if (a.Hc % TH || a.Wc % TW || a.Co != 128 || a.Ci != NF) {
        set_error("v_conv1 kernel: unexpected layer shape");
        return 3;
    }
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = a.N * (a.Hc / TH) * (a.Wc / TW);
    const int gx = tiles < ncu ? tiles : ncu;
    hipLaunchKernelGGL(k_conv_v1<0>, dim3(gx), dim3(512), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
