// v_conv1 (network.py:139-143: Conv2D(128, 5x5, 'same') on the normalised 5-frame mouth crops ->
// BatchNorm -> LeakyReLU(0.3) -> MaxPooling2D(2x2)) fused with VideoNormalizer.normalize
// (data_processor.py:208-212) and the f32 -> bf16 cast, gfx950 — row-run formulation.
//
// The K axis is split by kernel row: K-slice ky holds k = kx * 6 + frame (kx < 5, frame < 6; frame 5 and
// k = 30, 31 carry zero weights).  The normalised window is stored in LDS as 12-byte pixels (frames 0..4
// as bf16 and a zero), so the 32 k of slice ky for output pixel (y, x) are the 64 contiguous bytes that
// start at window pixel (y + ky, x): the MFMA A fragments are read straight from the window (two
// ds_read2_b32 per fragment: the rows are only 4-byte aligned) and nothing is rearranged.  Against the
// dense im2col kernel (conv_v1.hip: K = 128 in 4 slices, loader waves rebuilding a 64-byte im2col row per
// lane per slice, one barrier per slice) this costs 5 slices of MFMAs instead of 4, but the loader work
// drops to one window per tile and the compute waves meet the loaders at one barrier per tile.
//   * 512 threads: 4 compute waves (v_mfma_f32_16x16x32_bf16, issue priority) + 4 loader waves;
//   * weights: 5 slices x 128 co x 32 k bf16 (40 KB) resident in LDS for the whole launch;
//   * window: 20 x 20 pixels x 12 B, two LDS slots; tile k+2's f32 window is in flight in the loader
//     registers while tile k computes, tile k+1's is normalised and stored;
//   * compute wave w owns conv-pixel rows 4w .. 4w+3 of the 16 x 16 tile as 4 blocks of 4x4 pixels x 128
//     output channels; block row r = 4 q + 2 dy + dx is pixel (2 (q >> 1) + dy, 2 (q & 1) + dx), so a lane's
//     4 accumulator rows are one 2x2 pool window and BN / pool / LeakyReLU happen in registers.
// Persistent over tiles in XCD-aware order (as conv_stream.hip).
#include "avse_common.h"

namespace avse {
AVSE_DEBUG_RECORD(debug_read_v1r)
namespace {

constexpr float LRELU = 0.3f;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr int kOOB = 0x7fffff00;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }
// weights image: row (slice, co) 64 B, 16-B k-group s at s ^ wsw(co) (conflict-free for the 16x16x32
// B-operand lane groups, tools/lds_swizzle_search.py)
__device__ __forceinline__ int wsw(int co) { return 2 * ((co >> 2) & 1); }

// NF (template): video frames per clip, 5 (25 / 29.97 fps) or 6 (30 fps: the 12-byte window pixel's sixth half
// holds a real frame instead of the zero, and the weights' k = kx * 6 + 5 rows are the sixth frame's)
constexpr int TH = 16, TW = 16, KS = 5, PAD = 2;
constexpr int HH = TH + KS - 1, HW = TW + KS - 1, HPIX = HH * HW;   // 20 x 20 window
constexpr int PB = 12;                                              // bytes per window pixel
// LDS row pitch 24 pixels (20 used): 20 gave 2-way bank conflicts on the A-fragment ds_read2_b32, 24 none
// (tools/lds_swizzle_search.py --v1r); columns 20..23 stay zero (the row run of x = 15 reads 4 B of x = 20)
constexpr int HWP = 24;
constexpr int HSLOT = HH * HWP * PB + 64;                           // + zero tail read by the last row runs
constexpr int NSL = KS;                                             // K-slices per tile (one per kernel row)
constexpr int WIMG = NSL * 128 * 64;                                // 40 KB resident weights
constexpr int SSH = 2 * 128 * 4;                                    // BN scale / shift
constexpr int NWS = 3;                                              // window slots
// pooled f32 tile (8 x 8 px x 128 co), row pitch 576 B: the compute waves' ds_write_b32 (pixels P, P+1 in
// one 32-lane group) land 16 banks apart, the loaders' lane-linear ds_read_b128 are conflict-free
constexpr int SPITCH = 576;
constexpr int STG = 64 * SPITCH;
constexpr int LDS_BYTES = WIMG + NWS * HSLOT + SSH + 2 * STG;
constexpr int LDS_LAUNCH = LDS_BYTES + (kDebugBuild ? 16 : 0);      // checked build: + the window-slot tags
constexpr int PPL = (HPIX + 255) / 256;                             // window pixels per loader lane (2)
static_assert(HSLOT % 16 == 0 && LDS_BYTES <= 160 * 1024, "LDS");

// ABL: ablation mask for tools/v1r_ablate.hip only (0 in the library): 1 = loaders skip the output pass,
// 2 = loaders skip the per-tile window work, 4 = no MFMAs, 8 = no barrier in the tile loop
template <int ABL = 0, int NF = 5>
__global__ __launch_bounds__(512, 1) void k_conv_v1r(HaloArgs a) {
    static_assert(NF == 5 || NF == 6, "frames");
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const wimg = lds;
    char* const halo = lds + WIMG;                  // [NWS][HSLOT]
    float* const ssh = reinterpret_cast<float*>(halo + NWS * HSLOT);
    char* const stg = halo + NWS * HSLOT + SSH;     // [2][STG] pooled raw maxima, compute -> loader
    int* const tags = reinterpret_cast<int*>(lds + LDS_BYTES);   // checked build: window index held by each slot

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;

    const int tiles_x = a.Wc / TW, tiles_per_clip = tiles_x * (a.Hc / TH);
    const int ntiles = a.N * tiles_per_clip;
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    auto tile_origin = [&](int k, int& clip, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip = t / tiles_per_clip;
        const int tt = t - clip * tiles_per_clip;
        oy0 = (tt / tiles_x) * TH;
        ox0 = (tt % tiles_x) * TW;
    };

    if (wave >= 4) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;
        {   // resident weights [slice][co][32] (host packing) and the BN tail
            const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, (long long)WIMG);
#pragma unroll
            for (int i = 0; i < WIMG / 16 / 256; ++i) {
                const int C = L + 256 * i, row = C >> 2, sl = C & 3;
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, C * 16, 0, 0);
                *reinterpret_cast<i32x4*>(wimg + row * 64 + ((sl ^ wsw(row & 127)) << 4)) = v;
            }
            if (L < 128) {
                ssh[L] = a.scale[L];
                ssh[128 + L] = a.shift[L];
            }
            // zero the pitch padding (columns 20..23) and the tails of both slots: never written afterwards
            for (int i = L; i < NWS * HSLOT / 4; i += 256) {
                const int off = (i * 4) % HSLOT;
                if (off >= HH * HWP * PB || (off / PB) % HWP >= HW) reinterpret_cast<int*>(halo)[i] = 0;
            }
        }
        const long long clip_bytes = (long long)a.Hc * a.Wc * NF * 4;
        const bool norm = a.vmean != nullptr;
        const __amdgpu_buffer_rsrc_t mrs = make_rsrc(norm ? a.vmean : a.video, (long long)a.Hc * a.Wc * 4);
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(norm ? a.vstd : a.video, (long long)a.Hc * a.Wc * 4);
        // two register sets: window k+2 is loaded two tiles ahead, so the vmcnt wait for it never waits on
        // output stores younger than two tiles (vmcnt retires in issue order, stores included)
        f32x4 v4[2][PPL];
        float v1[2][PPL], v5[2][PPL], pm[2][PPL], ps[2][PPL];
        int pok[2][PPL];
        auto win_load = [&](auto set, int k) {
            constexpr int Q = decltype(set)::value;
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const __amdgpu_buffer_rsrc_t vrs =
                make_rsrc(reinterpret_cast<const char*>(a.video) + (long long)clip * clip_bytes, clip_bytes);
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                const int wy = P / HW, wx = P - wy * HW;
                const int iy = oy0 + wy - PAD, ix = ox0 + wx - PAD;
                const int ok = (int)(P < HPIX) & (int)((unsigned)iy < (unsigned)a.Hc) & (int)((unsigned)ix < (unsigned)a.Wc);
                const int pix = iy * a.Wc + ix;
                const int voff = ok ? pix * NF * 4 : kOOB, moff = ok ? pix * 4 : kOOB;
                v4[Q][e] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, voff, 0, 0));
                v1[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 16, 0));
                if constexpr (NF == 6)
                    v5[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 20, 0));
                pm[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mrs, moff, 0, 0));
                ps[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, moff, 0, 0));
                pok[Q][e] = ok;
            }
        };
        // VideoNormalizer ((v - mean) / std, one reciprocal per pixel), then 'same' zero padding, bf16
        auto win_store = [&](auto set, int hs) {
            constexpr int Q = decltype(set)::value;
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                if (P >= HPIX) continue;
                // v_rcp_f32 (1 ulp) and packed conversions: the loader shares its SIMD's issue with the MFMA wave
                const float rs = __builtin_amdgcn_rcpf(ps[Q][e]);
                float f[6] = {v4[Q][e][0], v4[Q][e][1], v4[Q][e][2], v4[Q][e][3], v1[Q][e], NF == 6 ? v5[Q][e] : 0.f};
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const float n = norm ? (f[i] - pm[Q][e]) * rs : f[i];
                    f[i] = pok[Q][e] ? n : 0.f;
                }
                const int wy = P / HW, wx = P - wy * HW;
                unsigned* d = reinterpret_cast<unsigned*>(halo + hs * HSLOT + (wy * HWP + wx) * PB);
                d[0] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){f[0], f[1]}, bf16x2));
                d[1] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){f[2], f[3]}, bf16x2));
                d[2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){f[4], f[5]}, bf16x2));
            }
        };
        // output pass of tile k: BN (|scale|, shift) + LeakyReLU(0.3) on the pooled raw maxima the compute
        // waves left in staging slot k & 1, bf16, 8-B stores.  Float4 F = L + 256 r: pooled pixel F / 32,
        // channels 4 (F % 32) .. +3 (lane-constant), so a 32-lane half stores one pixel's 256 contiguous bytes
        const int c4 = (L & 31) * 4;
        float osc[4], osh[4];
        const int Wp = a.Wc / 2;
        // store offsets: a lane-constant VGPR part (pixel column L >> 5, channels c4) and a wave-uniform part per
        // tile and row, passed as the store's soffset.  (A per-tile 32-bit VGPR product here was emitted as
        // v_mad_u64_u32 whose undefined high addend half reused a window-load destination register, so the
        // compiler's waitcnt pass drained every window load in flight at each output pass.)
        const int ovlane = ((L >> 5) * a.out_pix_stride + a.out_c_off + c4) * 2;
        const int orow = Wp * a.out_pix_stride * 2;
        auto out_pass = [&](int k) {
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const long long cb = a.out_clip_stride * 2;
            const __amdgpu_buffer_rsrc_t ors = make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip * cb, cb);
            const char* sbase = stg + (k & 1) * STG + (L >> 5) * SPITCH + c4 * 4;
            const int otile = __builtin_amdgcn_readfirstlane(((oy0 >> 1) * Wp + (ox0 >> 1)) * a.out_pix_stride * 2);
#pragma unroll
            for (int r = 0; r < 8; ++r) {   // pooled pixel (r, L >> 5) of the 8 x 8 tile
                const f32x4 m = *reinterpret_cast<const f32x4*>(sbase + 8 * r * SPITCH);
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = fmaf(m[e], osc[e], osh[e]);
                    asm("v_max_f32 %0, %1, %2" : "=v"(v[e]) : "v"(x), "v"(LRELU * x));   // LeakyReLU, no canonicalise
                }
                const bf16x2 lo = __builtin_convertvector((f32x2){v[0], v[1]}, bf16x2);
                const bf16x2 hi = __builtin_convertvector((f32x2){v[2], v[3]}, bf16x2);
                const i32x2 o = {__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi)};
                __builtin_amdgcn_raw_buffer_store_b64(o, ors, ovlane, otile + r * orow, 0);
            }
        };
        using Q0 = std::integral_constant<int, 0>;
        using Q1 = std::integral_constant<int, 1>;
        // checked build: one loader lane tags the slot after the window's LDS stores (a wave's LDS operations
        // complete in order); the compute waves compare the tags at both ends of a tile
        auto tag = [&](int hs, int k) {
            if (kDebugBuild && L == 0) tags[hs] = k;
        };
        win_load(Q0{}, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        win_store(Q0{}, 0);
        tag(0, 0);
        if (nmine > 1) {
            win_load(Q1{}, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            win_store(Q1{}, 1);
            tag(1, 1);
        }
        if (nmine > 2) win_load(Q0{}, 2);
        if (nmine > 3) win_load(Q1{}, 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // B_-1: weights, BN tail, windows 0 and 1
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            osc[e] = ssh[c4 + e];
            osh[e] = ssh[128 + c4 + e];
        }
        // iteration k (set k & 1 holds window k+2): output pass of tile k-1, window k+2 -> LDS slot (k+2) % 3,
        // window k+4's loads into the freed set, barrier B_k
        auto iter = [&](auto set, int k) {
            const bool out = k >= 1 && !(ABL & 1);
            if (out) out_pass(k - 1);
            if (k + 2 < nmine && !(ABL & 2)) {
                // no hand-counted vmcnt here: the window registers are ordinary results of the buffer-load
                // builtins, so the compiler's waitcnt pass waits for exactly the loads each store reads (with
                // the stores and window k+3's loads issued after them still in flight; DESIGN.md §3 v_conv1)
                win_store(set, (k + 2) % NWS);     // slot of window k-1, last read during tile k-1
                tag((k + 2) % NWS, k + 2);
                if (k + 4 < nmine) win_load(set, k + 4);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (!(ABL & 8)) barrier_raw();   // B_k: staging k written, window k+2 stored
        };
        for (int k = 0; k < nmine; k += 2) {
            iter(Q0{}, k);
            if (k + 1 < nmine) iter(Q1{}, k + 1);
        }
        if (!(ABL & 1)) out_pass(nmine - 1);
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    const int r16 = lane & 15, kg = lane >> 4;
    const int q = r16 >> 2, dy = (r16 >> 1) & 1, dx = r16 & 1;
    // window byte offset of this lane's 16 bytes of slice 0 in block 0: pixel (4w + 2(q>>1) + dy, 2(q&1) + dx)
    const int abase = ((4 * w + 2 * (q >> 1) + dy) * HWP + 2 * (q & 1) + dx) * PB + 16 * kg;
    const int bbase = r16 * 64 + ((kg ^ wsw(r16)) << 4);   // + slice * 8192 + 1024 j
    auto frags = [&](int hs, int ky, i32x4 (&fa)[4], i32x4 (&fb)[8]) {
        const char* hp = halo + hs * HSLOT + abase + ky * HWP * PB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned* p = reinterpret_cast<const unsigned*>(hp + 4 * i * PB);   // block i: 4 pixels right
            fa[i] = (i32x4){(int)p[0], (int)p[1], (int)p[2], (int)p[3]};
        }
        const char* wp = wimg + ky * 8192 + bbase;
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[j] = *reinterpret_cast<const i32x4*>(wp + 1024 * j);
    };
    barrier_raw();   // B_-1

    f32x4 acc[4][8];
    // pool: the 4 accumulator rows of a lane are one 2x2 window (raw maxima: scale >= 0 after the host sign
    // fold, so BN commutes); inline asm keeps the compiler from canonicalising the operands (2 instead of 4
    // instructions per window).  The loader waves apply BN / LeakyReLU and store (out_pass).
    auto max4 = [](f32x4 v) {
        float r;
        asm volatile("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, %0, %4" : "=&v"(r) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
        return r;
    };
    // staging: pooled pixel P = (2w + (kg >> 1)) * 8 + 2i + (kg & 1), channel 16 j + r16 at P * SPITCH + 4 co
    char* const sl0 = stg + ((2 * w + (kg >> 1)) * 8 + (kg & 1)) * SPITCH + r16 * 4;
    auto epilogue = [&](int k) {
        char* const sb = sl0 + (k & 1) * STG;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) *reinterpret_cast<float*>(sb + 2 * i * SPITCH + 64 * j) = max4(acc[i][j]);
    };
    // the first K-slice of a tile starts its chains from a zero C operand (no restart instructions in the epilogue)
    auto mfmas = [&](const i32x4 (&ca)[4], const i32x4 (&cb)[8], bool first) {
        if constexpr ((ABL & 4) != 0) return;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ca[i]),
                                                                     __builtin_bit_cast(bf16x8, cb[j]),
                                                                     first ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
    };
    // slice s: MFMAs on (ca, cb) interleaved with the fragment reads of slice s+1 into (xa, xb)
    auto slice = [&](int hs, int ky_next, i32x4 (&ca)[4], i32x4 (&cb)[8], i32x4 (&xa)[4], i32x4 (&xb)[8], bool first) {
        frags(hs, ky_next, xa, xb);
        mfmas(ca, cb, first);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    i32x4 fa[4], fb[8], na[4], nb[8];
    // one tile: slice 0 in (xa, xb); tile k+1's slice 0 lands in (ya, yb) (parity flips per tile)
    auto tile = [&](int k, i32x4 (&xa)[4], i32x4 (&xb)[8], i32x4 (&ya)[4], i32x4 (&yb)[8]) {
        const int hs = k % NWS, hn = (k + 1) % NWS;
        if (kDebugBuild && lane == 0) {   // after B_{k-1}: window k in slot hs (and k + 1 in hn, read in slice 4)
            AVSE_CHECK_DEV(tags[hs] == k, DK_V1R, 1, tags[hs], k);
            if (k + 1 < nmine) AVSE_CHECK_DEV(tags[hn] == k + 1, DK_V1R, 2, tags[hn], k + 1);
        }
        slice(hs, 1, xa, xb, ya, yb, true);
        slice(hs, 2, ya, yb, xa, xb, false);
        slice(hs, 3, xa, xb, ya, yb, false);
        slice(hs, 4, ya, yb, xa, xb, false);
        // slice 4, with tile k+1's first fragments (window k+1 was stored before B_{k-1}; past the last tile
        // the read hits a stale slot and is never used)
        slice(hn, 0, xa, xb, ya, yb, false);
        if (kDebugBuild && lane == 0) AVSE_CHECK_DEV(tags[hs] == k, DK_V1R, 3, tags[hs], k);   // not yet replaced
        epilogue(k);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!(ABL & 8)) barrier_raw();   // B_k: staging k is written; window k is no longer read
    };
    frags(0, 0, fa, fb);
    for (int k = 0; k < nmine; k += 2) {
        tile(k, fa, fb, na, nb);
        if (k + 1 < nmine) tile(k + 1, na, nb, fa, fb);
    }
}

// ------------------------------------------------------------------------------------------------------------
// k_conv_v1s: v_conv1 with split-f16 operands (AVSE_F32_SPLIT, DESIGN.md §3 "split-f16"), the same row-run K
// layout.  The normalised window is stored twice — h = f16(x) and l = f16(x - h), 12-byte pixels each — and the
// weights as Bh / Bl images [piece][kernel row][Co][32] f16 (80 KB, resident; scaled by a per-channel power of two
// that the BN scale undoes).  A K-slice is three groups of 32 v_mfma_f32_16x16x32_f16 (Ah Bh, Ah Bl, Al Bh, each MFMA
// rounding its 32 products once into fp32; Al Bl dropped, see V1S_LL), ordered so that at most 24 fragments are live:
//   Ah Bh (reading Bl) -> Ah Bl (reading Al, then the next slice's Ah) -> Al Bh (reading the next slice's Bh).
// With four times the MFMAs per window the compute waves run the epilogue themselves (BN + LeakyReLU on the pooled
// maxima, split, stores into the next layer's split-pair layout: per pixel and 16 channels [h(16) | l(16)]); the
// loader waves only stage windows.  Window / barrier protocol as k_conv_v1r (3 slots, window k+2 stored while
// tile k computes).
constexpr int HIMG = HSLOT;                                    // one window image (h or l)
constexpr int SSLOT = 2 * HIMG;                                // window slot: h image, l image
constexpr int WIMG_S = 2 * NSL * 128 * 64;                     // Bh, Bl: 80 KB
constexpr int LDS_S = WIMG_S + NWS * SSLOT + SSH;
// the l x l product (2^-22 of |a b|, below the pieces' own representation error) is dropped: three MFMA groups per
// K-slice instead of four (AVSE_V1S_LL=1 keeps it, for A/B and accuracy checks)
#ifndef AVSE_V1S_LL
#define AVSE_V1S_LL 0
#endif
constexpr bool V1S_LL = AVSE_V1S_LL != 0;
// ablation builds only (0 in the library): 1 = no epilogue stores, 2 = loaders skip the window staging, 4 = no MFMAs
#ifndef AVSE_V1S_ABL
#define AVSE_V1S_ABL 0
#endif
constexpr int V1S_ABL = AVSE_V1S_ABL;
static_assert(LDS_S <= 160 * 1024, "LDS (split v_conv1)");
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// CW compute waves + 4 loader waves.  CW = 4: compute wave w owns conv rows 4w .. 4w+3 x all 128 channels (one
// compute wave per SIMD); CW = 8: rows 4 (w & 3) .. x channels 64 (w >> 2) .. +63 — two compute waves per SIMD, so one
// wave's MFMAs cover the other's LDS waits (half the accumulators, the A fragments read by both)
template <int CW, int NF = 5>
__global__ __launch_bounds__(64 * (CW + 4), 1) void k_conv_v1s(HaloArgs a) {
    static_assert(CW == 4 || CW == 8, "compute waves");
    static_assert(NF == 5 || NF == 6, "frames");
    constexpr int NJ = 32 / CW;                      // 16-channel column blocks per compute wave
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const wimg = lds;                          // [2 pieces][5 rows][128 co][64 B]
    char* const halo = lds + WIMG_S;                 // [NWS][h image | l image]
    float* const ssh = reinterpret_cast<float*>(halo + NWS * SSLOT);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave < CW ? (wave & 3) : wave - CW;   // compute: row block; loader: loader index
    const int cb0 = wave < CW ? (wave >> 2) * NJ : 0;  // compute: first column block

    const int tiles_x = a.Wc / TW, tiles_per_clip = tiles_x * (a.Hc / TH);
    const int ntiles = a.N * tiles_per_clip;
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    auto tile_origin = [&](int k, int& clip, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip = t / tiles_per_clip;
        const int tt = t - clip * tiles_per_clip;
        oy0 = (tt / tiles_x) * TH;
        ox0 = (tt % tiles_x) * TW;
    };

    if (wave >= CW) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;
        {
            const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, (long long)WIMG_S);
#pragma unroll
            for (int i = 0; i < WIMG_S / 16 / 256; ++i) {
                const int C = L + 256 * i, row = C >> 2, sl = C & 3;
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, C * 16, 0, 0);
                *reinterpret_cast<i32x4*>(wimg + row * 64 + ((sl ^ wsw(row & 127)) << 4)) = v;
            }
            if (L < 128) {
                ssh[L] = a.scale[L];
                ssh[128 + L] = a.shift[L];
            }
            for (int i = L; i < NWS * SSLOT / 4; i += 256) {   // pitch padding and tails of every image
                const int off = (i * 4) % HIMG;
                if (off >= HH * HWP * PB || (off / PB) % HWP >= HW) reinterpret_cast<int*>(halo)[i] = 0;
            }
        }
        const long long clip_bytes = (long long)a.Hc * a.Wc * NF * 4;
        const bool norm = a.vmean != nullptr;
        const __amdgpu_buffer_rsrc_t mrs = make_rsrc(norm ? a.vmean : a.video, (long long)a.Hc * a.Wc * 4);
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(norm ? a.vstd : a.video, (long long)a.Hc * a.Wc * 4);
        f32x4 v4[2][PPL];
        float v1[2][PPL], v5[2][PPL], pm[2][PPL], ps[2][PPL];
        int pok[2][PPL];
        auto win_load = [&](auto set, int k) {
            constexpr int Q = decltype(set)::value;
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const __amdgpu_buffer_rsrc_t vrs =
                make_rsrc(reinterpret_cast<const char*>(a.video) + (long long)clip * clip_bytes, clip_bytes);
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                const int wy = P / HW, wx = P - wy * HW;
                const int iy = oy0 + wy - PAD, ix = ox0 + wx - PAD;
                const int ok = (int)(P < HPIX) & (int)((unsigned)iy < (unsigned)a.Hc) & (int)((unsigned)ix < (unsigned)a.Wc);
                const int pix = iy * a.Wc + ix;
                const int voff = ok ? pix * NF * 4 : kOOB, moff = ok ? pix * 4 : kOOB;
                v4[Q][e] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, voff, 0, 0));
                v1[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 16, 0));
                if constexpr (NF == 6)
                    v5[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 20, 0));
                pm[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mrs, moff, 0, 0));
                ps[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, moff, 0, 0));
                pok[Q][e] = ok;
            }
        };
        // VideoNormalizer ((v - mean) / std: an IEEE division, the reference's numpy op), 'same' zero padding, split
        bool in_bad = false;   // range guard of the split video input (avse_common.h pair_out_of_range)
        auto win_store = [&](auto set, int hs) {
            constexpr int Q = decltype(set)::value;
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                if (P >= HPIX) continue;
                float f[6] = {v4[Q][e][0], v4[Q][e][1], v4[Q][e][2], v4[Q][e][3], v1[Q][e], NF == 6 ? v5[Q][e] : 0.f};
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const float n = norm ? (f[i] - pm[Q][e]) / ps[Q][e] : f[i];
                    f[i] = pok[Q][e] ? n : 0.f;
                }
                _Float16 h[6], l[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    h[i] = (_Float16)f[i];
                    l[i] = (_Float16)(f[i] - (float)h[i]);
                    in_bad |= pair_out_of_range(f[i]);
                }
                const int wy = P / HW, wx = P - wy * HW;
                unsigned* dh = reinterpret_cast<unsigned*>(halo + hs * SSLOT + (wy * HWP + wx) * PB);
                unsigned* dl = reinterpret_cast<unsigned*>(halo + hs * SSLOT + HIMG + (wy * HWP + wx) * PB);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    dh[i] = __builtin_bit_cast(unsigned, (f16x2){h[2 * i], h[2 * i + 1]});
                    dl[i] = __builtin_bit_cast(unsigned, (f16x2){l[2 * i], l[2 * i + 1]});
                }
            }
        };
        using Q0 = std::integral_constant<int, 0>;
        using Q1 = std::integral_constant<int, 1>;
        win_load(Q0{}, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        win_store(Q0{}, 0);
        if (nmine > 1) {
            win_load(Q1{}, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            win_store(Q1{}, 1);
        }
        if (nmine > 2) win_load(Q0{}, 2);
        if (nmine > 3) win_load(Q1{}, 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // B_-1: weights, BN tail, windows 0 and 1
        auto iter = [&](auto set, int k) {
            if (k + 2 < nmine) {
                if constexpr (!(V1S_ABL & 2)) win_store(set, (k + 2) % NWS);   // slot of window k-1, last read during tile k-1
                if (k + 4 < nmine) win_load(set, k + 4);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();   // B_k: window k+2 stored; window k is no longer read
        };
        for (int k = 0; k < nmine; k += 2) {
            iter(Q0{}, k);
            if (k + 1 < nmine) iter(Q1{}, k + 1);
        }
        range_report(a.range_flag, a.range_in_bit, in_bad);
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    const int r16 = lane & 15, kg = lane >> 4;
    const int q = r16 >> 2, dy = (r16 >> 1) & 1, dx = r16 & 1;
    const int abase = ((4 * w + 2 * (q >> 1) + dy) * HWP + 2 * (q & 1) + dx) * PB + 16 * kg;
    const int bbase = r16 * 64 + ((kg ^ wsw(r16)) << 4) + 1024 * cb0;   // + piece * 40960 + slice * 8192 + 1024 j
    auto fragA = [&](int hs, int piece, int ky, i32x4 (&fa)[4]) {
        const char* hp = halo + hs * SSLOT + piece * HIMG + abase + ky * HWP * PB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned* p = reinterpret_cast<const unsigned*>(hp + 4 * i * PB);
            fa[i] = (i32x4){(int)p[0], (int)p[1], (int)p[2], (int)p[3]};
        }
    };
    auto fragB = [&](int piece, int ky, i32x4 (&fb)[NJ]) {
        const char* wp = wimg + piece * (NSL * 8192) + ky * 8192 + bbase;
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = *reinterpret_cast<const i32x4*>(wp + 1024 * j);
    };
    barrier_raw();   // B_-1

    f32x4 acc[4][NJ];
    auto mfmas = [&](const i32x4 (&ca)[4], const i32x4 (&cb)[NJ], bool first) {
        if constexpr ((V1S_ABL & 4) != 0) {   // keep the fragments live without the matrix work
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][0][0] += __builtin_bit_cast(float, ca[i][0] ^ cb[i][1]);
            return;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ca[i]),
                                                                    __builtin_bit_cast(f16x8, cb[j]),
                                                                    first ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
    };
    // a group of 4 NJ MFMAs with ND DS reads spread over it (at most one read per MFMA, the rest after the last)
    auto sched = [](auto nds) {
        constexpr int ND = decltype(nds)::value, NM = 4 * NJ, P = ND < NM ? ND : NM;
#pragma unroll
        for (int r = 0; r < P; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        }
        if constexpr (NM > P) __builtin_amdgcn_sched_group_barrier(0x008, NM - P, 0);
        if constexpr (ND > P) __builtin_amdgcn_sched_group_barrier(0x100, ND - P, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // K-slice ky of window slot hs, with (ah, bh) = its Ah / Bh fragments in registers; reads the next slice's
    // (hsn, kyn) Ah / Bh into (nah, nbh)
    auto slice = [&](int hs, int ky, int hsn, int kyn, i32x4 (&ah)[4], i32x4 (&bh)[NJ], i32x4 (&nah)[4],
                     i32x4 (&nbh)[NJ], bool first) {
        i32x4 bl[NJ], al[4];
        fragB(1, ky, bl);
        mfmas(ah, bh, first);
        sched(std::integral_constant<int, NJ>{});
        fragA(hs, 1, ky, al);
        mfmas(ah, bl, false);
        sched(std::integral_constant<int, 16>{});
        fragA(hsn, 0, kyn, nah);
        if constexpr (V1S_LL) {
            mfmas(al, bl, false);
            sched(std::integral_constant<int, 16>{});
            fragB(0, kyn, nbh);
        } else {
            fragB(0, kyn, nbh);
        }
        mfmas(al, bh, false);
        sched(std::integral_constant<int, V1S_LL ? NJ : 16 + NJ>{});
    };
    const int Wp = a.Wc / 2;
    const long long cbytes = a.out_clip_stride * 2;
    bool bad = false;   // range guard of the stored pairs
    auto epilogue = [&](int k) {
        int clip, oy0, ox0;
        tile_origin(k, clip, oy0, ox0);
        const __amdgpu_buffer_rsrc_t ors = make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip * cbytes, cbytes);
        const int py = (oy0 >> 1) + 2 * w + (kg >> 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int px = (ox0 >> 1) + 2 * i + (kg & 1);
            const int pbase = (py * Wp + px) * a.out_pix_stride + a.out_c_off + 32 * cb0 + r16;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const float mx = fmaxf(fmaxf(acc[i][j][0], acc[i][j][1]), fmaxf(acc[i][j][2], acc[i][j][3]));
                const int co = 16 * (cb0 + j) + r16;
                float x = fmaf(mx, ssh[co], ssh[128 + co]);
                x = fmaxf(x, LRELU * x);
                const _Float16 h = (_Float16)x;
                const _Float16 l = (_Float16)(x - (float)h);
                bad |= pair_out_of_range(x);
                if constexpr (V1S_ABL & 1) {
                    if (x == 12345.f) __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ors, 0, 0, 0);
                    continue;
                }
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ors, (pbase + 32 * j) * 2, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, l), ors, (pbase + 32 * j + 16) * 2, 0, 0);
            }
        }
    };
    i32x4 fa[4], fb[NJ], na[4], nb[NJ];
    auto tile = [&](int k, i32x4 (&xa)[4], i32x4 (&xb)[NJ], i32x4 (&ya)[4], i32x4 (&yb)[NJ]) {
        const int hs = k % NWS, hn = (k + 1) % NWS;
        slice(hs, 0, hs, 1, xa, xb, ya, yb, true);
        slice(hs, 1, hs, 2, ya, yb, xa, xb, false);
        slice(hs, 2, hs, 3, xa, xb, ya, yb, false);
        slice(hs, 3, hs, 4, ya, yb, xa, xb, false);
        // slice 4 reads tile k+1's first fragments (window k+1 was stored before B_{k-1}; past the last tile the
        // read hits a stale slot and is never used)
        slice(hs, 4, hn, 0, xa, xb, ya, yb, false);
        epilogue(k);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // B_k: window k is no longer read
    };
    fragA(0, 0, 0, fa);
    fragB(0, 0, fb);
    for (int k = 0; k < nmine; k += 2) {
        tile(k, fa, fb, na, nb);
        if (k + 1 < nmine) tile(k + 1, na, nb, fa, fb);
    }
    range_report(a.range_flag, a.range_bit, bad);
}

// ------------------------------------------------------------------------------------------------------------
// k_conv_v1p: split v_conv1 for 5-frame clips (25 / 29.97 fps) with K = 128 instead of k_conv_v1s's 5 x 32 = 160 (125
// real k: 22 % of v1s's MFMA products multiply zero weights).  The 16 k-groups of 8 (four K-slices of 32) are each two
// 8-byte LDS reads per lane from one window image laid out per window row y' (0..19) as
//   P  at   0: pixel x' (0..19): frames 0..3                                (8 B)
//   R  at 160: x (0..15): frame 4 of pixels x .. x + 3 of the row           (8 B)
//   S0 at 288: x (0..15), rows y' < 16: frame 4 of pixels (y' .. y' + 3, x + 4)
//   S1 at 416: x (0..15), rows y' < 16: frame 4 of pixel (y' + 4, x + 4), three zeros
// and the groups, g = 4 slice + kg (kg = lane >> 4; the B image's k order, capi.hip build_layer HALO_V1P):
//   slice 0, kg = ky (0..3): P(py + ky, px), P(py + ky, px + 1)        kx 0, 1 x frames 0..3
//   slice 1, kg = ky:        P(py + ky, px + 2), P(py + ky, px + 3)    kx 2, 3 x frames 0..3
//   slice 2, kg = ky:        P(py + ky, px + 4), R(py + ky, px)        kx 4 x frames 0..3, then kx 0..3 x frame 4
//   slice 3: kg 0..2 = slices 0..2's groups for ky = 4; kg 3: S0(py, px), S1(py, px)   (ky 0..4, kx 4) x frame 4
// so that in slices 0..2 a lane's offsets are its row base + kg rows + a constant (ds_read immediates).
// Row pitch 544 B: 8 extra LDS cycles over the 64 of a slice's conflict-free A reads (bank model of
// MI355X_MICROARCH.md §LDS, ds_read_b64: two 32-lane groups, banks (a / 4) mod 64).  The loaders scatter frame 4
// into R / S0 / S1 (ds_write_b16); S1's zero halves are written once.  Everything else is k_conv_v1s: three MFMA
// groups per slice (Ah Bh, Ah Bl, Al Bh), compute waves run the epilogue, three window slots.
constexpr int VP_PITCH = 544, VP_R = 160, VP_S0 = 288, VP_S1 = 416;
constexpr int VP_IMG = HH * VP_PITCH;                          // one piece (h or l) of a window
constexpr int VP_SLOT = 2 * VP_IMG;
constexpr int VP_NSL = 4;                                      // K-slices
constexpr int VP_WIMG = 2 * VP_NSL * 128 * 64;                 // Bh, Bl: 64 KB
constexpr int LDS_P = VP_WIMG + NWS * VP_SLOT + SSH;
static_assert(LDS_P <= 160 * 1024 && VP_SLOT % 16 == 0, "LDS (packed split v_conv1)");
static_assert(VP_R >= HW * 8 && VP_S0 >= VP_R + TW * 8 && VP_S1 >= VP_S0 + TW * 8 && VP_PITCH >= VP_S1 + TW * 8, "row");

template <int CW>
__global__ __launch_bounds__(64 * (CW + 4), 1) void k_conv_v1p(HaloArgs a) {
    static_assert(CW == 4 || CW == 8, "compute waves");
    constexpr int NF = 5;
    constexpr int NJ = 32 / CW;
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const wimg = lds;                          // [2 pieces][4 slices][128 co][64 B]
    char* const halo = lds + VP_WIMG;                // [NWS][h image | l image]
    float* const ssh = reinterpret_cast<float*>(halo + NWS * VP_SLOT);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave < CW ? (wave & 3) : wave - CW;
    const int cb0 = wave < CW ? (wave >> 2) * NJ : 0;

    const int tiles_x = a.Wc / TW, tiles_per_clip = tiles_x * (a.Hc / TH);
    const int ntiles = a.N * tiles_per_clip;
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    auto tile_origin = [&](int k, int& clip, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip = t / tiles_per_clip;
        const int tt = t - clip * tiles_per_clip;
        oy0 = (tt / tiles_x) * TH;
        ox0 = (tt % tiles_x) * TW;
    };

    if (wave >= CW) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;
        {
            const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, (long long)VP_WIMG);
#pragma unroll
            for (int i = 0; i < VP_WIMG / 16 / 256; ++i) {
                const int C = L + 256 * i, row = C >> 2, sl = C & 3;
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, C * 16, 0, 0);
                *reinterpret_cast<i32x4*>(wimg + row * 64 + ((sl ^ wsw(row & 127)) << 4)) = v;
            }
            if (L < 128) {
                ssh[L] = a.scale[L];
                ssh[128 + L] = a.shift[L];
            }
            // S1's three zero halves of every entry (never written by the window stores, which write its first half)
            for (int i = L; i < NWS * 2 * TH * TW; i += 256) {
                const int img = i / (TH * TW), e = i - img * (TH * TW);
                char* p = halo + img * VP_IMG + (e / TW) * VP_PITCH + VP_S1 + (e % TW) * 8;
                *reinterpret_cast<unsigned short*>(p + 2) = 0;
                *reinterpret_cast<unsigned*>(p + 4) = 0u;
            }
        }
        const long long clip_bytes = (long long)a.Hc * a.Wc * NF * 4;
        const bool norm = a.vmean != nullptr;
        const __amdgpu_buffer_rsrc_t mrs = make_rsrc(norm ? a.vmean : a.video, (long long)a.Hc * a.Wc * 4);
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(norm ? a.vstd : a.video, (long long)a.Hc * a.Wc * 4);
        f32x4 v4[2][PPL];
        float v1[2][PPL], pm[2][PPL], ps[2][PPL];
        int pok[2][PPL];
        auto win_load = [&](auto set, int k) {
            constexpr int Q = decltype(set)::value;
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const __amdgpu_buffer_rsrc_t vrs =
                make_rsrc(reinterpret_cast<const char*>(a.video) + (long long)clip * clip_bytes, clip_bytes);
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                const int wy = P / HW, wx = P - wy * HW;
                const int iy = oy0 + wy - PAD, ix = ox0 + wx - PAD;
                const int ok = (int)(P < HPIX) & (int)((unsigned)iy < (unsigned)a.Hc) & (int)((unsigned)ix < (unsigned)a.Wc);
                const int pix = iy * a.Wc + ix;
                const int voff = ok ? pix * NF * 4 : kOOB, moff = ok ? pix * 4 : kOOB;
                v4[Q][e] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, voff, 0, 0));
                v1[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 16, 0));
                pm[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mrs, moff, 0, 0));
                ps[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, moff, 0, 0));
                pok[Q][e] = ok;
            }
        };
        bool in_bad = false;
        auto win_store = [&](auto set, int hs) {
            constexpr int Q = decltype(set)::value;
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int P = L + 256 * e;
                if (P >= HPIX) continue;
                float f[5] = {v4[Q][e][0], v4[Q][e][1], v4[Q][e][2], v4[Q][e][3], v1[Q][e]};
                _Float16 h[5], l[5];
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const float n = norm ? (f[i] - pm[Q][e]) / ps[Q][e] : f[i];
                    f[i] = pok[Q][e] ? n : 0.f;
                    h[i] = (_Float16)f[i];
                    l[i] = (_Float16)(f[i] - (float)h[i]);
                    in_bad |= pair_out_of_range(f[i]);
                }
                const int wy = P / HW, wx = P - wy * HW;
#pragma unroll
                for (int pc = 0; pc < 2; ++pc) {
                    const _Float16* v = pc ? l : h;
                    char* img = halo + hs * VP_SLOT + pc * VP_IMG;
                    *reinterpret_cast<i32x2*>(img + wy * VP_PITCH + wx * 8) =
                        (i32x2){(int)__builtin_bit_cast(unsigned, (f16x2){v[0], v[1]}),
                                (int)__builtin_bit_cast(unsigned, (f16x2){v[2], v[3]})};
                    const unsigned short q = __builtin_bit_cast(unsigned short, v[4]);
#pragma unroll
                    for (int j = 0; j < 4; ++j)   // R(wy, wx - j)[j]
                        if (wx - j >= 0 && wx - j < TW)
                            *reinterpret_cast<unsigned short*>(img + wy * VP_PITCH + VP_R + (wx - j) * 8 + 2 * j) = q;
                    if (wx >= 4) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)   // S0(wy - i, wx - 4)[i]
                            if (wy - i >= 0 && wy - i < TH)
                                *reinterpret_cast<unsigned short*>(img + (wy - i) * VP_PITCH + VP_S0 + (wx - 4) * 8 + 2 * i) = q;
                        if (wy >= 4)   // S1(wy - 4, wx - 4)[0] (wy - 4 < 16 always)
                            *reinterpret_cast<unsigned short*>(img + (wy - 4) * VP_PITCH + VP_S1 + (wx - 4) * 8) = q;
                    }
                }
            }
        };
        using Q0 = std::integral_constant<int, 0>;
        using Q1 = std::integral_constant<int, 1>;
        win_load(Q0{}, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        win_store(Q0{}, 0);
        if (nmine > 1) {
            win_load(Q1{}, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            win_store(Q1{}, 1);
        }
        if (nmine > 2) win_load(Q0{}, 2);
        if (nmine > 3) win_load(Q1{}, 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // B_-1: weights, BN tail, windows 0 and 1
        auto iter = [&](auto set, int k) {
            if (k + 2 < nmine) {
                if constexpr (!(V1S_ABL & 2)) win_store(set, (k + 2) % NWS);
                if (k + 4 < nmine) win_load(set, k + 4);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();   // B_k: window k+2 stored; window k is no longer read
        };
        for (int k = 0; k < nmine; k += 2) {
            iter(Q0{}, k);
            if (k + 1 < nmine) iter(Q1{}, k + 1);
        }
        range_report(a.range_flag, a.range_in_bit, in_bad);
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    const int r16 = lane & 15, kg = lane >> 4;
    const int q = r16 >> 2, dy = (r16 >> 1) & 1, dx = r16 & 1;
    const int py = 4 * w + 2 * (q >> 1) + dy, px = 2 * (q & 1) + dx;
    const int bbase = r16 * 64 + ((kg ^ wsw(r16)) << 4) + 1024 * cb0;   // + piece * 32768 + slice * 8192 + 1024 j
    // fragment (piece, slice s, column block i) of window slot hs: two 8-B reads at the lane's k-group offsets
    const int pbk = (py + kg) * VP_PITCH + px * 8;   // slices 0..2: + the slice's constant
    // slice 3: kg < 3 the ky = 4 groups of slices 0..2, kg = 3 S0 / S1
    const int o30 = kg == 3 ? py * VP_PITCH + px * 8 + VP_S0 : (py + 4) * VP_PITCH + px * 8 + 16 * kg;
    const int o31 = kg == 3 ? o30 + (VP_S1 - VP_S0) : kg == 2 ? o30 + (VP_R - 32) : o30 + 8;
    // The lane's base address is rebuilt per fragment set from the slot (an SGPR) and pinned, so that the compiler
    // addresses the pieces by immediates instead of holding one precomputed address per (slot, piece, slice, i) in
    // VGPRs (16 spills); contiguous piece pairs merge into ds_read2_b64 (8 cycles per 16 B, like v1s's two
    // ds_read2_b32; conflict-free at the 544-B pitch: 16 lanes at 32 r + 8 c mod 128 B)
    auto fragA = [&](int hs, int piece, int s, i32x4 (&fa)[4]) {
        const int sb = hs * VP_SLOT + piece * VP_IMG;
        if (s < 3) {
            int b0 = sb + pbk;
            asm volatile("" : "+v"(b0));
            const char* hp = halo + b0 + 16 * s;
            constexpr int D[3] = {8, 8, VP_R - 32};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const i32x2 x0 = *reinterpret_cast<const i32x2*>(hp + 32 * i);
                const i32x2 x1 = *reinterpret_cast<const i32x2*>(hp + D[s < 3 ? s : 0] + 32 * i);
                fa[i] = (i32x4){x0[0], x0[1], x1[0], x1[1]};
            }
        } else {
            int b0 = sb + o30, b1 = sb + o31;
            asm volatile("" : "+v"(b0), "+v"(b1));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const i32x2 x0 = *reinterpret_cast<const i32x2*>(halo + b0 + 32 * i);
                const i32x2 x1 = *reinterpret_cast<const i32x2*>(halo + b1 + 32 * i);
                fa[i] = (i32x4){x0[0], x0[1], x1[0], x1[1]};
            }
        }
    };
    auto fragB = [&](int piece, int s, i32x4 (&fb)[NJ]) {
        const char* wp = wimg + piece * (VP_NSL * 8192) + s * 8192 + bbase;
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = *reinterpret_cast<const i32x4*>(wp + 1024 * j);
    };
    barrier_raw();   // B_-1

    f32x4 acc[4][NJ];
    auto mfmas = [&](const i32x4 (&ca)[4], const i32x4 (&cb)[NJ], bool first) {
        if constexpr ((V1S_ABL & 4) != 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][0][0] += __builtin_bit_cast(float, ca[i][0] ^ cb[i][1]);
            return;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ca[i]),
                                                                    __builtin_bit_cast(f16x8, cb[j]),
                                                                    first ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
    };
    auto sched = [](auto nds) {
        constexpr int ND = decltype(nds)::value, NM = 4 * NJ, P = ND < NM ? ND : NM;
#pragma unroll
        for (int r = 0; r < P; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        }
        if constexpr (NM > P) __builtin_amdgcn_sched_group_barrier(0x008, NM - P, 0);
        if constexpr (ND > P) __builtin_amdgcn_sched_group_barrier(0x100, ND - P, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // slice s of window slot hs, (ah, bh) its Ah / Bh fragments; reads the next slice's (hsn, sn) Ah / Bh
    auto slice = [&](int hs, int s, int hsn, int sn, i32x4 (&ah)[4], i32x4 (&bh)[NJ], i32x4 (&nah)[4],
                     i32x4 (&nbh)[NJ], bool first) {
        i32x4 bl[NJ], al[4];
        fragB(1, s, bl);
        mfmas(ah, bh, first);
        sched(std::integral_constant<int, NJ>{});
        fragA(hs, 1, s, al);
        mfmas(ah, bl, false);
        sched(std::integral_constant<int, 8>{});
        fragA(hsn, 0, sn, nah);
        fragB(0, sn, nbh);
        mfmas(al, bh, false);
        sched(std::integral_constant<int, 8 + NJ>{});
    };
    const int Wp = a.Wc / 2;
    const long long cbytes = a.out_clip_stride * 2;
    bool bad = false;
    auto epilogue = [&](int k) {
        int clip, oy0, ox0;
        tile_origin(k, clip, oy0, ox0);
        const __amdgpu_buffer_rsrc_t ors = make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip * cbytes, cbytes);
        const int opy = (oy0 >> 1) + 2 * w + (kg >> 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int opx = (ox0 >> 1) + 2 * i + (kg & 1);
            const int pbase = (opy * Wp + opx) * a.out_pix_stride + a.out_c_off + 32 * cb0 + r16;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const float mx = fmaxf(fmaxf(acc[i][j][0], acc[i][j][1]), fmaxf(acc[i][j][2], acc[i][j][3]));
                const int co = 16 * (cb0 + j) + r16;
                float x = fmaf(mx, ssh[co], ssh[128 + co]);
                x = fmaxf(x, LRELU * x);
                const _Float16 h = (_Float16)x;
                const _Float16 l = (_Float16)(x - (float)h);
                bad |= pair_out_of_range(x);
                if constexpr (V1S_ABL & 1) {
                    if (x == 12345.f) __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ors, 0, 0, 0);
                    continue;
                }
                // (measured: dword channel pairs, the partner's pieces by DPP, 0.693 vs 0.663 ms, r06o)
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ors, (pbase + 32 * j) * 2, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, l), ors, (pbase + 32 * j + 16) * 2, 0, 0);
            }
        }
    };
    i32x4 fa[4], fb[NJ], na[4], nb[NJ];
    // The two compute waves of a SIMD (w, w + 4) take turns on the matrix pipe: wave w runs tile k's epilogue after its
    // MFMAs, wave w + 4 before tile k + 1's (past the barrier: the epilogue reads no window), so between two barriers
    // one wave's BN / split / stores overlap the other's MFMAs instead of both idling the pipe at once
#ifndef AVSE_V1P_STAGGER
#define AVSE_V1P_STAGGER 1
#endif
    const bool late = AVSE_V1P_STAGGER && CW == 8 && wave >= 4;
    auto tile = [&](int k, i32x4 (&xa)[4], i32x4 (&xb)[NJ], i32x4 (&ya)[4], i32x4 (&yb)[NJ]) {
        const int hs = k % NWS, hn = (k + 1) % NWS;
        slice(hs, 0, hs, 1, xa, xb, ya, yb, true);
        slice(hs, 1, hs, 2, ya, yb, xa, xb, false);
        slice(hs, 2, hs, 3, xa, xb, ya, yb, false);
        // slice 3 reads tile k+1's first fragments (past the last tile a stale slot, never used)
        slice(hs, 3, hn, 0, ya, yb, xa, xb, false);
        if (!late) epilogue(k);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // B_k: window k is no longer read
    };
    fragA(0, 0, 0, fa);
    fragB(0, 0, fb);
    for (int k = 0; k < nmine; ++k) {
        if (late && k > 0) epilogue(k - 1);
        tile(k, fa, fb, na, nb);
    }
    if (late) epilogue(nmine - 1);
    range_report(a.range_flag, a.range_bit, bad);
}

}  // namespace

#ifndef AVSE_V1S_CW
#define AVSE_V1S_CW 8
#endif
int launch_conv_v1r(const HaloArgs& a, hipStream_t s) {
    if (a.variant == HALO_V1P) {
        constexpr int CW = AVSE_V1S_CW;
        if (int rc = ensure_lds_attr((const void*)k_conv_v1p<CW>, LDS_P)) return rc;
        if (!a.split || a.Hc % TH || a.Wc % TW || a.Co != 128 || a.Ci != 5 || !a.w || a.out_mode != OUT_S16) {
            set_error("v_conv1 packed split kernel: unexpected layer shape, packing or output format");
            return 3;
        }
        int dev = 0, ncu = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        const int tiles = a.N * (a.Hc / TH) * (a.Wc / TW);
        int gx = ncu >= 8 ? ncu / 8 * 8 : ncu;
        if (gx > tiles) gx = tiles;
        hipLaunchKernelGGL((k_conv_v1p<CW>), dim3(gx), dim3(64 * (CW + 4)), LDS_P, s, a);
        AVSE_HIP_CHECK(hipGetLastError());
        return 0;
    }
    if (a.split) {
        constexpr int CW = AVSE_V1S_CW;
        const void* kf = a.Ci == 6 ? (const void*)k_conv_v1s<CW, 6> : (const void*)k_conv_v1s<CW, 5>;
        if (int rc = ensure_lds_attr(kf, LDS_S)) return rc;
        if (a.Hc % TH || a.Wc % TW || a.Co != 128 || (a.Ci != 5 && a.Ci != 6) || !a.w || a.out_mode != OUT_S16) {
            set_error("v_conv1 split kernel: unexpected layer shape, packing or output format");
            return 3;
        }
        int dev = 0, ncu = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        const int tiles = a.N * (a.Hc / TH) * (a.Wc / TW);
        int gx = ncu >= 8 ? ncu / 8 * 8 : ncu;
        if (gx > tiles) gx = tiles;
        if (a.Ci == 6) hipLaunchKernelGGL((k_conv_v1s<CW, 6>), dim3(gx), dim3(64 * (CW + 4)), LDS_S, s, a);
        else hipLaunchKernelGGL((k_conv_v1s<CW, 5>), dim3(gx), dim3(64 * (CW + 4)), LDS_S, s, a);
        AVSE_HIP_CHECK(hipGetLastError());
        return 0;
    }
    const void* kf = a.Ci == 6 ? (const void*)k_conv_v1r<0, 6> : (const void*)k_conv_v1r<0, 5>;
    if (int rc = ensure_lds_attr(kf, LDS_LAUNCH)) return rc;
    if (a.Hc % TH || a.Wc % TW || a.Co != 128 || (a.Ci != 5 && a.Ci != 6) || !a.w) {
        set_error("v_conv1 row-run kernel: unexpected layer shape or missing packing");
        return 3;
    }
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = a.N * (a.Hc / TH) * (a.Wc / TW);
    int gx = ncu >= 8 ? ncu / 8 * 8 : ncu;
    if (gx > tiles) gx = tiles;
    if (a.Ci == 6) hipLaunchKernelGGL((k_conv_v1r<0, 6>), dim3(gx), dim3(512), LDS_LAUNCH, s, a);
    else hipLaunchKernelGGL((k_conv_v1r<0, 5>), dim3(gx), dim3(512), LDS_LAUNCH, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
