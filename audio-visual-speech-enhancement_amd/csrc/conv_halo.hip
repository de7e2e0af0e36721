// Halo-tiled MFMA convolution for the video encoder (network.py:138-175), bf16, gfx950.
//
// Each 512-thread workgroup (8 wavefronts, 2 per SIMD) owns a 256-pixel output tile
// (NCLIP clips x TH x TW conv pixels) x 128 output channels.  The input window of the tile
// (TH+KS-1) x (TW+KS-1) x 128 channels is staged in LDS ONCE per 128-channel group and every
// tap reads its A fragments from it with a shifted address — 25x (5x5) / 9x (3x3) less L2
// traffic than an im2col gather.  Weights stream through a double-buffered 8 KB LDS slot per
// K-step (one 16-byte load per thread per step), K-step = 32 input channels of one tap
// (one v_mfma_f32_16x16x32_bf16 per 16x16 tile).
//
// M ordering: a 16-row MFMA fragment is a 4x4 block of conv pixels = 2x2 pooled pixels; the four
// accumulator rows a lane holds are one 2x2 pool window, so MaxPooling2D (network.py:142) is
// done in registers in the epilogue after the folded BN scale/shift, then LeakyReLU.
//
// LDS halo layout: one 256-byte row per pixel (128 bf16 channels, sixteen 16-byte slots); slot s
// of pixel (y, x) is stored at slot s ^ (((x & 3) << 1) | ((y & 1) << 3)).  With the fragment
// ordering above this makes every ds_read_b128 of an A fragment bank-conflict free for every
// tap offset (exhaustively checked over the four lane groups and all 16 (y, x) phases).
//
// V1 mode (v_conv1, Cin = 5): the halo holds 8 channels per pixel (16 bytes: 5 normalised video
// frames + 3 zeros); the loader fuses VideoNormalizer.normalize (data_processor.py:208-212) and
// the f32 -> bf16 cast, reading the raw [N][128][128][5] float32 video.  A K-step covers 4 taps x
// 8 channels (lane group g takes tap 4*step + g).
#include <cstdlib>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;

__device__ __forceinline__ int wswz(int row) { return ((row >> 3) & 1) * 3; }
__device__ __forceinline__ int hswz(int y, int x) { return ((x & 3) << 1) | ((y & 1) << 3); }

// Bounds-checked loads through a buffer resource spanning the clips [clip0, N) of an NHWC tensor:
// an offset at or past the range returns zeros in hardware, so TF 'SAME' zero padding and ragged
// clip tiles need no branch (a branch around each load makes hipcc drain vmcnt per load).
constexpr int kOOB = 0x7fffff00;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t clip_rsrc(const void* base, int clip0, long long clip_bytes, int N) {
    long long rem = (long long)(N - clip0) * clip_bytes;
    if (rem < 0) rem = 0;
    const int nrec = rem > kOOB ? kOOB : (int)rem;
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (long long)clip0 * clip_bytes), (short)0, nrec,
                                             0x00020000);
}

// ABL: ablation mask for tools/halo_ablate.hip only (0 in the library): 1 = no fragment reads in
// the K loop, 2 = no per-step barrier, 4 = no halo staging, 8 = no weight streaming, 16 = no MFMAs.
template <int KS, int TH, int TW, int NCLIP, bool V1, bool SCHED, int ABL = 0>
__global__ __launch_bounds__(512, 2) void k_conv_halo(HaloArgs a) {
    constexpr int HH = TH + KS - 1, HW = TW + KS - 1;
    constexpr int HPIX = NCLIP * HH * HW;                 // halo pixels
    constexpr int PIXB = V1 ? 16 : 256;                   // bytes per halo pixel
    constexpr int HBYTES = ((HPIX * PIXB + 255) / 256) * 256;
    constexpr int BPR = TW / 4;                           // 4x4 blocks per tile row
    constexpr int BPC = (TH / 4) * BPR;                   // blocks per clip tile
    static_assert(NCLIP * TH * TW == 256, "tile must be 256 conv pixels");
    constexpr int NTAP = KS * KS;
    constexpr int SPG = halo_slices_per_group(KS, V1);    // K-slices per channel group
    static_assert(V1 || SPG == 4 * KS * KS, "non-V1 slices: 4 chunks x KS^2 taps, no padding");
    constexpr int HCH = V1 ? 1 : (HPIX * 16 + 511) / 512; // 16-B halo chunks per thread
    constexpr int WSTEP = HALO_NT * 8192;                 // weight bytes per barrier step

    extern __shared__ __attribute__((aligned(16))) char lds[];
    char* halo = lds;                                     // + one 256-byte slack row (HBYTES)
    char* wbuf = lds + HBYTES + 256;                      // 3 x HALO_NT x [128 co][64 B]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int wm = wid & 3, wn = wid >> 2;
    const int fr = lane & 15, fg = lane >> 4;

    // tile coordinates
    const int tiles_x = a.Wc / TW, tiles_y = a.Hc / TH;
    const int t = blockIdx.x;
    const int clip0 = (t / (tiles_x * tiles_y)) * NCLIP;
    const int tt = t % (tiles_x * tiles_y);
    const int oy0 = (tt / tiles_x) * TH, ox0 = (tt % tiles_x) * TW;   // conv-pixel origin of the tile
    const int co0 = blockIdx.y * 128;
    constexpr int PAD = (KS - 1) / 2;

    // per-lane fragment origins (halo coords of tap (0,0) for this lane's row)
    int fy[4], fx[4], fcl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int F = wm * 4 + i;
        const int cl = F / BPC, b = F % BPC;
        const int r = fr;
        const int q = r >> 2;
        fcl[i] = cl;
        fy[i] = 4 * (b / BPR) + 2 * (q >> 1) + ((r >> 1) & 1);
        fx[i] = 4 * (b % BPR) + 2 * (q & 1) + (r & 1);
    }
    // byte offset of each fragment row's tap-(0,0) pixel in the halo; x & 3 and y & 1 of a lane's
    // pixels do not depend on the fragment (block origins are multiples of 4)
    int abase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) abase[i] = ((fcl[i] * HH + fy[i]) * HW + fx[i]) * PIXB;
    const int xm = fx[0] & 3, ym = fy[0] & 1;
    int boff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + 16 * j + fr;
        boff[j] = row * 64 + ((fg ^ wswz(row)) << 4);
    }

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int ngroups = V1 ? 1 : a.Ci / 128;
    constexpr int steps_per_group = SPG / HALO_NT;
    // weights: [slice][Co][32] bf16; this block's 128 channels of one slice are 8 KB contiguous
    const char* wsrc = reinterpret_cast<const char*>(a.w) + (size_t)co0 * 64;
    const size_t wslice = (size_t)a.Co * 64;
    const int wrow = tid >> 2, wg = tid & 3;
    const int woff = wrow * 64 + ((wg ^ wswz(wrow)) << 4);

    for (int cg = 0; cg < ngroups; ++cg) {
        __syncthreads();   // previous group's readers are done with halo / wbuf
        // ---- stage the halo for channel group cg ----
        if constexpr ((ABL & 4) != 0) {
        } else if constexpr (V1) {
            for (int p = tid; p < HPIX; p += 512) {
                const int cl = p / (HH * HW), rr = p % (HH * HW);
                const int y = rr / HW, x = rr % HW;
                const int iy = oy0 + y - PAD, ix = ox0 + x - PAD;
                const int clip = clip0 + cl;
                bf16x8 v;
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = (bf16_t)0.f;
                if (clip < a.N && iy >= 0 && iy < a.Hc && ix >= 0 && ix < a.Wc) {
                    const float* src = a.video + (((size_t)clip * a.Hc + iy) * a.Wc + ix) * 5;
                    float m = 0.f, sd = 1.f;
                    if (a.vmean) { m = a.vmean[iy * a.Wc + ix]; sd = a.vstd[iy * a.Wc + ix]; }
#pragma unroll
                    for (int c = 0; c < 5; ++c) v[c] = (bf16_t)(a.vmean ? (src[c] - m) / sd : src[c]);
                }
                *reinterpret_cast<bf16x8*>(halo + p * 16) = v;
            }
        } else {
            const __amdgpu_buffer_rsrc_t rs = clip_rsrc(a.in, clip0, (long long)a.Hc * a.Wc * a.Ci * 2, a.N);
            i32x4 hv[HCH];
#pragma unroll
            for (int h = 0; h < HCH; ++h) {
                const int c = tid + 512 * h;
                const int p = min(c >> 4, HPIX - 1), sl = c & 15;
                const int cl = p / (HH * HW), rr = p % (HH * HW);
                const int y = rr / HW, x = rr % HW;
                const int iy = oy0 + y - PAD, ix = ox0 + x - PAD;
                const bool ok = (c >> 4) < HPIX && iy >= 0 && iy < a.Hc && ix >= 0 && ix < a.Wc;
                const int off = ok ? (((cl * a.Hc + iy) * a.Wc + ix) * a.Ci + cg * 128 + sl * 8) * 2 : kOOB;
                hv[h] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
            }
#pragma unroll
            for (int h = 0; h < HCH; ++h) {
                const int c = tid + 512 * h;
                const int p = c >> 4, sl = c & 15;
                const int rr = p % (HH * HW);
                const int y = rr / HW, x = rr % HW;
                // pieces past the halo land in the 256-byte slack row after it
                const int dst = p < HPIX ? p * 256 + ((sl ^ hswz(y, x)) << 4) : HBYTES;
                *reinterpret_cast<i32x4*>(halo + dst) = hv[h];
            }
        }
        // ---- K loop: weights ring of 3 LDS slots (HALO_NT slices each), fragments one step ahead ----
        const int slice0 = cg * SPG;
        auto gload = [&](int st, i32x4* wv) {
#pragma unroll
            for (int u = 0; u < HALO_NT; ++u)
                wv[u] = *reinterpret_cast<const i32x4*>(wsrc + (size_t)(slice0 + st * HALO_NT + u) * wslice + tid * 16);
        };
        auto lstore = [&](int st, const i32x4* wv) {
#pragma unroll
            for (int u = 0; u < HALO_NT; ++u)
                *reinterpret_cast<i32x4*>(wbuf + (st % 3) * WSTEP + u * 8192 + woff) = wv[u];
        };
        auto frags = [&](int st, i32x4 (&fa)[HALO_NT][4], i32x4 (&fb)[HALO_NT][4]) {
            const char* wb = wbuf + (st % 3) * WSTEP;
#pragma unroll
            for (int u = 0; u < HALO_NT; ++u) {
                const int slice = st * HALO_NT + u;                   // wave-uniform (SALU)
                if constexpr (V1) {
                    const int tap = 4 * slice + fg;
                    const int tp = tap < NTAP ? tap : NTAP - 1;     // padded taps have zero weights
                    const int toff = ((tp / KS) * HW + tp % KS) * 16;
#pragma unroll
                    for (int i = 0; i < 4; ++i) fa[u][i] = *reinterpret_cast<const i32x4*>(halo + abase[i] + toff);
                } else {
                    const int cc = slice / NTAP, tap = slice % NTAP;   // slice = 32-channel chunk x tap
                    const int ky = tap / KS, kx = tap % KS;
                    // slot swizzle of this lane's pixels at this tap: identical for its 4 fragments
                    const int m = ((((xm + kx) & 3) << 1) | (((ym + ky) & 1) << 3)) ^ (cc * 4 + fg);
                    const int off = (ky * HW + kx) * 256 + (m << 4);
#pragma unroll
                    for (int i = 0; i < 4; ++i) fa[u][i] = *reinterpret_cast<const i32x4*>(halo + abase[i] + off);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) fb[u][j] = *reinterpret_cast<const i32x4*>(wb + u * 8192 + boff[j]);
            }
        };
        i32x4 wv[HALO_NT];
        gload(0, wv);
        lstore(0, wv);
        gload(min(1, steps_per_group - 1), wv);
        lstore(1, wv);
        __syncthreads();
        if constexpr (SCHED) {
            // Software pipeline, one barrier per step st (ring slot = step % 3):
            //   1. store the weights of step st+2 (global-loaded one step ago) into the slot step st-1
            //      used — its fragment reads completed before the previous barrier;
            //   2. issue the global weight loads of step st+3 (a whole step of latency budget);
            //   3. issue the fragment reads of step st+1 (slot written before the previous barrier);
            //   4. the 8*HALO_NT MFMAs of step st on fragments already in registers.
            // The DS store precedes the reads, so lgkmcnt (in order for LDS) never makes the barrier wait
            // on anything but reads that have had the whole MFMA block to land, and sched_barrier keeps
            // the compiler from sinking the reads below the MFMAs.  Branch-free: prefetch indices are
            // clamped; a store past the end lands in a slot nobody reads again in this group.
            i32x4 fa[HALO_NT][4], fb[HALO_NT][4], na[HALO_NT][4], nb[HALO_NT][4];
            frags(0, fa, fb);
            if constexpr ((ABL & 1) != 0) frags(0, na, nb);
            gload(min(2, steps_per_group - 1), wv);
            auto step = [&](int st, i32x4 (&ca)[HALO_NT][4], i32x4 (&cb)[HALO_NT][4], i32x4 (&xa)[HALO_NT][4],
                            i32x4 (&xb)[HALO_NT][4]) {
                if constexpr (!(ABL & 8)) {
                    lstore(st + 2, wv);
                    gload(min(st + 3, steps_per_group - 1), wv);
                }
                if constexpr (!(ABL & 1)) frags(min(st + 1, steps_per_group - 1), xa, xb);
                if constexpr (!(ABL & 16)) {
#pragma unroll
                for (int u = 0; u < HALO_NT; ++u)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8, ca[u][i]), __builtin_bit_cast(bf16x8, cb[u][j]), acc[i][j], 0, 0, 0);
                }
                // issue order: the LDS stores and weight loads, then one fragment read per MFMA pair, so
                // neither wave of a SIMD blocks in-order issue behind a full LDS queue while the matrix
                // pipe idles
                __builtin_amdgcn_sched_group_barrier(0x200, HALO_NT, 0);          // DS write
                __builtin_amdgcn_sched_group_barrier(0x020, HALO_NT, 0);          // VMEM read
#pragma unroll
                for (int k = 0; k < 8 * HALO_NT; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);            // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);            // DS read
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (!(ABL & 2)) __syncthreads();
            };
            for (int st = 0; st < steps_per_group; st += 2) {
                step(st, fa, fb, na, nb);
                if (st + 1 < steps_per_group) step(st + 1, na, nb, fa, fb);
            }
        } else {
        i32x4 fa[HALO_NT][4], fb[HALO_NT][4];
        frags(0, fa, fb);
        for (int st = 0; st < steps_per_group; ++st) {
            if (st + 2 < steps_per_group) gload(st + 2, wv);
            i32x4 na[HALO_NT][4], nb[HALO_NT][4];
            if (st + 1 < steps_per_group) frags(st + 1, na, nb);   // slot written before the previous barrier
#pragma unroll
            for (int u = 0; u < HALO_NT; ++u)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[u][i]),
                                                                           __builtin_bit_cast(bf16x8, fb[u][j]), acc[i][j], 0, 0, 0);
            if (st + 2 < steps_per_group) lstore(st + 2, wv);     // slot last read two steps ago
            __syncthreads();
#pragma unroll
            for (int u = 0; u < HALO_NT; ++u)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    fa[u][i] = na[u][i];
                    fb[u][i] = nb[u][i];
                }
        }
        }
    }

    // ---- epilogue: folded BN scale/shift -> 2x2 max pool (in-lane quad) -> LeakyReLU -> store ----
    bf16_t* out = reinterpret_cast<bf16_t*>(a.out);
    const int Wp = a.Wc / 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int co = co0 + wn * 64 + 16 * j + fr;
        const float sc = a.scale[co], sh = a.shift[co];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int F = wm * 4 + i;
            const int cl = F / BPC, b = F % BPC;
            const int clip = clip0 + cl;
            if (clip >= a.N) continue;
            const int q = fg;   // this lane's rows 4q..4q+3 = pool window q of the fragment
            const int py = (oy0 + 4 * (b / BPR)) / 2 + (q >> 1);
            const int px = (ox0 + 4 * (b % BPR)) / 2 + (q & 1);
            float v0 = acc[i][j][0] * sc + sh, v1 = acc[i][j][1] * sc + sh;
            float v2 = acc[i][j][2] * sc + sh, v3 = acc[i][j][3] * sc + sh;
            float x = fmaxf(fmaxf(v0, v1), fmaxf(v2, v3));
            x = x >= 0.f ? x : LRELU * x;
            out[(size_t)clip * a.out_clip_stride + (size_t)(py * Wp + px) * a.out_pix_stride + a.out_c_off + co] = (bf16_t)x;
        }
    }
}

template <int KS, int TH, int TW, int NCLIP, bool V1, bool SCHED>
int launch_halo_t(const HaloArgs& a, hipStream_t s) {
    constexpr int HH = TH + KS - 1, HW = TW + KS - 1;
    constexpr int HPIX = NCLIP * HH * HW;
    constexpr int PIXB = V1 ? 16 : 256;
    constexpr int HBYTES = ((HPIX * PIXB + 255) / 256) * 256;
    const size_t shm = HBYTES + 256 + 3 * HALO_NT * 8192;
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_halo<KS, TH, TW, NCLIP, V1, SCHED>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        attr = true;
    }
    if (a.Hc % TH || a.Wc % TW || a.Co % 128) { set_error("halo conv: tile does not divide the layer"); return 3; }
    const int tiles = ((a.N + NCLIP - 1) / NCLIP) * (a.Hc / TH) * (a.Wc / TW);
    hipLaunchKernelGGL((k_conv_halo<KS, TH, TW, NCLIP, V1, SCHED>), dim3(tiles, a.Co / 128), dim3(512), shm, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

int launch_conv_halo(const HaloArgs& a, hipStream_t s) {
    // AVSE_HALO_MODE = stream (default: persistent LDS-DMA kernel, conv_stream.hip)
    //                | pipe (8-wave halo kernel, explicit pipeline) | tile (8-wave, compiler schedule)
    static const int mode = [] {
        const char* e = std::getenv("AVSE_HALO_MODE");
        if (e && e[0] == 't') return 0;
        if (e && e[0] == 'p') return 1;
        return 2;
    }();
    const bool pipe = mode == 1;
    if (mode == 2 && a.variant != HALO_V1) return launch_conv_stream(a, s);
    switch (a.variant) {
        case HALO_V1: {
            // AVSE_V1_IM2COL=1 (read per launch): the dense-im2col kernel (A/B switch)
            const char* e = std::getenv("AVSE_V1_IM2COL");
            if ((e && e[0] == '1') || !a.w2) return launch_conv_v1(a, s);
            HaloArgs r = a;
            r.w = a.w2;
            return launch_conv_v1r(r, s);
        }
        case HALO_K5:
            return pipe ? launch_halo_t<5, 16, 16, 1, false, true>(a, s) : launch_halo_t<5, 16, 16, 1, false, false>(a, s);
        case HALO_K3_16:
            return pipe ? launch_halo_t<3, 16, 16, 1, false, true>(a, s) : launch_halo_t<3, 16, 16, 1, false, false>(a, s);
        case HALO_K3_8:
            return pipe ? launch_halo_t<3, 8, 8, 4, false, true>(a, s) : launch_halo_t<3, 8, 8, 4, false, false>(a, s);
    }
    set_error("bad halo variant");
    return 3;
}

}  // namespace avse
