// Fused decoder tail on split-f16 operands (AVSE_F32_SPLIT, gfx950), one workgroup per HALF clip:
//   d_deconv4  Conv2DTranspose(64, 4x4, stride 1, 'same') + BatchNorm + LeakyReLU(0.3)   network.py:125-127
//   d_deconv5  Conv2DTranspose(64, 5x5, stride 2, 'same') + BatchNorm + LeakyReLU(0.3)   network.py:129-131
//   d_deconv6  Conv2DTranspose(1, 1x1) -> the [80, 20] enhanced spectrogram            network.py:133
//
// Why: layer by layer (k_conv_win for d_deconv4, k_conv's four phases + the fused d_deconv6 dot for d_deconv5) the two
// layers took 0.235 + 0.211 ms per 512 clips, ~210 TF for 3-4 f16 products per fp32 MAC, latency-bound (PMC: waves
// waiting 40-46 %, MFMA busy 35-44 %): per-tile prologues / epilogues, a barrier per 64-byte slab, and d_deconv4's
// output written to HBM and gathered back per tap.  The bf16 path fuses them per clip (conv_dec.hip), but a clip's
// d_deconv4 output as f16 pairs (40 x 10 x 64 x 4 B, padded: 188 KB) does not fit the 160-KB LDS.  Here a workgroup
// owns the d_deconv5 output rows of half a clip (h = 0: rows 0..39, h = 1: rows 40..79 of 80), which read d_deconv4
// rows 20 h - 1 .. 20 h + 20: it computes the 21 of those inside the image (one row beyond its half: 5 % more
// d_deconv4 work) into an LDS image and runs d_deconv5 + d_deconv6 from there.
//   * d_deconv4's input (d_deconv3's split pairs, [40][10][8 chunks of 16 channels x (h | l)]) streams through two LDS
//     windows, one per 16-channel chunk (24 x 14 pixels of 64 B at a 96-B row pitch), the next chunk's window loaded
//     during the current chunk's 16 taps; weights through an LDS ring of 4-slab groups (64 rows x [Wh(16) | Wl(16)]),
//     every lane moving 8 B of the slab 8 ahead per slab; one barrier per group;
//   * M fragments are 16 consecutive pixels of the row-major 10-wide grid (d_deconv4: 14 fragments for 210 pixels,
//     d_deconv5: 13 per phase for 200): fewer padding slots than 8 x 2 blocks (15 each), and a pixel pitch of 18 makes
//     every tap's ds_read_b128 lane groups bank-conflict free (exhaustive check over fragments, taps and chunks);
//   * 8 waves, two per SIMD: wave w owns output-channel block w & 3 (16 channels) and fragments 7 (w >> 2) .. + 6;
//     per slab it reads 7 pixel fragments + the Wh / Wl fragments of its block (9 ds_read_b128) for 14
//     v_mfma_f32_16x16x32_f16: D = W x A, [Wh | Wh] x [Ah | Al] and [Wl | Wl] x [Ah | Al] (all four products, as k_conv)
//     summed per 8 slabs into a zeroed partial that joins the running sum (k_conv's blocked fp32 summation);
//   * d_deconv4's epilogue (BN + LeakyReLU with the layer's activation exponent folded, the range guard, the pair
//     split) stores 8 B of h and 8 B of l per lane and fragment into the zero-bordered image over the dead windows;
//   * d_deconv5 walks its four stride phases (4 / 6 / 6 / 9 taps x 4 chunks; every phase a whole number of ring groups)
//     with immediate tap offsets; each phase's epilogue folds BN, LeakyReLU and d_deconv6's 64 -> 1 dot: 4 channels
//     in-lane, the lane rows by two xor shuffles, the four channel blocks (waves) through LDS in a fixed order.
#include <cstdlib>
#include <utility>

#include "avse_common.h"

namespace avse {
namespace {

// timing ablations (tools/_ab variant libraries only; 0 in the library): 1 = no MFMAs (fragment reads kept alive),
// 2 = no fragment reads in the loops (MFMAs on the prologue's fragments), 4 = no barriers in the loops.  Measured
// (profiles/r06c_split_tail_ablate.txt, B = 512): full 0.335 ms, 1: 0.188, 2: 0.306, 4: 0.326.  Also measured and
// not kept: the stream kernels' three-product slab pairs (Wl Al dropped, A' by v_permlane32_swap): 0.343 vs 0.335 ms
// (the tail is not MFMA-issue-bound: 14 MFMAs per slab per wave, ~54 % MFMA busy)
#ifndef AVSE_DECTS_ABL
#define AVSE_DECTS_ABL 0
#endif
constexpr int DABL = AVSE_DECTS_ABL;
constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;
constexpr int H = 40, W = 10;                        // d_deconv4 / d_deconv5 grid of a clip
constexpr int CI4 = 128, CO = 64;                    // d_deconv4 128 -> 64, d_deconv5 64 -> 64 (real channels)
constexpr int NW = 8, NT = 64 * NW;
constexpr int R4 = 21;                               // d_deconv4 rows a half computes
constexpr int F4 = 14, F5 = 13, SL = 7;              // fragments (d4, d5 per phase), slots per wave
// d_deconv4 window: local output row r reads window row r + dy + 2 (dy in -2..1); 24 rows x 14 columns loaded, rows up
// to 25 read by the padding slots (q >= 210: their results are dropped)
constexpr int P4 = 18, S4 = 96, ROWS4 = 26, WBUF = ROWS4 * P4 * S4;   // 44,928 B per buffer
constexpr int LROWS4 = 24, LCOLS4 = 14, NPC = 3;                     // 24 x 14 x 4 pieces <= 3 x 512
// d_deconv5 image: image row i <-> d_deconv4 row 20 h - 1 + i (i = 0..21; 22 only read by padding slots), column
// x + 1; 64 channels = 4 chunks of [h(16) | l(16)] per pixel (256 B at a 288-B pitch)
constexpr int P5 = 18, S5 = 288, ROWS5 = 23, OIMG = ROWS5 * P5 * S5;   // 119,232 B over the windows
constexpr int REGION = ((OIMG > 2 * WBUF ? OIMG : 2 * WBUF) + 1023) / 1024 * 1024;
constexpr int BOFF = REGION;                                           // weight ring: 2 groups x 4 slabs x 4 KB
constexpr int PAR = BOFF + 2 * 4 * 4096;
constexpr int PSC4 = PAR, PSH4 = PAR + 256, PSC5 = PAR + 512, PSH5 = PAR + 768, PW6 = PAR + 1024;
constexpr int XP = PAR + 1280;                                         // d_deconv6 partials [4 blocks][208] f32
constexpr int LDS_BYTES = XP + 4 * 16 * F5 * 4;                        // 157,184
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
static_assert(2 * SL == F4 && 16 * F4 >= R4 * W && 16 * F5 >= H / 2 * W && 16 * (F5 - 1) < H / 2 * W, "fragments");

constexpr int ph_ny(int p) { return 2 + (p >> 1); }
constexpr int ph_nx(int p) { return 2 + (p & 1); }
constexpr int ph_nt(int p) { return ph_ny(p) * ph_nx(p); }
constexpr int ph_woff(int p) { int s = 0; for (int q = 0; q < p; ++q) s += CO * ph_nt(q) * CO; return s; }   // real elems
constexpr int ph_gstart(int p) { int s = 0; for (int q = 0; q < p; ++q) s += 4 * ph_nt(q); return s; }      // slabs
constexpr int ph_of(int g) { int p = 0; while (p < 3 && g >= ph_gstart(p + 1)) ++p; return p; }
static_assert(ph_gstart(4) % 4 == 0 && (4 * ph_nt(0)) % 4 == 0, "every phase is whole ring groups");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ int wsw(int row) { return 2 * ((row >> 2) & 1); }   // weight-slab slot swizzle (k_conv's)
__device__ __forceinline__ i32x4 lds16(const char* base, int off) { return *reinterpret_cast<const i32x4*>(base + off); }
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bn_lrelu(float acc, float sc, float sh) {
    const float v = fmaf(acc, sc, sh);
    return fmaxf(v, LRELU * v);
}
// LDS stores of this wave drained, then the workgroup barrier (global loads stay in flight across it)
__device__ __forceinline__ void lds_barrier_raw() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
}
__device__ __forceinline__ void lds_barrier() { lds_barrier_raw(); }
__device__ __forceinline__ void loop_barrier() {
    if constexpr (!(DABL & 4)) lds_barrier_raw();
}
template <int... I, typename F>
__device__ __forceinline__ void unroll(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

__global__ __launch_bounds__(NT, 1) void k_dec_tail_s16(DecTailArgs a) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int clip = blockIdx.x >> 1, half = blockIdx.x & 1;
    const int cb = w & 3, fr0 = SL * (w >> 2);     // channel block, first fragment
    const bool s6 = w < 4;                        // slot 6 is a d_deconv5 fragment (12 < 13) for waves 0..3 only

    // weight slabs through the LDS ring: lane tid moves 8 B (half kh of 16-B group kq) of row tid >> 3
    const int brow = tid >> 3, kq = (tid >> 1) & 3, kh = tid & 1;
    const int bst = BOFF + brow * 64 + ((kq ^ wsw(brow)) << 4) + kh * 8;           // + slot * 16384 + pos * 4096
    // this wave's Wh / Wl fragments: row 16 cb + r16, 16-B group (kg & 1) / 2 + (kg & 1)
    const int brd = 16 * cb + r16;
    const int bfh = BOFF + brd * 64 + (((kg & 1) ^ wsw(brd)) << 4);
    const int bfl = BOFF + brd * 64 + (((2 + (kg & 1)) ^ wsw(brd)) << 4);
    auto st8 = [&](int addr, i32x2 v) { *reinterpret_cast<i32x2*>(lds + addr) = v; };
    auto read_w = [&](int off, i32x4 (&f)[2]) {
        f[0] = lds16(lds, bfh + off);
        f[1] = lds16(lds, bfl + off);
    };

    f32x4 acc[SL], part[SL];
    auto zero_all = [&]() {
#pragma unroll
        for (int i = 0; i < SL; ++i) acc[i] = part[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    };
    auto flush = [&]() {   // blocked fp32 summation (k_conv FP32_BLOCK = 8 slabs)
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            acc[i] += part[i];
            part[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    // D = W x A: a lane holds channels 16 cb + 4 kg .. + 3 of pixel r16 of each fragment
    auto mfma_all = [&](const i32x4 (&fa)[SL], const i32x4 (&fw)[2], bool slot6) {
        if constexpr (DABL & 1) {
#pragma unroll
            for (int i = 0; i < SL; ++i) asm volatile("" ::"v"(fa[i]));
            asm volatile("" ::"v"(fw[0]), "v"(fw[1]));
            return;
        }
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            if (i == SL - 1 && !slot6) continue;
            part[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fw[0]), __builtin_bit_cast(f16x8, fa[i]),
                                                             part[i], 0, 0, 0);
            part[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fw[1]), __builtin_bit_cast(f16x8, fa[i]),
                                                             part[i], 0, 0, 0);
        }
    };

    if (tid < 64) {   // epilogue parameters (read as broadcast quads in the epilogues)
        reinterpret_cast<float*>(lds + PSC4)[tid] = a.sc4[tid];
        reinterpret_cast<float*>(lds + PSH4)[tid] = a.sh4[tid];
        reinterpret_cast<float*>(lds + PSC5)[tid] = a.sc5[tid];
        reinterpret_cast<float*>(lds + PSH5)[tid] = a.sh5[tid];
        reinterpret_cast<float*>(lds + PW6)[tid] = a.w6[tid];
    }
    auto par4 = [&](int base) { return *reinterpret_cast<const f32x4*>(lds + base + (16 * cb + 4 * kg) * 4); };

    // =============================== d_deconv4 ===============================
    const int r0 = 19 * half;                        // first d_deconv4 row of this half
    bool range_bad = false;
    {
        // window piece k of lane tid: 16 B (sg = tid & 3) of window pixel p = tid / 4 + 128 k (24 rows x 14 columns);
        // window pixel (wr, wc) = input pixel (r0 - 2 + wr, wc - 2), zero outside the image
        const long long in_clip = (long long)H * W * CI4 * 4;   // bytes of a clip's pairs
        const __amdgpu_buffer_rsrc_t rsIn = make_rsrc(reinterpret_cast<const char*>(a.in) + clip * in_clip, in_clip);
        int psrc[NPC], pdst[NPC];
        bool pok[NPC];
#pragma unroll
        for (int k = 0; k < NPC; ++k) {
            const int p = (tid >> 2) + (NT / 4) * k, sg = tid & 3;
            const int wr = p / LCOLS4, wc = p - wr * LCOLS4;
            const int iy = r0 - 2 + wr, ix = wc - 2;
            pok[k] = p < LROWS4 * LCOLS4;
            const bool in = pok[k] && iy >= 0 && iy < H && ix >= 0 && ix < W;
            psrc[k] = in ? ((iy * W + ix) * CI4 * 2 + sg * 8) * 2 : kOOB;
            pdst[k] = (wr * P4 + wc) * S4 + sg * 16;
        }
        // weights: row n = [8192 B]: slab (tap t, chunk c) at byte 512 t + 64 c
        const __amdgpu_buffer_rsrc_t rsW = make_rsrc(a.w4, (long long)CO * 16 * CI4 * 4);
        const int vbl = brow * (16 * CI4 * 4) + kq * 16 + kh * 8;
        auto bpiece = [&](auto tt, int csoff) {
            constexpr int t = decltype(tt)::value;
            return __builtin_amdgcn_raw_buffer_load_b64(rsW, vbl + t * 512, csoff, 0);
        };
        // fragment bases: slot i = fragment fr0 + i, pixel q = 16 f + r16 -> (q / 10, q % 10), tap (-2, -2)
        int vb[SL];
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int q = 16 * (fr0 + i) + r16, r = q / W, x = q - r * W;
            vb[i] = (r * P4 + x) * S4 + kg * 16;
        }
        // prologue: window chunk 0 -> buffer 0; weight slabs 0..3 -> ring slot 0, 4..7 in registers
        {
            i32x4 pc[NPC];
#pragma unroll
            for (int k = 0; k < NPC; ++k) pc[k] = __builtin_amdgcn_raw_buffer_load_b128(rsIn, psrc[k], 0, 0);
#pragma unroll
            for (int k = 0; k < NPC; ++k)
                if (pok[k]) *reinterpret_cast<i32x4*>(lds + pdst[k]) = pc[k];
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
        zero_all();
        lds_barrier();

        i32x4 fa[2][SL], fw[2][2];
        // next chunk's window pieces: loaded at tap k < NPC, stored at tap k + 12, before the chunk's last barrier
        // (stored 3 taps after the load: 0.335 vs 0.333 ms, not their latency)
        constexpr int PST = 12;
        i32x4 pr[NPC];
        int wb = 0;      // byte offset of the window buffer being read
        auto read_a = [&](auto tt, i32x4 (&f)[SL]) {
            constexpr int t = decltype(tt)::value % 16;
            constexpr int imm = ((3 - t / 4) * P4 + (3 - t % 4)) * S4;   // tap (1 - t/4, 1 - t%4) from (-2, -2)
#pragma unroll
            for (int i = 0; i < SL; ++i) f[i] = lds16(lds + imm + wb, vb[i]);
        };
        read_a(std::integral_constant<int, 0>{}, fa[0]);
        read_w(0, fw[0]);
        // slab S = 16 c + t; group S / 4 in ring slot (S / 4) & 1; barrier every 4 slabs (t % 4 == 3)
        for (int c = 0; c < 8; ++c) {
            const int nb = (c & 1) ? 0 : WBUF;           // next chunk -> the other buffer
            const int cs = c * 64, cn = (c + 1) * 64;    // this / next chunk's byte offset in a pixel / weight tap
            unroll(std::make_integer_sequence<int, 16>{}, [&](auto tt) {
                constexpr int t = decltype(tt)::value;
                __builtin_amdgcn_sched_barrier(0);
                // weights of slab S + 4 (loaded 4 slabs ago) -> group slot (S / 4 + 1) & 1; slab S + 8 -> registers
                st8(bst + (((t / 4) + 1) & 1) * 16384 + (t % 4) * 4096, pb[t & 3]);
                if constexpr (t + 8 < 16) pb[t & 3] = bpiece(std::integral_constant<int, t + 8>{}, cs);
                else pb[t & 3] = bpiece(std::integral_constant<int, t + 8 - 16>{}, cn);   // past the layer: unused
                // window piece t of chunk c + 1 (after the last chunk: a harmless re-read, never stored)
                if constexpr (t < NPC) pr[t] = __builtin_amdgcn_raw_buffer_load_b128(rsIn, psrc[t], cn, 0);
                if constexpr (t >= PST && t - PST < NPC) {
                    if (pok[t - PST] && c < 7) *reinterpret_cast<i32x4*>(lds + nb + pdst[t - PST]) = pr[t - PST];
                }
                if constexpr (t % 4 == 3) loop_barrier();
                if constexpr (t == 15) wb = nb;
                // the next slab's fragments go out before this slab's MFMAs
                if constexpr (DABL & 2) {
                } else if constexpr (t < 15) {
                    read_a(std::integral_constant<int, t + 1>{}, fa[(t + 1) & 1]);
                } else if (c < 7) {
                    read_a(std::integral_constant<int, 0>{}, fa[0]);
                }
                if constexpr (!(DABL & 2)) read_w((((t + 1) / 4) & 1) * 16384 + ((t + 1) % 4) * 4096, fw[(t + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
                mfma_all(fa[t & 1], fw[t & 1], true);
                if constexpr (t % 8 == 7) flush();
            });
        }
        lds_barrier();   // every window read done: the d_deconv5 image goes over the windows

        // image border: the zero row (h = 0: image row 0 = d_deconv4 row -1; h = 1: row 21 = row 40) and columns 0, 11
        // of rows 0..21 (256 data bytes per pixel = 16 pieces)
        {
            const int zrow = half ? 21 : 0;
            for (int u = tid; u < (12 + 2 * 22) * 16; u += NT) {
                const int px = u >> 4, pc = u & 15;
                const int i = px < 12 ? zrow : (px - 12) >> 1, xi = px < 12 ? px : ((px - 12) & 1) * 11;
                *reinterpret_cast<i32x4*>(lds + (i * P5 + xi) * S5 + pc * 16) = (i32x4){0, 0, 0, 0};
            }
        }
        // epilogue: BN + LeakyReLU (the layer's activation exponent folded into sc4 / sh4) -> pairs at image pixel
        // (r + 1 - h, x + 1), channels 16 cb + 4 kg + e: 8 B of h pieces, 8 B of l pieces
        const f32x4 sc = par4(PSC4), sh = par4(PSH4);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int q = 16 * (fr0 + i) + r16;
            if (q >= R4 * W) continue;
            const int r = q / W, x = q - r * W;
            const int px = ((r + 1 - half) * P5 + x + 1) * S5 + cb * 64 + 8 * kg;
            f16x4 hv, lv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float y = bn_lrelu(acc[i][e], sc[e], sh[e]);
                range_bad |= pair_out_of_range(y);
                hv[e] = (_Float16)y;
                lv[e] = (_Float16)(y - (float)hv[e]);
            }
            *reinterpret_cast<f16x4*>(lds + px) = hv;
            *reinterpret_cast<f16x4*>(lds + px + 32) = lv;
        }
        lds_barrier();
    }
    range_report(a.range_flag, a.range_bit, range_bad);

    // =============================== d_deconv5 + d_deconv6 ===============================
    float* const outc = a.out + (long long)clip * (4 * H * W);
    const __amdgpu_buffer_rsrc_t rsW5 = make_rsrc(a.w5, (long long)ph_woff(4) * 4);
    int vrow5[3];   // this lane's ring piece in a weight row of kpad 4, 6, 9 taps x 64 (bytes per row 4 kpad)
    vrow5[0] = brow * (4 * CO * 4) + kq * 16 + kh * 8;
    vrow5[1] = brow * (6 * CO * 4) + kq * 16 + kh * 8;
    vrow5[2] = brow * (9 * CO * 4) + kq * 16 + kh * 8;
    auto bpiece5 = [&](auto gg) {   // ring piece of global slab g (past the end: phase 3's slab 0, unused)
        constexpr int g = decltype(gg)::value < ph_gstart(4) ? decltype(gg)::value : ph_gstart(3);
        constexpr int p = ph_of(g), sl = g - ph_gstart(p);
        constexpr int kk = p == 0 ? 0 : p == 3 ? 2 : 1;   // phase 0: 4 taps, 1 / 2: 6, 3: 9
        return __builtin_amdgcn_raw_buffer_load_b64(rsW5, vrow5[kk], ph_woff(p) * 4 + sl * 64, 0);
    };
    int vb5[SL];
#pragma unroll
    for (int i = 0; i < SL; ++i) {
        const int q = 16 * (fr0 + i) + r16, yl = q / W, x = q - yl * W;
        vb5[i] = (yl * P5 + x) * S5 + kg * 16;   // tap (-1, -1)
    }
    auto read_a5 = [&](auto gg, i32x4 (&f)[SL]) {
        constexpr int g = decltype(gg)::value;
        constexpr int p = ph_of(g), sl = g - ph_gstart(p), tap = sl / 4, c = sl % 4;
        constexpr int dy = (p >> 1) - tap / ph_nx(p), dx = (p & 1) - tap % ph_nx(p);
        constexpr int imm = ((dy + 1) * P5 + (dx + 1)) * S5 + c * 64;
#pragma unroll
        for (int i = 0; i < SL - 1; ++i) f[i] = lds16(lds + imm, vb5[i]);
        if (s6) f[SL - 1] = lds16(lds + imm, vb5[SL - 1]);
    };
    float* const xp = reinterpret_cast<float*>(lds + XP);
    auto epilogue5 = [&](auto pp) {
        constexpr int p = decltype(pp)::value, py = p >> 1, px = p & 1;
        flush();
        const f32x4 sc = par4(PSC5), sh = par4(PSH5), w6 = par4(PW6);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            if (i == SL - 1 && !s6) continue;
            float d = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) d = fmaf(bn_lrelu(acc[i][e], sc[e], sh[e]), w6[e], d);
            d += __shfl_xor(d, 16);
            d += __shfl_xor(d, 32);
            const int q = 16 * (fr0 + i) + r16;
            if (kg == 0 && q < H / 2 * W) xp[cb * (16 * F5) + q] = d;   // this block's 16-channel share
        }
        lds_barrier();
        if (tid < H / 2 * W) {   // the four channel blocks in a fixed order, + bias
            const int q = tid, yl = q / W, x = q - yl * W;
            const float v = ((xp[q] + xp[16 * F5 + q]) + xp[32 * F5 + q]) + xp[48 * F5 + q];
            outc[(2 * (H / 2 * half + yl) + py) * (2 * W) + 2 * x + px] = v + a.b6;
        }
        zero_all();
    };

    // weight slabs 0..3 -> slot 0, 4..7 in flight (every d_deconv4 read of the ring finished before the barriers above)
    i32x2 pb[4];
    {
        i32x2 w0[4];
        unroll(std::make_integer_sequence<int, 4>{}, [&](auto tt) {
            constexpr int t = decltype(tt)::value;
            w0[t] = bpiece5(tt);
            pb[t] = bpiece5(std::integral_constant<int, t + 4>{});
        });
#pragma unroll
        for (int t = 0; t < 4; ++t) st8(bst + t * 4096, w0[t]);
    }
    zero_all();
    lds_barrier();
    i32x4 fa[2][SL], fw[2][2];
    read_a5(std::integral_constant<int, 0>{}, fa[0]);
    read_w(0, fw[0]);
    // global slab g: store g + 4 -> slot ((g / 4) + 1) & 1, load g + 8, barrier every 4 slabs; the fragments of g + 1
    // go out before g's MFMAs (a phase's last slab: after its epilogue, whose barrier also orders the xp buffer)
    unroll(std::make_integer_sequence<int, ph_gstart(4)>{}, [&](auto gg) {
        constexpr int g = decltype(gg)::value, p = ph_of(g);
        constexpr bool last = g + 1 == ph_gstart(p + 1);
        __builtin_amdgcn_sched_barrier(0);
        st8(bst + (((g / 4) + 1) & 1) * 16384 + (g % 4) * 4096, pb[g & 3]);
        pb[g & 3] = bpiece5(std::integral_constant<int, g + 8>{});
        if constexpr (g % 4 == 3) loop_barrier();
        if constexpr (!last && !(DABL & 2)) {
            read_a5(std::integral_constant<int, g + 1>{}, fa[(g + 1) & 1]);
            read_w((((g + 1) / 4) & 1) * 16384 + ((g + 1) % 4) * 4096, fw[(g + 1) & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_all(fa[g & 1], fw[g & 1], s6);
        if constexpr (!last && (g - ph_gstart(p)) % 8 == 7) flush();
        if constexpr (last) {
            epilogue5(std::integral_constant<int, p>{});
            if constexpr (p < 3) {
                read_a5(std::integral_constant<int, g + 1>{}, fa[(g + 1) & 1]);
                read_w((((g + 1) / 4) & 1) * 16384 + ((g + 1) % 4) * 4096, fw[(g + 1) & 1]);
            }
        }
    });
}

}  // namespace

bool dec_tail_s16_supported(const DecTailArgs& a) {
    // the compile-time geometry above (network.py's layers at the 200-ms segment; the tap grids checked as for the bf16
    // tail: dec_tail_supported)
    if (a.N <= 0 || a.nt4 != 16 || a.kpad4 != 16 * CI4 || a.dy4 != 1 || a.dx4 != 1 || a.nx4 != 4) return false;
    if (a.pt4 != 2 || a.pl4 != 2 || a.pt5 != 1 || a.pl5 != 1) return false;
    for (int p = 0; p < 4; ++p)
        if (a.nt5[p] != ph_nt(p) || a.kpad5[p] != ph_nt(p) * CO || a.dy5[p] != (p >> 1) || a.dx5[p] != (p & 1) ||
            a.nx5[p] != ph_nx(p) || a.woff5[p] != ph_woff(p))
            return false;
    return true;
}

int launch_dec_tail_s16(const DecTailArgs& a, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_dec_tail_s16, LDS_BYTES)) return rc;
    hipLaunchKernelGGL(k_dec_tail_s16, dim3(2 * a.N), dim3(NT), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
