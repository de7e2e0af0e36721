// Fused decoder tail, one workgroup per clip (bf16, gfx950):
//   d_deconv4  Conv2DTranspose(64, 4x4, stride 1, 'same') + BatchNorm + LeakyReLU(0.3)   network.py:125-127
//   d_deconv5  Conv2DTranspose(64, 5x5, stride 2, 'same') + BatchNorm + LeakyReLU(0.3)   network.py:129-131
//   d_deconv6  Conv2DTranspose(1, 1x1) -> the [80, 20] enhanced spectrogram            network.py:133
//
// Why: run layer by layer (k_conv, conv.hip) these two layers cost ~0.21 ms per 512 clips at ~450 TFLOP/s:
// every 64-byte K slab of a 128-pixel tile paid a workgroup barrier plus per-slab im2col staging, and each
// tile exposed its prologue / epilogue latency (ablations of the window-staged variant).  Here a
// clip's whole working set stays in LDS:
//   * d_deconv4's input (d_deconv3's [40][10][128] output) streams through two LDS window buffers, one per
//     32-channel chunk, zero-padded to 43 x 14 pixels; the next chunk's window is loaded during the current
//     chunk's 16 taps;
//   * weights go through an LDS ring of 4-slab groups (2 x 4 x 4 KB): every lane moves 8 B of the slab 8
//     ahead per slab (registers) and stores the slab 4 ahead; one barrier per group publishes the next group
//     (and, every 16 slabs, the next window).  Loading each wave's B fragments straight from L2 cost 4x the
//     VMEM instructions and registers the compiler could not hold a ring in;
//   * 8 waves, two per SIMD; wave w owns the 16-pixel M fragments w, w + 8, w + 16, w + 24 (32 slots for the
//     25 fragments of the 40 x 10 grid; slots past the grid are computed and dropped) x all 64 output
//     channels: per 32-deep K slab 4 A + 4 B fragments (ds_read_b128, read one slab ahead), 16
//     v_mfma_f32_16x16x32_bf16.  With one wave per SIMD (7 slots each) the same loop ran at ~38 cycles per
//     MFMA (s_memtime) against ~18 in a micro-benchmark of the bare step (tools/mfma_micro.hip): nothing
//     covered a wave's LDS and barrier waits (0.149 -> 0.132 ms);
//   * the geometry is compile-time (the host checks the layer shapes and tap grids): a d_deconv4 fragment
//     read is one ds_read_b128 at a per-lane base + an immediate; d_deconv5 adds one scalar tap offset per
//     slab.  The first version computed runtime tap offsets with an XOR swizzle per fragment (~5 VALU per
//     fragment per slab) in the 8 free issue cycles a 16x16x32 MFMA leaves;
//   * M fragments are 8 x 2 pixel blocks and pixel rows are padded (d_deconv4 window 96-B rows of 64 B,
//     d_deconv5 image 160-B rows of 128 B, pitch 14): bank-conflict free for every tap without a swizzle
//     (checked exhaustively over fragments, taps and the four ds_read_b128 lane groups);
//   * the d_deconv4 result (BN, LeakyReLU, rounded to bf16 exactly like the layer-by-layer path) is written
//     into a zero-padded 42 x 14 image over the dead windows, which d_deconv5 reads for its four stride
//     phases (sub-pixel decomposition as in k_conv: only the taps that hit a phase);
//   * the MFMAs compute D = W x A (channels x pixels), so a lane's 4 accumulator rows are 4 consecutive channels of
//     one pixel: d_deconv4's epilogue stores 8 B per lane and fragment (it was 4 x 4 two-byte LDS stores);
//   * d_deconv5's epilogue folds BN, LeakyReLU, the bf16 rounding of its output and d_deconv6's 64 -> 1
//     dot + bias: 16 channels in-lane, then the four lane rows by three permlane swaps for four fragment slots;
//     one float per output pixel is stored.
#include <cstdlib>
#include <utility>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;
constexpr int H = 40, W = 10, HW = H * W;           // d_deconv4 / d_deconv5 phase grid
constexpr int CI4 = 128, CO = 64;                    // d_deconv4 128 -> 64, d_deconv5 64 -> 64
constexpr int NW = 8, NT = 64 * NW;                  // waves (two per SIMD), threads
// fragment slots per wave: slots 0..2 = fragments w, w + 8, w + 16 x all 64 channels; slot 3 = fragment 24 x channels
// 16 w .. 16 w + 15 on waves 0..3 only (25 fragments x 4 channel blocks = 100 pairs: 13 / 12 per wave, 25 per SIMD,
// where 8 waves x 4 full slots computed 128 pairs and dropped 28)
constexpr int NF = 4, FX = 24;
constexpr int PXB = 1280;                            // d_deconv6 partials of fragment 24 (4 waves x 16 pixels, f32)
// d_deconv4: taps t -> (dy, dx) = (1 - t / 4, 1 - t % 4); window pixel (y + dy + 2, x + dx + 2)
constexpr int P4 = 14, ROWS4 = 43, S4 = 96, NPIX4 = ROWS4 * P4;   // 602 pixels, 96-B rows
constexpr int NPC = 5;                                            // 16-B pieces per lane per chunk (5 x 512 >= 602 x 4)
constexpr int WBUF = NPIX4 * S4;                                  // 57,792
// d_deconv5 phase p = 2 py + px: taps (py - a, px - b), a < 2 + py, b < 2 + px; image pixel (y + dy + 1, x + dx + 1)
constexpr int P5 = 14, ROWS5 = 42, S5 = 160, OIMG = ROWS5 * P5 * S5;   // 94,080 B over the windows
constexpr int BOFF = 2 * WBUF;                                        // weight slab ring: 2 groups x 4 slabs x 4 KB
constexpr int PAR = BOFF + 2 * 4 * 4096;                              // folded BN / d_deconv6 parameters (f32):
constexpr int PSC4 = PAR, PSH4 = PAR + 256, PSC5 = PAR + 512, PSH5 = PAR + 768, PW6 = PAR + 1024;   // 64 each
constexpr int LDS_BYTES = PAR + PXB + 256;                            // 149,888
static_assert(OIMG <= BOFF, "d_deconv5 image must fit over the d_deconv4 windows");

constexpr int ph_ny(int p) { return 2 + (p >> 1); }
constexpr int ph_nx(int p) { return 2 + (p & 1); }
constexpr int ph_nt(int p) { return ph_ny(p) * ph_nx(p); }
constexpr int ph_woff(int p) { int s = 0; for (int q = 0; q < p; ++q) s += CO * ph_nt(q) * CO; return s; }  // elements
constexpr int ph_pstart(int p) { int s = 0; for (int q = 0; q < p; ++q) s += (2 * ph_nt(q) + 3) / 4 * 4; return s; }  // padded
constexpr int ph_ofp(int g) { int p = 0; while (p < 3 && g >= ph_pstart(p + 1)) ++p; return p; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ int wsw(int row) { return 2 * ((row >> 2) & 1); }   // weight-slab slot swizzle
__device__ __forceinline__ i32x4 lds16(const char* base, int off) { return *reinterpret_cast<const i32x4*>(base + off); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bn_lrelu(float acc, float sc, float sh) {
    const float v = fmaf(acc, sc, sh);
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(LRELU * v));   // LeakyReLU, no canonicalise
    return r;
}
__device__ __forceinline__ auto pack4(float a, float b, float c, float d) {   // 4 bf16 (RNE, as (bf16_t) casts)
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    const bf16x2 lo = __builtin_convertvector((f32x2){a, b}, bf16x2), hi = __builtin_convertvector((f32x2){c, d}, bf16x2);
    return (i32x2){__builtin_bit_cast(int, lo), __builtin_bit_cast(int, hi)};
}
template <int... I, typename F>
__device__ __forceinline__ void unroll(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

__global__ __launch_bounds__(NT, 1) void k_dec_tail(DecTailArgs a) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kg = lane >> 4;
    const int clip = blockIdx.x;

    // ---- fragments: slot i = fragment w + 4 i (8 x 2 block (f / 5, f % 5)); lane row r16 -> (r16 >> 1, r16 & 1) ----
    int vb4[NF], vb5[NF];   // LDS byte address of this lane's row at the smallest tap offset, + 16 kg
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = i < 3 ? w + NW * i : FX;
        const int y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
        vb4[i] = (y * P4 + x) * S4 + kg * 16;   // tap (-2, -2)
        vb5[i] = (y * P5 + x) * S5 + kg * 16;   // tap (-1, -1)
    }

    // ---- weight slabs (64 rows x 64 B) through an LDS ring: lane tid loads / stores 16 B (kq = tid & 3) of row
    // tid >> 2; slab S sits in group S / 4, slot (S / 4) & 1, position S % 4; B fragment j of lane (r16, kg) =
    // row 16 j + r16, k-group kg (16-B slots XOR-swizzled by wsw(row): conflict-free) ----
    const int brow = tid >> 3, kq = (tid >> 1) & 3, kh = tid & 1;   // 8 B per lane: half kh of 16-B group kq
    const int bst = BOFF + brow * 64 + ((kq ^ wsw(brow)) << 4) + kh * 8;   // + slot * 16384 + pos * 4096
    const int bfr = BOFF + r16 * 64 + ((kg ^ wsw(r16)) << 4);        // + slot * 16384 + pos * 4096 + 1024 j
    const bool xw = w < 4;   // this wave computes slot 3 (fragment 24 x channel block w)
    auto read_b = [&](int base, i32x4 (&f)[4], i32x4& fx) {
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = lds16(lds, base + 1024 * j);
        if (xw) fx = lds16(lds, base + 1024 * w);
    };
    auto st16 = [&](int addr, i32x4 v) { *reinterpret_cast<i32x4*>(lds + addr) = v; };
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    auto st8 = [&](int addr, i32x2 v) { *reinterpret_cast<i32x2*>(lds + addr) = v; };

    f32x4 acc[NF][4];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < NF; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    };
    auto mfma_all = [&](const i32x4 (&fa)[NF], const i32x4 (&fb)[4], const i32x4& fbx) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[j]),   // W x A
                                                                     __builtin_bit_cast(bf16x8, fa[i]), acc[i][j], 0, 0, 0);
        if (xw)
            acc[3][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fbx), __builtin_bit_cast(bf16x8, fa[3]),
                                                                acc[3][0], 0, 0, 0);
    };

    // =============================== d_deconv4 ===============================
    {
        // window pieces: lane piece k = 16 B (sg = tid & 3) of window pixel p = tid / 4 + 64 k (p < 602)
        const long long in_clip = (long long)HW * CI4 * 2;
        const __amdgpu_buffer_rsrc_t rsIn = make_rsrc(reinterpret_cast<const char*>(a.in) + clip * in_clip, in_clip);
        int psrc[NPC];
#pragma unroll
        for (int k = 0; k < NPC; ++k) {
            const int p = (tid >> 2) + (NT / 4) * k, sg = tid & 3;
            const int wy = p / P4, wx = p - wy * P4;
            const int iy = wy - 2, ix = wx - 2;
            const bool ok = p < NPIX4 && iy >= 0 && iy < H && ix >= 0 && ix < W;
            psrc[k] = ok ? ((iy * W + ix) * CI4 + sg * 8) * 2 : kOOB;
        }
        const int pdst0 = (tid >> 2) * S4 + (tid & 3) * 16, pdst1 = pdst0 + WBUF;
        const bool last_ok = (tid >> 2) + (NT / 4) * (NPC - 1) < NPIX4;   // piece NPC-1 exists for this lane

        // weights: row r, k = tap * 128 + chunk * 32 + 8 kq; slab (chunk c, tap t) at byte t * 256 + c * 64
        const __amdgpu_buffer_rsrc_t rsW = make_rsrc(a.w4, (long long)CO * 16 * CI4 * 2);
        const int vbl = brow * (16 * CI4 * 2) + kq * 16 + kh * 8;
        auto bpiece = [&](auto tt, int csoff) {
            constexpr int t = decltype(tt)::value;
            return __builtin_amdgcn_raw_buffer_load_b64(rsW, vbl + t * 256, csoff, 0);
        };
        // epilogue parameters -> LDS (read per fragment in the epilogues: no registers held across the loops)
        if (tid < 64) {
            reinterpret_cast<float*>(lds + PSC4)[tid] = a.sc4[tid];
            reinterpret_cast<float*>(lds + PSH4)[tid] = a.sh4[tid];
            reinterpret_cast<float*>(lds + PSC5)[tid] = a.sc5[tid];
            reinterpret_cast<float*>(lds + PSH5)[tid] = a.sh5[tid];
            reinterpret_cast<float*>(lds + PW6)[tid] = a.w6[tid];
        }
        auto par4 = [&](int base, int j) { return *reinterpret_cast<const f32x4*>(lds + base + (16 * j + 4 * kg) * 4); };

        // prologue: window chunk 0 -> buffer 0; weight slabs 0, 1, 2 in flight
        {
            i32x4 pc[NPC];
#pragma unroll
            for (int k = 0; k < NPC; ++k) pc[k] = __builtin_amdgcn_raw_buffer_load_b128(rsIn, psrc[k], 0, 0);
#pragma unroll
            for (int k = 0; k < NPC; ++k)
                if (k < NPC - 1 || last_ok) *reinterpret_cast<i32x4*>(lds + pdst0 + k * (NT / 4) * S4) = pc[k];
        }
        // weight slabs 0..3 -> slot 0 now; 4..7 in flight (stored during slabs 0..3)
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
        zero_acc();
        __syncthreads();

        i32x4 fa[2][NF], fb[2][4], fbx[2];
        i32x4 pr[4];   // next chunk's window pieces: loaded at tap k < NPC, stored at tap k + 3
        int vq[NF];    // the fragment bases of the buffer being read: vb4 + (chunk & 1) * WBUF
#pragma unroll
        for (int i = 0; i < NF; ++i) vq[i] = vb4[i];
        auto read_a = [&](auto tt, i32x4 (&f)[NF]) {
            constexpr int t = decltype(tt)::value % 16;
            constexpr int imm = ((3 - t / 4) * P4 + (3 - t % 4)) * S4;   // tap (1 - t/4, 1 - t%4) from (-2, -2)
#pragma unroll
            for (int i = 0; i < 3; ++i) f[i] = lds16(lds + imm, vq[i]);
            if (xw) f[3] = lds16(lds + imm, vq[3]);
        };
        read_a(std::integral_constant<int, 0>{}, fa[0]);
        read_b(bfr, fb[0], fbx[0]);
        // slab S = 16 c + t; group S / 4 (slot parity (t / 4) & 1: 4 groups per chunk); every 4 slabs a barrier
        // publishes the next group's weights (stored during this group) and, at t = 15, the next chunk's window
        for (int c = 0; c < 4; ++c) {
            const int pdn = (c & 1) ? pdst0 : pdst1;     // next chunk -> the other buffer
            const int cs = c * 64, cn = (c + 1) * 64;    // this / next chunk's channel byte offset
            unroll(std::make_integer_sequence<int, 16>{}, [&](auto tt) {
                constexpr int t = decltype(tt)::value;
                __builtin_amdgcn_sched_barrier(0);
                // weights of slab S + 4 (loaded 4 slabs ago) -> slot of group S / 4 + 1; slab S + 8 -> registers
                st8(bst + (((t / 4) + 1) & 1) * 16384 + (t % 4) * 4096, pb[t & 3]);
                if constexpr (t + 8 < 16) pb[t & 3] = bpiece(std::integral_constant<int, t + 8>{}, cs);
                else pb[t & 3] = bpiece(std::integral_constant<int, t + 8 - 16>{}, cn);   // past the layer: reads zero
                // window piece t of chunk c + 1 (after the last chunk: a harmless re-read, never used)
                if constexpr (t < NPC) pr[t & 3] = __builtin_amdgcn_raw_buffer_load_b128(rsIn, psrc[t], cn, 0);
                if constexpr (t >= 3 && t - 3 < NPC) {
                    if (t - 3 < NPC - 1 || last_ok) st16(pdn + (t - 3) * (NT / 4) * S4, pr[(t - 3) & 3]);
                }
                if constexpr (t % 4 == 3) __syncthreads();
                if constexpr (t == 15) {
#pragma unroll
                    for (int i = 0; i < NF; ++i) vq[i] = vb4[i] + ((c + 1) & 1) * WBUF;
                }
                // the next slab's fragments (LDS) go out before this slab's MFMAs
                read_a(std::integral_constant<int, t + 1>{}, fa[(t + 1) & 1]);
                read_b(bfr + (((t + 1) / 4) & 1) * 16384 + ((t + 1) % 4) * 4096, fb[(t + 1) & 1], fbx[(t + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
                mfma_all(fa[t & 1], fb[t & 1], fbx[t & 1]);
            });
        }
        __syncthreads();   // every window read done: the d_deconv5 image goes over the windows

        // zero the d_deconv5 image (its padding ring reads as zero)
        for (int o = tid * 16; o < OIMG; o += NT * 16) *reinterpret_cast<i32x4*>(lds + o) = (i32x4){0, 0, 0, 0};
        __syncthreads();
        // epilogue: BN + LeakyReLU -> bf16 at image pixel (y + 1, x + 1); lane = block row r16, channels
        // 16 j + 4 kg .. + 3: one 8-B store per fragment pair (i, j)
        // BN quads read once per channel block (the interleaved LDS stores keep the compiler from reusing reads)
        f32x4 sc4q[4], sh4q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) { sc4q[j] = par4(PSC4, j); sh4q[j] = par4(PSH4, j); }
        auto st_quad = [&](int px, int j, const f32x4& v, const f32x4& sc, const f32x4& sh) {   // channels 16 j + 4 kg + e
            st8(px + 32 * j, pack4(bn_lrelu(v[0], sc[0], sh[0]), bn_lrelu(v[1], sc[1], sh[1]),
                                   bn_lrelu(v[2], sc[2], sh[2]), bn_lrelu(v[3], sc[3], sh[3])));
        };
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            if (i == 3 && !xw) continue;
            const int f = i < 3 ? w + NW * i : FX;
            const int y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
            const int px = ((y + 1) * P5 + x + 1) * S5 + 8 * kg;
            if (i < 3) {
#pragma unroll
                for (int j = 0; j < 4; ++j) st_quad(px, j, acc[i][j], sc4q[j], sh4q[j]);
            } else {
                st_quad(px, w, acc[3][0], par4(PSC4, w), par4(PSH4, w));
            }
        }
        __syncthreads();
    }

    // =============================== d_deconv5 + d_deconv6 ===============================
    auto par5 = [&](int base, int j) { return *reinterpret_cast<const f32x4*>(lds + base + (16 * j + 4 * kg) * 4); };
    float* const outc = a.out + (long long)clip * (4 * HW);
    const __amdgpu_buffer_rsrc_t rsW5 = make_rsrc(a.w5, (long long)ph_woff(4) * 2);
    // the padded slab sequence over the four phases (phase p: 2 nt slabs, slab = 2 tap + chunk, padded to a multiple
    // of 4) is compile-time: tap offsets, ring slots and weight offsets are immediates / scalar constants
    int vrow5[3];   // weight row byte offset of this lane's ring piece for kpad 256, 384, 576
    vrow5[0] = brow * (4 * CO * 2) + kq * 16 + kh * 8;
    vrow5[1] = brow * (6 * CO * 2) + kq * 16 + kh * 8;
    vrow5[2] = brow * (9 * CO * 2) + kq * 16 + kh * 8;
    auto bpiece5 = [&](auto gg) {   // ring piece of global padded slab g (past the end: phase 3's slab 0, unused)
        constexpr int g = decltype(gg)::value < ph_pstart(4) ? decltype(gg)::value : ph_pstart(3);
        constexpr int p = ph_ofp(g), sl = g - ph_pstart(p), sv = sl < 2 * ph_nt(p) ? sl : 0;
        constexpr int kk = p == 0 ? 0 : p == 3 ? 2 : 1;
        return __builtin_amdgcn_raw_buffer_load_b64(rsW5, vrow5[kk], ph_woff(p) * 2 + sv * 64, 0);
    };
    auto read_a5 = [&](auto gg, i32x4 (&f)[NF]) {
        constexpr int g = decltype(gg)::value;
        constexpr int p = ph_ofp(g), sl = g - ph_pstart(p), tap = sl / 2, c = sl % 2;
        constexpr int dy = (p >> 1) - tap / ph_nx(p), dx = (p & 1) - tap % ph_nx(p);
        constexpr int imm = ((dy + 1) * P5 + (dx + 1)) * S5 + c * 64;
#pragma unroll
        for (int i = 0; i < 3; ++i) f[i] = lds16(lds + imm, vb5[i]);
        if (xw) f[3] = lds16(lds + imm, vb5[3]);
    };
    auto epilogue5 = [&](auto pp) {
        constexpr int p = decltype(pp)::value, py = p >> 1, px = p & 1;
        // d_deconv6 partial dot of this lane's 16 channels (16 j + 4 kg + e) for block row r16 of each slot
        float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // channels 16 j + 4 kg + e
            const f32x4 sc = par5(PSC5, j), sh = par5(PSH5, j), w6 = par5(PW6, j);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)   // y rounded to bf16 as the unfused path stores it
                    part[i] = fmaf((float)(bf16_t)bn_lrelu(acc[i][j][e], sc[e], sh[e]), w6[e], part[i]);
        }
        if (xw) {   // slot 3: fragment 24, channels 16 w + 4 kg + e
            const f32x4 sc = par5(PSC5, w), sh = par5(PSH5, w), w6 = par5(PW6, w);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                part[3] = fmaf((float)(bf16_t)bn_lrelu(acc[3][0][e], sc[e], sh[e]), w6[e], part[3]);
        }
        // sum over the four lane rows (kg) of a slot, three swaps for four slots: lanes 0-31 <-> 32-63 pairs slots
        // (0, 1) and (2, 3), then rows 0 / 2 <-> 1 / 3: lane row kg ends with the total of slot {0, 2, 1, 3}[kg]
        auto swap_add = [](float x, float y, auto sw) {
            const auto r = sw(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, y));
            return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
        };
        auto sw32 = [](unsigned x, unsigned y) { return __builtin_amdgcn_permlane32_swap(x, y, false, false); };
        auto sw16 = [](unsigned x, unsigned y) { return __builtin_amdgcn_permlane16_swap(x, y, false, false); };
        const float tot = swap_add(swap_add(part[0], part[1], sw32), swap_add(part[2], part[3], sw32), sw16);
        const int i = ((kg & 1) << 1) | (kg >> 1);
        if (i < 3) {
            const int f = w + NW * i, y = 8 * (f / 5) + (r16 >> 1), x = 2 * (f % 5) + (r16 & 1);
            outc[(2 * y + py) * (2 * W) + 2 * x + px] = tot + a.b6;
        } else if (xw) {
            reinterpret_cast<float*>(lds + PAR + PXB)[16 * w + r16] = tot;   // this wave's 16-channel share
        }
        // fragment 24: the four waves' shares, summed in a fixed order by wave 0 (the buffer is rewritten only at the
        // next phase end, two or more slab-group barriers later)
        __syncthreads();
        if (w == 0 && lane < 16) {
            const float* xb = reinterpret_cast<const float*>(lds + PAR + PXB);
            const float v = ((xb[lane] + xb[16 + lane]) + xb[32 + lane]) + xb[48 + lane];
            const int y = 8 * (FX / 5) + (lane >> 1), x = 2 * (FX % 5) + (lane & 1);
            outc[(2 * y + py) * (2 * W) + 2 * x + px] = v + a.b6;
        }
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
    zero_acc();
    __syncthreads();
    i32x4 fa[2][NF], fb[2][4], fbx[2];
    read_a5(std::integral_constant<int, 0>{}, fa[0]);
    read_b(bfr, fb[0], fbx[0]);
    // global padded slab g: store g + 4 -> slot ((g / 4) + 1) & 1, load g + 8, barrier every 4 slabs; the fragments of
    // g + 1 (the next phase's first slab at a phase end, read after its epilogue) go out before g's MFMAs
    unroll(std::make_integer_sequence<int, ph_pstart(4)>{}, [&](auto gg) {
        constexpr int g = decltype(gg)::value, p = ph_ofp(g);
        constexpr bool real = g - ph_pstart(p) < 2 * ph_nt(p), last = g + 1 == ph_pstart(p + 1);
        __builtin_amdgcn_sched_barrier(0);
        st8(bst + (((g / 4) + 1) & 1) * 16384 + (g % 4) * 4096, pb[g & 3]);
        pb[g & 3] = bpiece5(std::integral_constant<int, g + 8>{});
        if constexpr (g % 4 == 3) __syncthreads();
        if constexpr (!last && g + 1 - ph_pstart(p) < 2 * ph_nt(p)) {
            read_a5(std::integral_constant<int, g + 1>{}, fa[(g + 1) & 1]);
            read_b(bfr + (((g + 1) / 4) & 1) * 16384 + ((g + 1) % 4) * 4096, fb[(g + 1) & 1], fbx[(g + 1) & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (real) mfma_all(fa[g & 1], fb[g & 1], fbx[g & 1]);
        if constexpr (last) {
            epilogue5(std::integral_constant<int, p>{});
            if constexpr (p < 3) {
                zero_acc();
                read_a5(std::integral_constant<int, g + 1>{}, fa[(g + 1) & 1]);
                read_b(bfr + (((g + 1) / 4) & 1) * 16384 + ((g + 1) % 4) * 4096, fb[(g + 1) & 1], fbx[(g + 1) & 1]);
            }
        }
    });
}

}  // namespace

bool dec_tail_supported(const DecTailArgs& a) {
    // the compile-time geometry above: window / image extents and tap grids of network.py's layers
    if (a.N <= 0 || a.nt4 != 16 || a.kpad4 != 16 * CI4 || a.dy4 != 1 || a.dx4 != 1 || a.nx4 != 4) return false;
    if (a.pt4 != 2 || a.pl4 != 2 || a.rows4 != 43 || a.pitch4 > P4 || a.pt5 != 1 || a.pl5 != 1 || a.rows5 != 42 || a.pitch5 > P5)
        return false;
    for (int p = 0; p < 4; ++p)
        if (a.nt5[p] != ph_nt(p) || a.kpad5[p] != ph_nt(p) * CO || a.dy5[p] != (p >> 1) || a.dx5[p] != (p & 1) ||
            a.nx5[p] != ph_nx(p) || a.woff5[p] != ph_woff(p))
            return false;
    return true;
}

int launch_dec_tail(const DecTailArgs& a, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_dec_tail, LDS_BYTES)) return rc;
    hipLaunchKernelGGL(k_dec_tail, dim3(a.N), dim3(NT), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
