// K2-K5: NHWC implicit-GEMM convolution on MFMA for gfx950, with the Keras layer tail fused.
//
// One kernel covers every layer of /root/reference/network.py's graph:
//   Convolution2D(padding='same')        (network.py:89-105, :139-169)  forward taps, stride (sy, sx)
//   Deconvolution2D(padding='same')      (network.py:113-133)            one launch, blockIdx.z = output
//                                                                         phase (sub-pixel split), each
//                                                                         phase a stride-1 gather conv
//   Dense                                (network.py:56, :69, :75)       1 tap, Hi = Wi = 1, Ci = K
// and fuses the epilogue: bias + BatchNormalization (folded to per-channel scale/shift on the
// host), LeakyReLU(0.3), MaxPooling2D(2,2) (video convs; rows of a tile are ordered so the four
// pixels of a pool window are the four accumulator rows one lane holds), Dropout = identity,
// Flatten/concatenate (strided output addressing into the fused 5248-wide embedding).
//
// GEMM view: M = output pixels (N clips x Hq x Wq), N = Cout, K = taps x Ci.  Tile 128 x BN,
// 256 threads = 4 wavefronts (2 x 2), each wave 64 x BN/2 built from 16x16 MFMA tiles.
// The K loop walks 64-byte "slabs": 32 bf16 (one v_mfma_f32_16x16x32_bf16) or 16 fp32 (four
// exact-fp32 v_mfma_f32_16x16x4_f32) per row, so the LDS geometry is identical for both dtypes.
// A (im2col gathered on the fly, 16-byte chunks, zero padding = TF 'SAME') and B (packed weights
// [Cout][Kpad]) are register-staged into a double-buffered, XOR-swizzled LDS tile (one barrier
// per slab; the next slab's global loads are in flight during the current slab's MFMAs).
#include <cstdlib>
#include <type_traits>

#include "avse_common.h"

namespace avse {
namespace {

constexpr int BM = 128;
constexpr int MAX_TAPS_LDS = 64;   // taps of one phase (largest: 25)
constexpr float LRELU = 0.3f;

template <typename T> struct Vec16;
template <> struct Vec16<bf16_t> { typedef i32x4 type; };
template <> struct Vec16<float> { typedef i32x4 type; };
template <> struct Vec16<_Float16> { typedef i32x4 type; };

__device__ __forceinline__ int swz(int row) { return ((row >> 3) & 1) * 3; }

__device__ __forceinline__ float to_f(bf16_t v) { return (float)v; }
__device__ __forceinline__ float to_f(float v) { return v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return (bf16_t)v; }
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }

// one output value at element rowbase + n of a layer output: OutT (bf16 / fp32), or with a.out_s16 the split pair
// layout (include/avse.h AVSE_F32_SPLIT: per pixel and 16 channels [h(16) | l(16)] f16; rowbase in halves)
// Returns true when a pair cannot hold x (pair_out_of_range: the caller folds it into one range report).
template <typename OutT>
__device__ __forceinline__ bool store_val(const ConvArgs& a, long long rowbase, int n, float x) {
    if (a.out_s16) {
        _Float16* o = reinterpret_cast<_Float16*>(a.out) + rowbase + 32 * (n >> 4) + (n & 15);
        const _Float16 h = (_Float16)x;
        o[0] = h;
        o[16] = (_Float16)(x - (float)h);
        return pair_out_of_range(x);
    }
    reinterpret_cast<OutT*>(a.out)[rowbase + n] = from_f<OutT>(x);
    return false;
}

struct RowInfo {
    int cbase;          // byte offset of the row's clip from the block's first clip
    int iy0, ix0;       // yq*sy, xq*sx
    bool valid;
};

// Buffer-resource loads: out-of-range offsets return zeros in hardware, so padding / ragged tiles
// need no branch around the load (a "load or zero" branch makes hipcc drain vmcnt per load).
constexpr int kOOB = 0x7fffff00;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);
}

// FAST (Ci a multiple of the slab, i.e. every layer but a_conv1): a slab never straddles a tap, so the A row
// offsets are computed once per tap and a slab's channel offset is the buffer load's scalar soffset; three LDS
// buffers make the buffer of every unrolled step compile-time.  The generic path decoded (tap, channel) and
// re-checked the bounds of both rows every slab: ~138 instructions per slab against 16 MFMAs of 16 cycles
// (a wave issues at most one instruction per 4 cycles), so the short-K layers were issue-bound.
// occupancy: more resident workgroups hide the per-tile load latency of the short-K layers (8-18 slabs per
// tile for the decoder): 4 per CU for BN = 64 (<= 128 VGPRs, 36 KB LDS), 3 for BN = 128 (<= 168, 48 KB)
// fp32: one workgroup per CU fewer (the blocked-summation partials below need another 32 / 64 VGPRs)
template <typename T, int BN, bool FAST, bool S16 = false> constexpr int conv_occupancy() {
    return !FAST ? 2 : (BN == 64 ? 4 : 3) - (sizeof(T) == 4 || S16 ? 1 : 0);
}
// fp32 blocked summation: the K loop accumulates FP32_BLOCK slabs (FP32_BLOCK * 16 products per output) into a
// zeroed partial that is then added to the running sum, so the running sum takes K / 128 roundings instead of
// K / 4 (one per 16x16x4 MFMA).
constexpr int FP32_BLOCK = kFp32Block;
// timing ablations of the FAST K loop (tools/kconv_ablate.hip only; 0 in the library): 1 = no global loads, 2 = no
// LDS slab stores, 4 = no MFMAs, 8 = no workgroup barrier in the loop, 16 = no fragment reads
#ifndef AVSE_KCONV_ABL
#define AVSE_KCONV_ABL 0
#endif
constexpr int KABL = AVSE_KCONV_ABL;   // avse_common.h (train.hip's block-exact split-K plans on it)

// S16 (AVSE_F32_SPLIT's generic layers): split-f16 products on the 16-bit matrix cores.  The LDS A slab row is
// [h(16) | l(16)] f16 of 16 real k (h = f16(x), l = f16(x - h)): with T = float (fp32 input: a_conv1, a no_halo
// v_conv1) store_slab splits the loaded floats into those 64 bytes; with T = _Float16 the input already holds the pairs
// in that layout (written by the producing layer's epilogue, a.out_s16) and a slab is copied as is — Ci, strides, kpad
// and w_off then count halves.  The host packs each weight slab row as [Bh(16) | Bl(16)] (per-channel power-of-two
// scaled, the BN scale undoes it).  Per slab two v_mfma_f32_16x16x32_f16 per fragment pair: the B fragment of the first
// reads the Bh half for every lane (k-group fg & 1), of the second the Bl half, so they sum Ah Bh + Al Bh and Ah Bl +
// Al Bl (conv_stream.hip's split notes; 4x fewer matrix-core cycles than four 16x16x4 f32 MFMAs per slab).  Outputs
// are fp32 or, with a.out_s16, pairs.
template <typename T, int BN, bool FAST, bool S16 = false>
__global__ __launch_bounds__(256, (conv_occupancy<T, BN, FAST, S16>())) void k_conv(ConvArgs a) {
    static_assert(!S16 || sizeof(T) == 4 || std::is_same_v<T, _Float16>, "split operands: fp32 or pair storage");
    static_assert(S16 || !std::is_same_v<T, _Float16>, "f16 storage only as split pairs");
    constexpr bool PAIRS = S16 && sizeof(T) == 2;   // the input holds split pairs (slab = 32 halves = 16 real k)
    using OutT = std::conditional_t<S16, float, T>;
    constexpr int CH = 16 / sizeof(T);          // elements per 16-byte chunk
    constexpr int SLAB = 64 / sizeof(T);        // elements per 64-byte k-slab
    constexpr int WN = BN / 2;                  // wave tile N
    constexpr int NJ = WN / 16;                 // 16-wide N fragments per wave
    constexpr int NI = 4;                       // 16-high M fragments per wave (64 rows)
    constexpr int BCH = BN * 4 / 256;           // B chunks per thread
    constexpr int NBUF = FAST ? 3 : 2;          // LDS buffers

    __shared__ __attribute__((aligned(16))) char lds[NBUF * (BM + BN) * 64];
    // this phase's tap table, staged in LDS: a per-lane global tap load feeding the A addresses made every
    // slab wait for vmcnt — which retires in order, so it also drained all the slabs in flight
    __shared__ int2 tap_lds[MAX_TAPS_LDS];
    // buffer b: A tile at lds + b*(BM+BN)*64, B tile right after it
#define AS(b) (lds + (b) * (BM + BN) * 64)
#define BS(b) (lds + (b) * (BM + BN) * 64 + BM * 64)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int zphase = blockIdx.z / a.ksplit, zsplit = blockIdx.z % a.ksplit;
    const ConvPhase ph = a.ph[zphase];
    const int M = a.N * a.Hq * a.Wq;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    // split-K: this block reduces slabs [s_begin, s_end) of the phase's K
    const int nslab_all = ph.kpad / SLAB;
    const int sps = a.ksplit_slabs > 0 ? a.ksplit_slabs : (nslab_all + a.ksplit - 1) / a.ksplit;
    const int s_begin = zsplit * sps;
    const int s_end = min(nslab_all, s_begin + sps);
    for (int i = threadIdx.x; i < ph.ntaps && i < MAX_TAPS_LDS; i += 256) tap_lds[i] = a.taps[ph.tap_off + i];
    __syncthreads();

    // ---- per-thread A rows (2 chunks: rows r and r + 64, same chunk column g) ----
    const int g = tid & 3;
    const int clip_first = a.pool ? (m0 >> 2) / ((a.Hq >> 1) * (a.Wq >> 1)) : m0 / (a.Hq * a.Wq);
    const long long clip_bytes = a.in_clip_stride * (long long)sizeof(T);
    const __amdgpu_buffer_rsrc_t rsA = make_rsrc(reinterpret_cast<const char*>(a.in) + clip_first * clip_bytes,
                                                 (a.N - clip_first) * clip_bytes);
    RowInfo ri[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int row = (tid >> 2) + 64 * h;
        const int m = m0 + row;
        ri[h].valid = m < M;
        const int mm = ri[h].valid ? m : m0;
        int clip, yq, xq;
        if (a.pool) {
            const int p = mm >> 2, q = mm & 3;
            const int pw = a.Wq >> 1, phh = a.Hq >> 1;
            clip = p / (phh * pw);
            const int r = p - clip * phh * pw;
            yq = 2 * (r / pw) + (q >> 1);
            xq = 2 * (r % pw) + (q & 1);
        } else {
            clip = mm / (a.Hq * a.Wq);
            const int r = mm - clip * a.Hq * a.Wq;
            yq = r / a.Wq;
            xq = r % a.Wq;
        }
        ri[h].cbase = (int)((clip - clip_first) * clip_bytes);
        ri[h].iy0 = yq * a.sy;
        ri[h].ix0 = xq * a.sx;
    }
    // chunk k position: tap j, channel c (incremental across slabs)
    int kj = (s_begin * SLAB + g * CH) / a.Ci;
    int kc = s_begin * SLAB + g * CH - kj * a.Ci;

    const __amdgpu_buffer_rsrc_t rsB = make_rsrc(reinterpret_cast<const char*>(a.w) + ph.w_off * sizeof(T),
                                                 (long long)a.Co * ph.kpad * sizeof(T));

    // ---- FAST path state: load cursor (slab lk = tap kjf x chunks-per-tap + csf), per-tap A row offsets ----
    const int cpt = FAST ? a.Ci / SLAB : 1;
    int lk = s_begin, kjf = s_begin / cpt, csf = s_begin - kjf * cpt;
    int aoff[2], boff[BCH];
    auto tap_offs = [&]() {
        const bool tap_ok = kjf < ph.ntaps;
        const int2 t = tap_lds[tap_ok ? kjf : ph.ntaps - 1];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int iy = ri[h].iy0 + t.x, ix = ri[h].ix0 + t.y;
            const bool ok = ri[h].valid && tap_ok && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
            aoff[h] = ok ? ri[h].cbase + ((iy * a.Wi + ix) * a.Ci + g * CH) * (int)sizeof(T) : kOOB;
        }
    };
    if constexpr (FAST) {
        tap_offs();
#pragma unroll
        for (int h = 0; h < BCH; ++h) {
            const int c = tid + 256 * h;
            const int n = n0 + (c >> 2);
            boff[h] = n < a.Co ? (n * ph.kpad + (c & 3) * CH) * (int)sizeof(T) : kOOB;
        }
    }

    // epilogue parameters of this lane's columns, loaded before the K loop so that their latency is hidden
    // (loaded at the end they exposed one global-load latency per tile: ~20 us on d_deconv5's 3200 tiles)
    float esc[NJ], esh[NJ], ewf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WN + 16 * j + (lane & 15);
        const bool ok = n < a.Co && a.ksplit == 1;
        esc[j] = ok ? a.scale[n] : 0.f;
        esh[j] = ok ? a.shift[n] : 0.f;
        ewf[j] = (ok && a.fuse_w) ? a.fuse_w[n] : 0.f;
    }

    // P register stages: slabs s+1 .. s+P-1 are in flight while slab s computes (a layer with a short K loop
    // was a serial chain of one global-load latency per slab: ~0.7-1.2 us each, measured at batch 8)
    constexpr int P = 3;
    i32x4 ras[P][2], rbs[P][BCH];
    auto load_slab = [&](int s, i32x4 (&ra)[2], i32x4 (&rb)[BCH]) {
        if constexpr (FAST && (KABL & 1)) {
            ra[0][0] ^= s;   // keep the register sets live without the loads
            return;
        }
        if constexpr (FAST) {
            // A: the channel chunk is the scalar offset (an out-of-range row offset stays out of range);
            // B: rows past Cout and slabs past the phase's K read zeros (range-checked voffset)
#pragma unroll
            for (int h = 0; h < 2; ++h) ra[h] = __builtin_amdgcn_raw_buffer_load_b128(rsA, aoff[h], csf * 64, 0);
#pragma unroll
            for (int h = 0; h < BCH; ++h) rb[h] = __builtin_amdgcn_raw_buffer_load_b128(rsB, boff[h] + lk * 64, 0, 0);
            ++lk;
            if (++csf == cpt) {
                csf = 0;
                ++kjf;
                tap_offs();
            }
            return;
        }
        // A
        const bool tap_ok = kj < ph.ntaps;
        const int2 t = tap_lds[tap_ok ? kj : ph.ntaps - 1];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int iy = ri[h].iy0 + t.x, ix = ri[h].ix0 + t.y;
            const bool ok = ri[h].valid && tap_ok && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
            const int off = ok ? ri[h].cbase + ((iy * a.Wi + ix) * a.Ci + kc) * (int)sizeof(T) : kOOB;
            ra[h] = __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0);
        }
        // B (rows past Cout read zeros)
#pragma unroll
        for (int h = 0; h < BCH; ++h) {
            const int c = tid + 256 * h;
            const int row = c >> 2, gg = c & 3;
            const int n = n0 + row;
            const int off = n < a.Co ? (n * ph.kpad + s * SLAB + gg * CH) * (int)sizeof(T) : kOOB;
            rb[h] = __builtin_amdgcn_raw_buffer_load_b128(rsB, off, 0, 0);
        }
        // advance the A chunk position by one slab
        kc += SLAB;
        while (kc >= a.Ci) { kc -= a.Ci; ++kj; }
    };
    bool in_bad = false;   // S16 on an fp32 input: an input value the pair split cannot hold (range guard)
    auto store_slab = [&](int buf, const i32x4 (&ra)[2], const i32x4 (&rb)[BCH]) {
        if constexpr (FAST && (KABL & 2)) {
            if (ra[0][0] == 0x7fffffff && rb[0][0] == 0x7fffffff) *reinterpret_cast<int*>(AS(buf)) = 1;
            return;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = (tid >> 2) + 64 * h;
            if constexpr (S16 && !PAIRS) {
                // floats 4g .. 4g+3 of the row: their h pieces to k-group g >> 1 (half g & 1), l pieces to 2 + (g >> 1)
                const f32x4 x = __builtin_bit_cast(f32x4, ra[h]);
                f16x4 hi, lo;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    hi[e] = (_Float16)x[e];
                    lo[e] = (_Float16)(x[e] - (float)hi[e]);
                    in_bad |= pair_out_of_range(x[e]);
                }
                char* rp = AS(buf) + row * 64 + (g & 1) * 8;
                *reinterpret_cast<f16x4*>(rp + (((g >> 1) ^ swz(row)) << 4)) = hi;
                *reinterpret_cast<f16x4*>(rp + (((2 + (g >> 1)) ^ swz(row)) << 4)) = lo;
            } else {
                *reinterpret_cast<i32x4*>(AS(buf) + row * 64 + ((g ^ swz(row)) << 4)) = ra[h];
            }
        }
#pragma unroll
        for (int h = 0; h < BCH; ++h) {
            const int c = tid + 256 * h;
            const int row = c >> 2, gg = c & 3;
            *reinterpret_cast<i32x4*>(BS(buf) + row * 64 + ((gg ^ swz(row)) << 4)) = rb[h];
        }
    };

    f32x4 acc[NI][NJ], part[NI][NJ];   // part: fp32 blocked summation only
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int nblk = 0;

    const int fr = lane & 15, fg = lane >> 4;
    if (s_begin < s_end) {
    // loads past s_end read zeros (taps past ntaps / rows past the phase's weights are out of range)
#pragma unroll
    for (int p = 0; p < P; ++p) load_slab(s_begin + p, ras[p], rbs[p]);
    store_slab(0, ras[0], rbs[0]);
    load_slab(s_begin + P, ras[0], rbs[0]);   // set of slab x: (x - s_begin) % P
    __syncthreads();

    auto step = [&](auto qidx, int s) {
        constexpr int q = decltype(qidx)::value;           // (s - s_begin) % P
        constexpr int qn = (q + 1) % P;
        const int buf = FAST ? q : (s - s_begin) & 1;      // FAST: three buffers, slab x in buffer (x - s_begin) % 3
        i32x4 fa[NI], fb[NJ], fl[NJ];
        if constexpr (FAST && (KABL & 16)) {
#pragma unroll
            for (int i = 0; i < NI; ++i) fa[i] = (i32x4){s + i, lane, 0, 0};
#pragma unroll
            for (int j = 0; j < NJ; ++j) fb[j] = fl[j] = (i32x4){s - j, lane, 1, 0};
        } else {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int row = wm * 64 + 16 * i + fr;
            fa[i] = *reinterpret_cast<const i32x4*>(AS(buf) + row * 64 + ((fg ^ swz(row)) << 4));
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = wn * WN + 16 * j + fr;
            fb[j] = *reinterpret_cast<const i32x4*>(BS(buf) + row * 64 + (((S16 ? (fg & 1) : fg) ^ swz(row)) << 4));
            if constexpr (S16) fl[j] = *reinterpret_cast<const i32x4*>(BS(buf) + row * 64 + (((2 + (fg & 1)) ^ swz(row)) << 4));
        }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                if constexpr (FAST && (KABL & 4)) {
                    part[i][j][0] += __builtin_bit_cast(float, fa[i][0] ^ fb[j][1] ^ fl[j][2]);
                } else if constexpr (S16) {
                    part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        __builtin_bit_cast(f16x8, fa[i]), __builtin_bit_cast(f16x8, fb[j]), part[i][j], 0, 0, 0);
                    part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        __builtin_bit_cast(f16x8, fa[i]), __builtin_bit_cast(f16x8, fl[j]), part[i][j], 0, 0, 0);
                } else if constexpr (sizeof(T) == 2) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
                } else {
                    const f32x4 av = __builtin_bit_cast(f32x4, fa[i]);
                    const f32x4 bv = __builtin_bit_cast(f32x4, fb[j]);
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], part[i][j], 0, 0, 0);
                }
            }
        if constexpr (sizeof(T) == 4 || S16) {
            if (++nblk == FP32_BLOCK) {
                nblk = 0;
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        acc[i][j] += part[i][j];
                        part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
                    }
            }
        }
        if constexpr (FAST) {
            // unconditional: past s_end the loads read zeros / unused rows and the buffer is never read
            // (buffer qn held slab s-2, read before the barrier of step s-2)
            store_slab(qn, ras[qn], rbs[qn]);
            load_slab(s + 1 + P, ras[qn], rbs[qn]);
        } else if (s + 1 < s_end) {
            store_slab(buf ^ 1, ras[qn], rbs[qn]);   // slab s+1, loaded P-1 steps ago
            load_slab(s + 1 + P, ras[qn], rbs[qn]);  // refill with slab s+1+P (the load cursor is sequential)
        }
        if constexpr (!(FAST && (KABL & 8))) __syncthreads();
    };
    for (int s = s_begin; s < s_end; s += P) {
        step(std::integral_constant<int, 0>{}, s);
        if (s + 1 < s_end) step(std::integral_constant<int, 1>{}, s + 1);
        if (s + 2 < s_end) step(std::integral_constant<int, 2>{}, s + 2);
    }
    }

#undef AS
#undef BS
    if constexpr (S16 && !PAIRS) range_report(a.range_flag, a.range_in_bit, in_bad);
    if constexpr (sizeof(T) == 4 || S16) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] += part[i][j];
    }
    // ---- epilogue: scale/shift (bias + BN), [pool], LeakyReLU, strided NHWC store ----
    if (a.ksplit > 1) {
        // raw fp32 partial sums in MFMA-native order, consumed only by k_splitk_reduce_tiles: unit
        // ((zsplit * tiles + tile) * NI*NJ + i*NJ + j) * 256 + tid is this thread's f32x4 of fragment (i, j)
        // (4 rows of one column), so every store instruction writes 4 contiguous KB (row-major partials
        // were 4-byte stores strided by Cout: 64 per lane, the bulk of a short-K dense layer's time)
        const int tiles = gridDim.x * gridDim.y, tile = blockIdx.y * gridDim.x + blockIdx.x;
        f32x4* part = reinterpret_cast<f32x4*>(a.partial) + (size_t)(zsplit * tiles + tile) * (NI * NJ) * 256 + tid;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) part[(i * NJ + j) * 256] = acc[i][j];
        return;
    }
    // output row -> element offset, decomposed once per (fragment, row) instead of per element: the
    // three runtime integer divisions per stored value used to be the floor of every short-K layer
    long long orow[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int mb = m0 + wm * 64 + 16 * i + 4 * fg;   // first of this lane's 4 rows
        if (a.pool) {
            const int p = mb >> 2;
            const int pw = a.Wq >> 1, phh = a.Hq >> 1;
            const int clip = p / (phh * pw);
            const int r = p - clip * phh * pw;
            orow[i][0] = mb < M ? clip * a.out_clip_stride + (long long)r * a.out_pix_stride + a.out_c_off : -1;
        } else {
            const int hw = a.Hq * a.Wq;
            int clip = mb / hw;
            int rr = mb - clip * hw;
            int yq = rr / a.Wq, xq = rr - yq * a.Wq;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int oy = yq * a.oys + ph.py, ox = xq * a.oxs + ph.px;
                orow[i][r] = mb + r < M ? clip * a.out_clip_stride + (long long)(oy * a.Wo + ox) * a.out_pix_stride + a.out_c_off : -1;
                if (++xq == a.Wq) { xq = 0; if (++yq == a.Hq) { yq = 0; ++clip; } }
            }
        }
    }
    if constexpr (BN == 64) {
        if (a.fuse_w) {   // d_deconv5 + d_deconv6: 64 -> 1 dot in the epilogue (all 64 channels are in this tile)
            float part[NI][4];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) part[i][r] = 0.f;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float x = acc[i][j][r] * esc[j] + esh[j];
                        if (a.act) x = x >= 0.f ? x : LRELU * x;
                        part[i][r] = fmaf(S16 ? x : to_f(from_f<OutT>(x)), ewf[j], part[i][r]);
                    }
            }
            // sum over the 16 lanes holding the same rows (lane bits 0..3 = column within a fragment): DPP
            // row_ror 8, 4, 2, 1 inside the 16-lane row (each add one VALU op; __shfl_xor went through LDS)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = part[i][r];
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xf, 0xf, false));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x122, 0xf, 0xf, false));
                    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xf, 0xf, false));
                    part[i][r] = v;
                }
            // then over the two column halves (wn = 0, 1) through LDS (the K loop ended on a barrier)
            float* red = reinterpret_cast<float*>(lds);
            if (wn == 1 && fr == 0)
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) red[wm * 64 + 16 * i + 4 * fg + r] = part[i][r];
            __syncthreads();
            if (wn == 0 && fr == 0)
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (orow[i][r] >= 0)
                            a.fuse_out[orow[i][r]] = part[i][r] + red[wm * 64 + 16 * i + 4 * fg + r] + a.fuse_bias;
            return;
        }
    }
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WN + 16 * j + fr;
        if (n >= a.Co) continue;
        const float sc = esc[j], sh = esh[j];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * sc + sh;
            if (a.pool) {
                if (orow[i][0] < 0) continue;
                float x = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
                if (a.act) x = x >= 0.f ? x : LRELU * x;
                bad |= store_val<OutT>(a, orow[i][0], n, x);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (orow[i][r] < 0) continue;
                    float x = v[r];
                    if (a.act) x = x >= 0.f ? x : LRELU * x;
                    bad |= store_val<OutT>(a, orow[i][r], n, x);
                }
            }
        }
    }
    if constexpr (S16) range_report(a.range_flag, a.range_bit, bad);
}

// split-K tail for k_conv's MFMA-native partials: one thread per f32x4 unit (4 rows of one column of one
// fragment), summed over the splits, then scale/shift, [2x2 max pool: the 4 rows are one window],
// LeakyReLU, strided store.  Single phase (dense layers, v_conv6).
template <typename T, int BN>
__global__ void k_splitk_reduce_tiles(ConvArgs a) {
    constexpr int WN = BN / 2, NJ = WN / 16, NIJ = 4 * NJ;
    const int M = a.N * a.Hq * a.Wq;
    const int mtiles = (M + BM - 1) / BM, tiles = mtiles * ((a.Co + BN - 1) / BN);
    const long long total = (long long)tiles * NIJ * 256;
    const f32x4* part = reinterpret_cast<const f32x4*>(a.partial);
    bool bad = false;
    for (long long u = blockIdx.x * (long long)blockDim.x + threadIdx.x; u < total; u += (long long)gridDim.x * blockDim.x) {
        const int tid = (int)(u & 255), ij = (int)((u >> 8) % NIJ), tile = (int)((u >> 8) / NIJ);
        const int bx = tile % mtiles, by = tile / mtiles, i = ij / NJ, j = ij % NJ;
        const int wid = tid >> 6, lane = tid & 63;
        const int n = by * BN + (wid & 1) * WN + 16 * j + (lane & 15);
        const int mb = bx * BM + (wid >> 1) * 64 + 16 * i + 4 * (lane >> 4);
        if (n >= a.Co || mb >= M) continue;
        f32x4 acc = part[u];
        for (int z = 1; z < a.ksplit; ++z) acc += part[(size_t)z * total + u];
        const float sc = a.scale[n], sh = a.shift[n];
        if (a.pool) {
            float x = fmaxf(fmaxf(acc[0] * sc + sh, acc[1] * sc + sh), fmaxf(acc[2] * sc + sh, acc[3] * sc + sh));
            if (a.act) x = x >= 0.f ? x : LRELU * x;
            const int p = mb >> 2, pw = a.Wq >> 1, phh = a.Hq >> 1;
            const int clip = p / (phh * pw), rr = p - clip * phh * pw;
            bad |= store_val<T>(a, clip * a.out_clip_stride + (long long)rr * a.out_pix_stride + a.out_c_off, n, x);
        } else {
            for (int r = 0; r < 4 && mb + r < M; ++r) {
                float x = acc[r] * sc + sh;
                if (a.act) x = x >= 0.f ? x : LRELU * x;
                const int m = mb + r, clip = m / (a.Hq * a.Wq), rr = m - clip * a.Hq * a.Wq;
                const int oy = (rr / a.Wq) * a.oys, ox = (rr % a.Wq) * a.oxs;
                bad |= store_val<T>(a, clip * a.out_clip_stride + (long long)(oy * a.Wo + ox) * a.out_pix_stride + a.out_c_off, n, x);
            }
        }
    }
    range_report(a.range_flag, a.range_bit, bad);
}

// video [N][128][128][F] f32 -> (x - mean) / std -> T [N][128][128][8] (channels F..7 zero; F <= 8)
template <typename T>
__global__ void k_video_prep(const float* __restrict__ v, const float* __restrict__ mean, const float* __restrict__ stdv,
                             T* __restrict__ out, long long npix, int F) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
        const int hw = (int)(p % (128 * 128));
        const float* src = v + p * F;
        float m = 0.f, s = 1.f;
        const bool norm = mean != nullptr;
        if (norm) { m = mean[hw]; s = stdv[hw]; }
        T o[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float x = c < F ? src[c] : 0.f;
            if (norm && c < F) x = (x - m) / s;
            o[c] = from_f<T>(x);
        }
        T* dst = out + p * 8;
#pragma unroll
        for (int c = 0; c < 8; ++c) dst[c] = o[c];
    }
}

// audio [N][80][T] f32 -> T [N][80][T][8] (channel 0 = value, 1..7 zero)
template <typename T>
__global__ void k_audio_prep(const float* __restrict__ a, T* __restrict__ out, long long npix) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
        T o[8];
        o[0] = from_f<T>(a[p]);
#pragma unroll
        for (int c = 1; c < 8; ++c) o[c] = from_f<T>(0.f);
        T* dst = out + p * 8;
#pragma unroll
        for (int c = 0; c < 8; ++c) dst[c] = o[c];
    }
}

// a_conv1 in the split dtype (network.py:89-91: Conv2D(64, 5x5, strides 2, 'same') on the one-channel mel image ->
// BatchNorm -> LeakyReLU), straight from the network input audio [N][H][W] f32 (no audio_prep copy): fp32 FMAs on the
// vector ALUs — the generic split k_conv spent 0.065 ms on its 2-slab K (K = 25) plus 0.012 ms of audio_prep; this
// kernel 0.040 ms.  A thread owns one output pixel and all 64 channels: the taps run in (ky, kx) order with fmaf (the
// loop not unrolled: unrolled, the compiler hoisted every weight read and the epilogue's loads over the FMAs — 256
// VGPRs and scratch; with the weights through scalar loads, 1,492 SGPR spills), each tap's input loaded three taps
// ahead, weights [tap][64] x 2^e_n and the folded BN scale x 2^-e_n / shift from LDS (exact), then LeakyReLU and the
// split pairs [h(16) | l(16)] x 4 as 16-B stores.  (Measured: 16 channels per thread, four waves per pixel block,
// 0.042 ms; eight lanes per pixel with lane-adjacent 16-B stores, 0.045 ms.)  The range guard reports input values
// past the pair range as before (range_in_bit: the recompute contract of include/avse.h) and stored pairs out of range.
struct AConv1Args {
    const float* in;          // [N][H][W]
    const float* w;           // [KH * KW][Co], x 2^e_n per output channel
    const float* scale;
    const float* shift;
    unsigned short* out;      // split pairs [N][Ho][Wo][Co / 16][h(16) | l(16)]
    long long N;
    int H, W, Ho, Wo, KH, KW, S, pt, pl;
    unsigned* range_flag;
    unsigned range_bit, range_in_bit;
};
constexpr int A1_CO = 64, A1_K = 5;
__global__ __launch_bounds__(256) void k_aconv1_split(AConv1Args a) {
    __shared__ __attribute__((aligned(16))) float ws[A1_K * A1_K * A1_CO];
    __shared__ __attribute__((aligned(16))) float ssc[A1_CO], ssh[A1_CO];
    for (int i = threadIdx.x; i < A1_K * A1_K * A1_CO / 4; i += 256)
        reinterpret_cast<float4*>(ws)[i] = reinterpret_cast<const float4*>(a.w)[i];
    if (threadIdx.x < A1_CO) {
        ssc[threadIdx.x] = a.scale[threadIdx.x];
        ssh[threadIdx.x] = a.shift[threadIdx.x];
    }
    __syncthreads();
    const int HW = a.Ho * a.Wo;
    const long long npix = a.N * HW;
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    bool bad = false, in_bad = false;
    if (p < npix) {
        const int clip = (int)(p / HW);   // (N x Ho x Wo < 2^31 checked at launch)
        const int r = (int)p - clip * HW, oy = r / a.Wo, ox = r - oy * a.Wo;
        const float* img = a.in + (long long)clip * a.H * a.W;
        auto tap_in = [&](int t) {
            const int ky = t / A1_K, kx = t - A1_K * (t / A1_K);
            const int iy = oy * a.S + ky - a.pt, ix = ox * a.S + kx - a.pl;
            const bool ok = t < A1_K * A1_K && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            return ok ? img[iy * a.W + ix] : 0.f;
        };
        float acc[A1_CO];
#pragma unroll
        for (int c = 0; c < A1_CO; ++c) acc[c] = 0.f;
        float v0 = tap_in(0), v1 = tap_in(1), v2 = tap_in(2);
#pragma unroll 1
        for (int t = 0; t < A1_K * A1_K; ++t) {
            const float v = v0;
            v0 = v1;
            v1 = v2;
            v2 = tap_in(t + 3);
            in_bad |= pair_out_of_range(v);
#pragma unroll
            for (int c = 0; c < A1_CO; c += 4) {
                const float4 w4 = *reinterpret_cast<const float4*>(ws + t * A1_CO + c);
                acc[c] = fmaf(v, w4.x, acc[c]);
                acc[c + 1] = fmaf(v, w4.y, acc[c + 1]);
                acc[c + 2] = fmaf(v, w4.z, acc[c + 2]);
                acc[c + 3] = fmaf(v, w4.w, acc[c + 3]);
            }
        }
        uint4* o = reinterpret_cast<uint4*>(a.out + p * A1_CO * 2);
#pragma unroll
        for (int g = 0; g < A1_CO / 16; ++g) {
            unsigned hw[8], lw[8];
#pragma unroll
            for (int c = 0; c < 16; c += 2) {
                const int n = 16 * g + c;
                float y0 = fmaf(acc[n], ssc[n], ssh[n]);
                float y1 = fmaf(acc[n + 1], ssc[n + 1], ssh[n + 1]);
                y0 = y0 >= 0.f ? y0 : 0.3f * y0;
                y1 = y1 >= 0.f ? y1 : 0.3f * y1;
                bad = bad || pair_out_of_range(y0) || pair_out_of_range(y1);
                const _Float16 h0 = (_Float16)y0, h1 = (_Float16)y1;
                const _Float16 l0 = (_Float16)(y0 - (float)h0), l1 = (_Float16)(y1 - (float)h1);
                hw[c / 2] = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
                lw[c / 2] = (unsigned)__builtin_bit_cast(unsigned short, l0) | ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
            }
            o[4 * g + 0] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            o[4 * g + 1] = make_uint4(hw[4], hw[5], hw[6], hw[7]);
            o[4 * g + 2] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
            o[4 * g + 3] = make_uint4(lw[4], lw[5], lw[6], lw[7]);
        }
    }
    range_report(a.range_flag, a.range_bit, bad);
    range_report(a.range_flag, a.range_in_bit, in_bad);
}

// d_deconv6 (network.py:133): 1x1 Conv2DTranspose 64 -> 1 + bias, no BN / activation.
template <typename T>
__global__ void k_out_conv(const T* __restrict__ in, const float* __restrict__ w, float bias, float* __restrict__ out,
                           long long npix) {
    __shared__ float ws[64];
    if (threadIdx.x < 64) ws[threadIdx.x] = w[threadIdx.x];
    __syncthreads();
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
        const T* src = in + p * 64;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < 64; ++c) acc = fmaf(to_f(src[c]), ws[c], acc);
        out[p] = acc + bias;
    }
}

__global__ void k_video_normalize(float* __restrict__ v, long long S, int H, int W, int F, const float* __restrict__ mean,
                                  const float* __restrict__ stdv) {
    const long long total = S * H * W * F;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const int hw = (int)((i / F) % ((long long)H * W));
        v[i] = (v[i] - mean[hw]) / stdv[hw];
    }
}

// deterministic two-pass mean((a-b)^2)
__global__ void k_mse_partial(const float* __restrict__ a, const float* __restrict__ b, long long n, float* partial) {
    __shared__ float red[4];
    float s = 0.f;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float d = a[i] - b[i];
        s = fmaf(d, d, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void k_mse_final(const float* __restrict__ partial, int np, long long n, float* loss) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < np; i += blockDim.x) s += partial[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *loss = (float)(((double)red[0] + red[1] + red[2] + red[3]) / (double)n);
}

inline unsigned grid_for(long long n, int block) {
    long long g = (n + block - 1) / block;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

int launch_conv(const ConvArgs& a, int dtype, hipStream_t s) {
    const int M = a.N * a.Hq * a.Wq;
    // short grids (< 256 tiles of 128 x 128) take 64-column tiles: twice the workgroups, and every output keeps its
    // summation order (the K loop is per fragment), so results are bitwise equal (batch-16 training step 6.56 -> 5.90
    // ms).  Not with split-K, whose reduction is planned on 128-column tiles, nor the fused d_deconv6 tail.  Split
    // pairs: up to 256 tiles (v_conv6 at N = 512: one 128-column workgroup per CU, 0.171 -> 0.161 ms with 64 columns;
    // a 512-tile bound also moved a_conv3 / d_deconv3, both slower)
    const long long tiles128 = (long long)((M + BM - 1) / BM) * ((a.Co + 127) / 128);
    const long long short_grid = dtype == kConvSplitPairs ? 257 : 256;
    const int BN = (a.Co <= 64 || (a.ksplit == 1 && !a.fuse_w && tiles128 < short_grid)) ? 64 : 128;
    if (a.ksplit < 1 || (a.ksplit > 1 && (a.nphase != 1 || !a.partial))) {
        set_error("bad split-K configuration");
        return 1;
    }
    if (a.fuse_w && (a.Co != 64 || a.ksplit != 1 || a.pool || !a.fuse_out)) {
        set_error("k_conv: fused 1x1 tail needs Co == 64, no split-K, no pool");
        return 1;
    }
    for (int p = 0; p < a.nphase; ++p)
        if (a.ph[p].ntaps > MAX_TAPS_LDS) {
            set_error("k_conv: too many taps in one phase");
            return 3;
        }
    dim3 grid((M + BM - 1) / BM, (a.Co + BN - 1) / BN, a.nphase * a.ksplit);
    const bool fast = a.Ci % ((dtype == 1 || dtype == kConvSplitPairs) ? 32 : 16) == 0;   // else the per-slab tap decode
    if (dtype == kConvSplitPairs) {
        if (fast) {
            if (BN == 64) hipLaunchKernelGGL((k_conv<_Float16, 64, true, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<_Float16, 128, true, true>), grid, dim3(256), 0, s, a);
        } else {
            if (BN == 64) hipLaunchKernelGGL((k_conv<_Float16, 64, false, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<_Float16, 128, false, true>), grid, dim3(256), 0, s, a);
        }
    } else if (dtype == kConvSplit) {
        if (fast) {
            if (BN == 64) hipLaunchKernelGGL((k_conv<float, 64, true, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<float, 128, true, true>), grid, dim3(256), 0, s, a);
        } else {
            if (BN == 64) hipLaunchKernelGGL((k_conv<float, 64, false, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<float, 128, false, true>), grid, dim3(256), 0, s, a);
        }
    } else if (dtype == 1) {
        if (fast) {
            if (BN == 64) hipLaunchKernelGGL((k_conv<bf16_t, 64, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<bf16_t, 128, true>), grid, dim3(256), 0, s, a);
        } else {
            if (BN == 64) hipLaunchKernelGGL((k_conv<bf16_t, 64, false>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<bf16_t, 128, false>), grid, dim3(256), 0, s, a);
        }
    } else {
        if (fast) {
            if (BN == 64) hipLaunchKernelGGL((k_conv<float, 64, true>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<float, 128, true>), grid, dim3(256), 0, s, a);
        } else {
            if (BN == 64) hipLaunchKernelGGL((k_conv<float, 64, false>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_conv<float, 128, false>), grid, dim3(256), 0, s, a);
        }
    }
    AVSE_HIP_CHECK(hipGetLastError());
    if (a.ksplit > 1) {
        const long long units = (long long)grid.x * grid.y * (BN / 2 / 16 * 4) * 256;
        const dim3 rg(grid_for(units, 256));
        if (dtype == 1) {
            if (BN == 64) hipLaunchKernelGGL((k_splitk_reduce_tiles<bf16_t, 64>), rg, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_splitk_reduce_tiles<bf16_t, 128>), rg, dim3(256), 0, s, a);
        } else {
            if (BN == 64) hipLaunchKernelGGL((k_splitk_reduce_tiles<float, 64>), rg, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_splitk_reduce_tiles<float, 128>), rg, dim3(256), 0, s, a);
        }
        AVSE_HIP_CHECK(hipGetLastError());
    }
    return 0;
}

// dst[r * stride + j] = src[j] for r < rows, j < row_bytes (16-B units when every address and size allows)
__global__ void k_broadcast_row(const char* __restrict__ src, char* __restrict__ dst, long long rows, long long row_bytes,
                                long long stride, int vec) {
    const long long units = row_bytes / vec, total = rows * units;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / units, j = (i - r * units) * vec;
        if (vec == 16) *reinterpret_cast<i32x4*>(dst + r * stride + j) = *reinterpret_cast<const i32x4*>(src + j);
        else dst[r * stride + j] = src[j];
    }
}

// range guard of a forward whose cached all-zero-video embedding was out of the pair range (capi.hip)
__global__ void k_flag_or(unsigned* flag, unsigned bits) {
    if (threadIdx.x == 0) atomicOr(flag, bits);
}

int launch_flag_or(unsigned* flag, unsigned bits, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_or, dim3(1), dim3(64), 0, s, flag, bits);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_broadcast_row(const void* src, void* dst, int64_t rows, int64_t row_bytes, int64_t stride_bytes, hipStream_t s) {
    const bool v16 = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0) && row_bytes % 16 == 0 && stride_bytes % 16 == 0;
    const int vec = v16 ? 16 : 1;
    hipLaunchKernelGGL(k_broadcast_row, dim3(grid_for(rows * (row_bytes / vec), 256)), dim3(256), 0, s, (const char*)src,
                       (char*)dst, (long long)rows, (long long)row_bytes, (long long)stride_bytes, vec);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_video_prep(const float* video, const float* mean, const float* stdv, void* out, int64_t N, int F, int dtype,
                      hipStream_t s) {
    const long long npix = (long long)N * 128 * 128;
    if (F < 1 || F > 8) { set_error("video frames per slice must be 1..8"); return 1; }
    if (dtype == 1) hipLaunchKernelGGL(k_video_prep<bf16_t>, dim3(grid_for(npix, 256)), dim3(256), 0, s, video, mean, stdv, (bf16_t*)out, npix, F);
    else hipLaunchKernelGGL(k_video_prep<float>, dim3(grid_for(npix, 256)), dim3(256), 0, s, video, mean, stdv, (float*)out, npix, F);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_audio_prep(const float* audio, void* out, int64_t npix, int dtype, hipStream_t s) {
    if (dtype == 1) hipLaunchKernelGGL(k_audio_prep<bf16_t>, dim3(grid_for(npix, 256)), dim3(256), 0, s, audio, (bf16_t*)out, npix);
    else hipLaunchKernelGGL(k_audio_prep<float>, dim3(grid_for(npix, 256)), dim3(256), 0, s, audio, (float*)out, npix);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_aconv1_split(const float* in, const float* w, const float* scale, const float* shift, void* out, int64_t N,
                        int H, int W, int Ho, int Wo, int KH, int KW, int S, int pt, int pl, int Co, unsigned* range_flag,
                        unsigned range_bit, unsigned range_in_bit, hipStream_t s) {
    if (Co != A1_CO || KH != A1_K || KW != A1_K || !w || N <= 0 || N * Ho * Wo >= (1LL << 31)) {
        set_error("a_conv1 split kernel: unexpected layer shape");
        return 3;
    }
    AConv1Args a{in, w, scale, shift, (unsigned short*)out, (long long)N, H, W, Ho, Wo, KH, KW, S, pt, pl,
                 range_flag, range_bit, range_in_bit};
    const long long npix = N * Ho * Wo;
    hipLaunchKernelGGL(k_aconv1_split, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_out_conv(const void* in, const float* w64, float bias, float* out, int64_t npix, int dtype, hipStream_t s) {
    if (dtype == 1) hipLaunchKernelGGL(k_out_conv<bf16_t>, dim3(grid_for(npix, 256)), dim3(256), 0, s, (const bf16_t*)in, w64, bias, out, (long long)npix);
    else hipLaunchKernelGGL(k_out_conv<float>, dim3(grid_for(npix, 256)), dim3(256), 0, s, (const float*)in, w64, bias, out, (long long)npix);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_video_normalize(float* video, int64_t S, int H, int W, int F, const float* mean, const float* stdv,
                           hipStream_t s) {
    const long long total = (long long)S * H * W * F;
    hipLaunchKernelGGL(k_video_normalize, dim3(grid_for(total, 256)), dim3(256), 0, s, video, (long long)S, H, W, F, mean, stdv);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_mse(const float* a, const float* b, int64_t n, float* loss, float* partial, hipStream_t s) {
    const int np = 256;
    hipLaunchKernelGGL(k_mse_partial, dim3(np), dim3(256), 0, s, a, b, (long long)n, partial);
    AVSE_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_mse_final, dim3(1), dim3(256), 0, s, partial, np, (long long)n, loss);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
