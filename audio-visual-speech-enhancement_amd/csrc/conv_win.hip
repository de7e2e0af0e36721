// Windowed split-pair convolution for the AVSE_F32_SPLIT layers whose every phase is a stride-1 gather over the input
// grid: d_deconv3 / d_deconv4 / d_deconv5 (Conv2DTranspose, network.py:121-133, as sub-pixel phases; d_deconv5 with
// d_deconv6, network.py:133, fused) and a_conv2 (Conv2D 4x4 stride 1 'same', network.py:93).
//
// k_conv (conv.hip) gathers each K slab's A rows (one tap x 16 channels of 128 output pixels) from global memory: a
// pixel's input is re-read once per tap (16 taps: 1.68 GB of A per d_deconv4 launch for a 105 MB input), and the 128-row
// tiles re-read the layer's weights once per tile (819 MB) — 41 % of k_conv's time at d_deconv4's shape is its global
// loads (tools/kconv_ablate.hip).  Here a 256-row tile (4 waves of 64 rows x all 64 output channels of its column
// block) stages, per 16-channel pair chunk, the input window its rows need for every tap in LDS once; the tap loop reads
// A fragments from the window at a per-lane pixel base plus a wave-uniform tap offset.  Weights stream through a 3-slab
// LDS ring as in k_conv (4 KB per 64-channel slab), at half k_conv's bytes per output row.  K order: chunk-outer,
// tap-inner; the arithmetic is k_conv's S16 pair form (two v_mfma_f32_16x16x32_f16 per slab: Ah Bh + Al Bh, Ah Bl +
// Al Bl) with the same fp32 blocked summation (8-slab blocks), in another K order (results equal k_conv's within fp32
// rounding, and per output row independent of the batch: no split-K).
//
// Window geometry (per tile and phase): the tile's rows m0 .. m0 + 255 (row-major over clip, yq, xq of the phase's
// output grid = the input grid Hi x Wi) cover clips c0 .. c1; region r (clip c0 + r, its rows ylo_r .. yhi_r) takes
// window rows wrow0_r .. + (yhi_r - ylo_r + spany - 1), window row w of the region holding input row ylo_r + dymin + w,
// window column v input column v + dxmin; rows / columns outside the image are zero (TF 'SAME' padding, transposed-conv
// crops).  Output row (y, x) at tap (dy, dx) reads window pixel (wrow0_r + y - ylo_r + dy - dymin) * WP + x + dx - dxmin.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "avse_common.h"

namespace avse {
namespace {

// tile rows: TM = 64 WGM (WGM waves along M, 4 / WGM along the 64 columns of the column block; a wave holds 64 rows x
// 64 / (4 / WGM) columns).  TM 128 (2 x 2 waves, three workgroups per CU) measured faster than TM 256 (4 x 1, two per
// CU): d_deconv4 0.258 ms (TM 256) vs k_conv's 0.244
#ifndef AVSE_WIN_WGM
#define AVSE_WIN_WGM 2
#endif
constexpr int WGM = AVSE_WIN_WGM, WN = 4 / WGM, NJ = 4 / WN;
constexpr int TM = 64 * WGM, BN = 64, NTH = 256;
constexpr int WIN_BYTES = WGM == 4 ? 32 * 1024 : 20 * 1024;   // one chunk's window (64 B per pixel: 16 channel pairs)
constexpr int NPIECE = WIN_BYTES / 16 / NTH;         // 16-B pieces per thread per window
constexpr int BSL = BN * 64;                         // one K slab of weights: 64 channels x 16 channel pairs
constexpr int LDS_BYTES = 2 * WIN_BYTES + 3 * BSL;   // 52 KB (TM 128: three workgroups per CU) / 76 KB (TM 256: two)
static_assert(WIN_BYTES % (16 * NTH) == 0, "whole pieces per thread");
constexpr int MAXREG = 8;                            // clips per tile (host-checked)
constexpr int MAXTAP = 32;
constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;

struct WinPhase {
    int dymin, dxmin;    // the phase's smallest tap offsets
    int spany;           // dymax - dymin + 1
    // the taps form a grid (host-checked): tap t = (dy0 + sy (t / nx), dx0 + sx (t % nx)), so the window byte offset
    // of tap t steps by sx 64 within a row and by sy WP 64 - sx nx 64 at a row end
    int toff0, nx, xstep, rowstep;
};
struct WinArgs {
    int WP;              // window pitch (pixels)
    WinPhase ph[MAX_PHASES];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ int bswz(int row) { return ((row >> 3) & 1) * 3; }   // k_conv's B-slab swizzle

template <bool FUSE>
__global__ __launch_bounds__(NTH, WGM == 2 ? 3 : 2) void k_conv_win(ConvArgs a, WinArgs g) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char* const win = lds;                   // [2][WIN_BYTES]
    char* const bs = lds + 2 * WIN_BYTES;    // [3][BSL]

    const int tid = threadIdx.x, lane = tid & 63, wm = (tid >> 6) % WGM, wn = (tid >> 6) / WGM;
    const int fr = lane & 15, fg = lane >> 4;
    const ConvPhase ph = a.ph[blockIdx.z];
    const WinPhase wph = g.ph[blockIdx.z];
    const int WP = g.WP;
    const int HW = a.Hq * a.Wq, M = a.N * HW;
    const int m0 = blockIdx.x * TM, n0 = blockIdx.y * BN;
    const int CIH = a.Ci;                     // halves per input pixel (the split pair layout)
    const int nch = CIH / 32, ntap = ph.ntaps, NS = nch * ntap;

    // ---- the tile's regions (wave-uniform) ----
    const int c0 = m0 / HW, last = min(m0 + TM, M) - 1, c1 = last / HW, nreg = c1 - c0 + 1;
    int ylo[MAXREG], wrow0[MAXREG], wtot = 0;   // (indexed with compile-time indices only: no scratch)
#pragma unroll
    for (int r = 0; r < MAXREG; ++r) {
        const int lo = r == 0 ? (m0 - c0 * HW) / a.Wq : 0;
        const int hi = r == nreg - 1 ? (last - c1 * HW) / a.Wq : a.Hq - 1;
        ylo[r] = lo;
        wrow0[r] = wtot;
        if (r < nreg) wtot += hi - lo + wph.spany;
    }
    const long long clip_b = a.in_clip_stride * 2;
    const __amdgpu_buffer_rsrc_t rsA = make_rsrc(reinterpret_cast<const char*>(a.in) + c0 * clip_b, (a.N - c0) * clip_b);
    const __amdgpu_buffer_rsrc_t rsB = make_rsrc(reinterpret_cast<const char*>(a.w) + ph.w_off * 2,
                                                 (long long)a.Co * ph.kpad * 2);

    // ---- window pieces of this thread: source offset for chunk 0 (kOOB: padding, reads zero) ----
    int psrc[NPIECE];
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) {
        const int q = tid + NTH * k, p = q >> 2, qq = q & 3;
        const int wrow = p / WP, wcol = p - wrow * WP;
        int src = kOOB;
        if (wrow < wtot) {
            int r = 0, yl = ylo[0], w0 = 0;   // the region: the last one whose first window row is <= wrow
#pragma unroll
            for (int rr = 1; rr < MAXREG; ++rr)
                if (rr < nreg && wrow >= wrow0[rr]) { r = rr; yl = ylo[rr]; w0 = wrow0[rr]; }
            const int iy = yl + wph.dymin + (wrow - w0), ix = wcol + wph.dxmin;
            if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi)
                src = (int)(r * clip_b + ((long long)(iy * a.Wi + ix) * CIH + qq * 8) * 2);
        }
        psrc[k] = src;
    }
    // ---- A fragment bases: window pixel of the lane's row at tap offset (dymin, dxmin) ----
    int abase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = min(m0 + wm * 64 + 16 * i + fr, M - 1);
        const int c = m / HW, pp = m - c * HW, y = pp / a.Wq, x = pp - y * a.Wq;
        const int r = c - c0;
        int wr0 = 0, yl = 0;
#pragma unroll
        for (int rr = 0; rr < MAXREG; ++rr)
            if (rr == r) { wr0 = wrow0[rr]; yl = ylo[rr]; }
        abase[i] = ((wr0 + y - yl) * WP + x) * 64 + fg * 16;
    }
    // ---- B: the thread's 16-B piece of a slab (row tid >> 2, quarter tid & 3) ----
    const int brow = tid >> 2, bq = tid & 3;
    const int bsrc = n0 + brow < a.Co ? ((n0 + brow) * ph.kpad) * 2 + bq * 16 : kOOB;
    const int bdst = brow * 64 + ((bq ^ bswz(brow)) << 4);
    // B slab s's offset (chunk-outer, tap-inner): t CIH 2 + c 64; the prologue's slabs 0..3, then stepped per slab
    auto bslab_off = [&](int s) {
        const int c = s / ntap, t = s - c * ntap;
        return t * CIH * 2 + c * 64;
    };
    int bt = 4 % ntap, bc = 4 / ntap;   // (tap, chunk) of slab s + 4 at step s

    // epilogue parameters (loaded before the K loop)
    float esc[NJ], esh[NJ], ewf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * 16 * NJ + 16 * j + fr;
        const bool ok = n < a.Co;
        esc[j] = ok ? a.scale[n] : 0.f;
        esh[j] = ok ? a.shift[n] : 0.f;
        ewf[j] = (FUSE && ok) ? a.fuse_w[n] : 0.f;
    }

    // ---- prologue: window of chunk 0, B slabs 0 .. 2 in flight, slab 0 in LDS ----
    {
        i32x4 pc[NPIECE];
#pragma unroll
        for (int k = 0; k < NPIECE; ++k) pc[k] = __builtin_amdgcn_raw_buffer_load_b128(rsA, psrc[k], 0, 0);
#pragma unroll
        for (int k = 0; k < NPIECE; ++k) *reinterpret_cast<i32x4*>(win + (tid + NTH * k) * 16) = pc[k];
    }
    i32x4 rb[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) rb[p] = __builtin_amdgcn_raw_buffer_load_b128(rsB, p < NS ? bsrc : kOOB, p < NS ? bslab_off(p) : 0, 0);
    *reinterpret_cast<i32x4*>(bs + bdst) = rb[0];
    rb[0] = __builtin_amdgcn_raw_buffer_load_b128(rsB, 3 < NS ? bsrc : kOOB, 3 < NS ? bslab_off(3) : 0, 0);
    __syncthreads();

    f32x4 acc[4][NJ], part[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int nblk = 0;
    i32x4 pw[NPIECE];   // the next chunk's window pieces
    int c = 0, t = 0, tx = 0;        // chunk / tap of slab s, tap column
    int toff = wph.toff0;            // window byte offset of tap t
    auto step = [&](auto qidx, int s) {
        constexpr int q = decltype(qidx)::value, qn = (q + 1) % 3;
        if (t == 0 && c + 1 < nch) {
#pragma unroll
            for (int k = 0; k < NPIECE; ++k) pw[k] = __builtin_amdgcn_raw_buffer_load_b128(rsA, psrc[k], (c + 1) * 64, 0);
        }
        const char* wb = win + (c & 1) * WIN_BYTES + toff;
        i32x4 fa[4], fb[NJ], fl[NJ];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const i32x4*>(wb + abase[i]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = wn * 16 * NJ + 16 * j + fr;
            fb[j] = *reinterpret_cast<const i32x4*>(bs + q * BSL + row * 64 + (((fg & 1) ^ bswz(row)) << 4));
            fl[j] = *reinterpret_cast<const i32x4*>(bs + q * BSL + row * 64 + (((2 + (fg & 1)) ^ bswz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa[i]),
                                                                    __builtin_bit_cast(f16x8, fb[j]), part[i][j], 0, 0, 0);
                part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa[i]),
                                                                    __builtin_bit_cast(f16x8, fl[j]), part[i][j], 0, 0, 0);
            }
        if (++nblk == kFp32Block) {
            nblk = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    acc[i][j] += part[i][j];
                    part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
                }
        }
        // B slab s + 1 -> slot qn (it held slab s - 2, read before the barrier of step s - 2); refill with slab s + 4
        *reinterpret_cast<i32x4*>(bs + qn * BSL + bdst) = rb[qn];
        rb[qn] = __builtin_amdgcn_raw_buffer_load_b128(rsB, s + 4 < NS ? bsrc : kOOB, bt * CIH * 2 + bc * 64, 0);
        if (++bt == ntap) {
            bt = 0;
            ++bc;
        }
        if (t == ntap - 1 && c + 1 < nch) {
            // the next chunk's window -> the other buffer (last read during chunk c - 1, before this chunk's first barrier)
#pragma unroll
            for (int k = 0; k < NPIECE; ++k)
                *reinterpret_cast<i32x4*>(win + ((c + 1) & 1) * WIN_BYTES + (tid + NTH * k) * 16) = pw[k];
        }
        if (++t == ntap) {
            t = 0;
            tx = 0;
            ++c;
            toff = wph.toff0;
        } else if (++tx == wph.nx) {
            tx = 0;
            toff += wph.rowstep;
        } else {
            toff += wph.xstep;
        }
        __syncthreads();
    };
    for (int s = 0; s < NS; s += 3) {
        step(std::integral_constant<int, 0>{}, s);
        if (s + 1 < NS) step(std::integral_constant<int, 1>{}, s + 1);
        if (s + 2 < NS) step(std::integral_constant<int, 2>{}, s + 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] += part[i][j];

    // ---- epilogue: bias + BN (scale / shift), LeakyReLU, the split pair store or the fused 64 -> 1 output dot ----
    long long orow[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * 64 + 16 * i + 4 * fg + r;
            const int cl = m / HW, pp = m - cl * HW, yq = pp / a.Wq, xq = pp - yq * a.Wq;
            const int oy = yq * a.oys + ph.py, ox = xq * a.oxs + ph.px;
            orow[i][r] = m < M ? cl * a.out_clip_stride + (long long)(oy * a.Wo + ox) * a.out_pix_stride + a.out_c_off : -1;
        }
    if constexpr (FUSE) {
        // d_deconv6 (network.py:133): out[pixel] = bias + sum over the 64 channels (the tile's column block: all of
        // them) of w6[c] y[c]: the wave's NJ channels per lane in-lane, over the 16 lanes of a row group (DPP row_ror 8,
        // 4, 2, 1), then over the WN column halves through LDS in a fixed order (the window memory: the K loop ended on
        // a barrier)
        float v[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x0 = 0.f;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    float x = acc[i][j][r] * esc[j] + esh[j];
                    x = x >= 0.f ? x : LRELU * x;
                    x0 = fmaf(x, ewf[j], x0);
                }
                x0 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x0), 0x128, 0xf, 0xf, false));
                x0 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x0), 0x124, 0xf, 0xf, false));
                x0 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x0), 0x122, 0xf, 0xf, false));
                x0 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x0), 0x121, 0xf, 0xf, false));
                v[i][r] = x0;
            }
        if constexpr (WN > 1) {
            float* red = reinterpret_cast<float*>(lds);
            if (wn == 1 && fr == 0)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) red[wm * 64 + 16 * i + 4 * fg + r] = v[i][r];
            __syncthreads();
            if (wn == 1) return;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[i][r] += red[wm * 64 + 16 * i + 4 * fg + r];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (fr == 0 && orow[i][r] >= 0) a.fuse_out[orow[i][r]] = v[i][r] + a.fuse_bias;
        return;
    }
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * 16 * NJ + 16 * j + fr;
        if (n >= a.Co) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (orow[i][r] < 0) continue;
                float x = acc[i][j][r] * esc[j] + esh[j];
                x = x >= 0.f ? x : LRELU * x;
                _Float16* o = reinterpret_cast<_Float16*>(a.out) + orow[i][r] + 32 * (n >> 4) + (n & 15);
                const _Float16 h = (_Float16)x;
                o[0] = h;
                o[16] = (_Float16)(x - (float)h);
                bad |= pair_out_of_range(x);
            }
    }
    range_report(a.range_flag, a.range_bit, bad);
}

}  // namespace

int launch_conv_win(const ConvArgs& a, const int2* htaps, hipStream_t s) {
    // what the kernel implements: split pairs in and out (or the fused d_deconv6 tail), every phase a stride-1 gather
    // over an input grid equal to its output grid, no pooling / split-K, whole 16-channel pair chunks, Co a multiple of 64
    if (a.ksplit != 1 || a.pool || a.sy != 1 || a.sx != 1 || a.Hq != a.Hi || a.Wq != a.Wi || a.Ci % 32 || a.Co % BN ||
        (!a.out_s16 && !a.fuse_w) || (a.fuse_w && (a.Co != BN || !a.fuse_out)))
        return -1;
    // where it is faster (A/B in the forward, one box, round 5): single-phase 16-tap layers — d_deconv4 0.244 -> 0.233
    // ms, a_conv2 0.135 -> 0.133; the multi-phase layers with 4-9 taps per phase (d_deconv1..3, d_deconv5) ran 5-10 %
    // slower than k_conv (short K loops per tile: the window prologue per chunk and the epilogue are not amortised)
    if (a.nphase != 1 || a.ph[0].ntaps < 16) return -1;
    WinArgs g;
    std::memset(&g, 0, sizeof(g));
    const int HW = a.Hq * a.Wq;
    int span_x = 1;
    for (int p = 0; p < a.nphase; ++p) {
        const ConvPhase& ph = a.ph[p];
        if (ph.ntaps < 1 || ph.ntaps > MAXTAP || ph.kpad != ph.ntaps * a.Ci) return -1;
        int y0 = 1 << 20, y1 = -(1 << 20), x0 = 1 << 20, x1 = -(1 << 20);
        for (int t = 0; t < ph.ntaps; ++t) {
            const int2 d = htaps[ph.tap_off + t];
            y0 = std::min(y0, d.x); y1 = std::max(y1, d.x);
            x0 = std::min(x0, d.y); x1 = std::max(x1, d.y);
        }
        g.ph[p].dymin = y0;
        g.ph[p].dxmin = x0;
        g.ph[p].spany = y1 - y0 + 1;
        span_x = std::max(span_x, x1 - x0 + 1);
    }
    g.WP = a.Wi + span_x - 1;   // a phase's window columns run from its own dxmin: Wi + its x span - 1 <= WP
    // the tap grid of each phase: nx taps per row, steps sx / sy of +-1 (checked tap by tap)
    for (int p = 0; p < a.nphase; ++p) {
        const ConvPhase& ph = a.ph[p];
        const int2* tp = htaps + ph.tap_off;
        int nx = 1;
        while (nx < ph.ntaps && tp[nx].x == tp[0].x) ++nx;
        if (ph.ntaps % nx) return -1;
        const int sx = nx > 1 ? tp[1].y - tp[0].y : 1, sy = ph.ntaps > nx ? tp[nx].x - tp[0].x : 1;
        if ((sx != 1 && sx != -1) || (sy != 1 && sy != -1)) return -1;
        for (int t = 0; t < ph.ntaps; ++t)
            if (tp[t].x != tp[0].x + sy * (t / nx) || tp[t].y != tp[0].y + sx * (t % nx)) return -1;
        WinPhase& w = g.ph[p];
        w.toff0 = ((tp[0].x - w.dymin) * g.WP + (tp[0].y - w.dxmin)) * 64;
        w.nx = nx;
        w.xstep = sx * 64;
        w.rowstep = sy * g.WP * 64 - sx * (nx - 1) * 64;
    }
    // worst-case window of a tile: its rows span at most TM / Wq + 1 image rows, over at most TM / HW + 2 clips, each
    // region spany - 1 rows more
    const int maxreg = TM / HW + 2;
    if (maxreg > MAXREG) return -1;
    for (int p = 0; p < a.nphase; ++p) {
        const int rows = std::min(TM / a.Wq + 2, maxreg * a.Hq) + maxreg * (g.ph[p].spany - 1);
        if ((long long)rows * g.WP * 64 > WIN_BYTES) return -1;
    }
    if (int rc = ensure_lds_attr(a.fuse_w ? (const void*)k_conv_win<true> : (const void*)k_conv_win<false>, LDS_BYTES))
        return rc;
    const int M = a.N * HW;
    const dim3 grid((M + TM - 1) / TM, a.Co / BN, a.nphase);
    if (a.fuse_w) hipLaunchKernelGGL(k_conv_win<true>, grid, dim3(NTH), LDS_BYTES, s, a, g);
    else hipLaunchKernelGGL(k_conv_win<false>, grid, dim3(NTH), LDS_BYTES, s, a, g);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
