// One Keras training step of the reference network, fp32, gfx950 — SpeechEnhancementNetwork.train
// (/root/reference/network.py:177-206: Model.fit with batch_size 16 on the model compiled at network.py:35-36 with
// optimizers.adam(lr=5e-4) and loss='mean_squared_error').
//
// Keras 2.0 training-mode semantics restated here (oracle/keras_train_ref.py restates the same in float64 autograd):
//   * BatchNormalization (eps 1e-3, momentum 0.99): normalises with the BATCH mean and biased variance over every
//     axis but the channel, and updates moving_mean / moving_variance <- m * 0.99 + batch * 0.01;
//   * LeakyReLU(0.3); MaxPooling2D(2, 2, 'same') on even grids (the gradient goes to the window's first maximum);
//   * Dropout(0.25) after each video pooling (network.py:142-174): kept values scaled by 1 / 0.75.  The mask comes
//     from a counter-based hash of (seed, layer, element) — reproducible, so the oracle can apply the same mask;
//   * loss = mean((y - t)^2) over every element; Adam (Keras 2.0: beta1 0.9, beta2 0.999, epsilon 1e-8,
//     lr_t = lr sqrt(1 - beta2^t) / (1 - beta1^t)).
//
// Device work per step (N clips):
//   forward   per layer: k_conv (fp32 MFMA implicit GEMM, conv.hip) with bias only -> z; column mean, then
//             column sum of squared deviations (two passes, double finish) -> batch stats + moving-average update;
//             k_act_fwd: BN + LeakyReLU [+ 2x2 max pool + dropout] -> the next layer's input (the concat buffer
//             for a_conv5 / v_conv6)
//   loss      k_mse: loss and dL/dy
//   backward  per layer, reverse: k_act_bwd (dropout, pool routing, LeakyReLU') -> dL/d(BN output);
//             column sums of g and g * xhat -> dgamma, dbeta; k_bn_bwd -> dz; column sum of dz -> dbias;
//             k_wgrad (LDS-tiled reduction over the batch's pixels, deterministic split + ordered reduce) -> dW;
//             k_conv on repacked weights -> dL/dx (strided convs as multi-phase gathers, transposed convs as strided
//             convs, dense as a GEMM with the Keras (in, out) matrix)
//   update    k_adam over the whole canonical parameter blob (moving statistics carry zero gradient: unchanged)
// Parameters, gradients and Adam moments live in the canonical blob layout (include/avse.h avse_weights_load), so
// export is a copy; forward / dgrad weight packings are written from it each step by k_pack, whose 64 x 64 tile
// list is built once on the host and checked there against the element-wise index maps.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/avse.h"
#include "avse_common.h"
#include "netplan.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr float BN_MOMENTUM = 0.99f;

__host__ __device__ inline uint32_t drop_hash(uint32_t seed, uint32_t layer, uint32_t idx) {
    uint32_t h = idx * 0x9E3779B1u ^ (seed * 0x85EBCA77u + layer * 0xC2B2AE3Du);
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}

inline unsigned grid_for(long long n, int block = 256, long long cap = 8192) {
    long long g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// One <= 64 x 64 tile of a weight packing: dst[which][dst + r dld + c] = P[src + r sr + c sc].  Every (layer, phase,
// tap) block of a packing is a strided 2-D view of the Keras kernel: a transpose (sr == 1: conv / dense forward,
// deconv dgrad) or a row copy (sc == 1).  The tile is read along the unit-stride axis, turned in LDS and written
// along dst rows, so both sides are coalesced (the index-map gather of round 2 read 4-byte words at a stride of
// cout: ~0.2 ms per batch-16 step).
struct PackTile {
    long long dst, src;
    int R, C, dld, sr, sc, which;
};

__global__ __launch_bounds__(256) void k_pack(float* __restrict__ wfwd, float* __restrict__ wdg, const float* __restrict__ P,
                                              const PackTile* __restrict__ tiles) {
    __shared__ float tile[64][65];
    const PackTile T = tiles[blockIdx.x];
    const int lo = threadIdx.x & 63, hi = threadIdx.x >> 6;
    if (T.sr == 1) {
        if (lo < T.R)
            for (int c = hi; c < T.C; c += 4) tile[lo][c] = P[T.src + lo + (long long)c * T.sc];
    } else if (lo < T.C) {
        for (int r = hi; r < T.R; r += 4) tile[r][lo] = P[T.src + (long long)r * T.sr + (long long)lo * T.sc];
    }
    __syncthreads();
    float* __restrict__ dst = T.which ? wdg : wfwd;
    if (lo < T.C)
        for (int r = hi; r < T.R; r += 4) dst[T.dst + (long long)r * T.dld + lo] = tile[r][lo];
}

// video [N][128][128][F] -> (x - mean) / std (VideoNormalizer, data_processor.py:208-212) -> [N][128][128][8]
__global__ void k_prep_video(const float* __restrict__ v, const float* __restrict__ mean, const float* __restrict__ stdv,
                             float* __restrict__ out, long long npix, int hw, int F) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
        const int q = (int)(p % hw);
        const float m = mean ? mean[q] : 0.f, s = stdv ? stdv[q] : 1.f;
        float o[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c] = c >= F ? 0.f : mean ? (v[p * F + c] - m) / s : v[p * F + c];
        float4* d = reinterpret_cast<float4*>(out + p * 8);
        d[0] = make_float4(o[0], o[1], o[2], o[3]);
        d[1] = make_float4(o[4], o[5], o[6], o[7]);
    }
}

// audio [N][80][T] -> [N][80][T][8] (expand_dims(-1), network.py:181, channel padded to the 8-wide chunk)
__global__ void k_prep_audio(const float* __restrict__ a, float* __restrict__ out, long long npix) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
        float4* d = reinterpret_cast<float4*>(out + p * 8);
        d[0] = make_float4(a[p], 0.f, 0.f, 0.f);
        d[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// Column reductions over the rows of a [M][ld] matrix (first C columns), one partial per row block:
//   MODE 0: sum x                       (means, bias gradients)
//   MODE 2: sum g, sum g * xhat         (BN backward; xhat = (z - mean) * inv from z)
//   MODE 3: per block: sum x (= MODE 0's partial) and sum (x - block mean)^2 (BN forward statistics in one launch)
// grid (ceil(C / 64), nblk), 256 threads = 64 columns x 4 row groups.
template <int MODE>
__global__ __launch_bounds__(256) void k_colreduce(const float* __restrict__ x, int ld, const float* __restrict__ z,
                                                   const float* __restrict__ mean, const float* __restrict__ inv,
                                                   long long M, int C, long long rows_per_blk, float* __restrict__ part) {
    __shared__ float s0[4][64], s1[4][64];
    const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
    const int c = blockIdx.x * 64 + cl;
    const long long r0 = blockIdx.y * rows_per_blk, r1 = min(M, r0 + rows_per_blk);
    float a0 = 0.f, a1 = 0.f;
    if (MODE == 3) {   // this block's sum (exactly MODE 0's partial), its mean, then the squared deviations about it
        if (c < C)
            for (long long g = r0 + rg; g < r1; g += 256) {
                float p0 = 0.f;
                const long long ge = min(r1, g + 256);
                for (long long r = g; r < ge; r += 4) p0 += x[r * ld + c];
                a0 += p0;
            }
        s0[rg][cl] = a0;
        __syncthreads();
        const float sb = s0[0][cl] + s0[1][cl] + s0[2][cl] + s0[3][cl];
        const float mb = sb / (float)max(r1 - r0, 1LL);
        if (c < C)
            for (long long g = r0 + rg; g < r1; g += 256) {
                float p1 = 0.f;
                const long long ge = min(r1, g + 256);
                for (long long r = g; r < ge; r += 4) { const float d = x[r * ld + c] - mb; p1 = fmaf(d, d, p1); }
                a1 += p1;
            }
        s1[rg][cl] = a1;
        __syncthreads();
        if (rg == 0 && c < C) {
            part[(long long)blockIdx.y * C + c] = sb;
            part[(long long)(gridDim.y + blockIdx.y) * C + c] = s1[0][cl] + s1[1][cl] + s1[2][cl] + s1[3][cl];
        }
        return;
    }
    if (c < C) {
        const float mu = (MODE == 2) ? mean[c] : 0.f;
        const float iv = (MODE == 2) ? inv[c] : 0.f;
        // two-level sums (see kWgGroup): partials p0 / p1 over 64 rows per thread, then into a0 / a1
        for (long long g = r0 + rg; g < r1; g += 256) {
            float p0 = 0.f, p1 = 0.f;
            const long long ge = min(r1, g + 256);
            for (long long r = g; r < ge; r += 4) {
                const float v = x[r * ld + c];
                if (MODE == 0) p0 += v;
                if (MODE == 2) { p0 += v; p1 = fmaf(v, (z[r * C + c] - mu) * iv, p1); }
            }
            a0 += p0;
            a1 += p1;
        }
    }
    s0[rg][cl] = a0;
    s1[rg][cl] = a1;
    __syncthreads();
    if (rg == 0 && c < C) {
        part[(long long)blockIdx.y * C + c] = s0[0][cl] + s0[1][cl] + s0[2][cl] + s0[3][cl];
        if (MODE == 2)
            part[(long long)(gridDim.y + blockIdx.y) * C + c] = s1[0][cl] + s1[1][cl] + s1[2][cl] + s1[3][cl];
    }
}

// Finish a column reduction in double: one 256-thread block per column, each thread summing a strided subset of the
// row-block partials, then a fixed LDS tree (deterministic):
//   STAGE 2: dbeta = S0, dgamma = S1 (into the gradient blob)
//   STAGE 3: out[c] = S (bias gradient)
template <int STAGE>
__global__ __launch_bounds__(256) void k_colfinish(const float* __restrict__ part, int nblk, int C, long long M,
                                                   float* __restrict__ mean, float* __restrict__ inv, float* __restrict__ mm,
                                                   float* __restrict__ mv, float* __restrict__ out0, float* __restrict__ out1) {
    __shared__ double rs[256], rt[256];
    const int c = blockIdx.x, tid = threadIdx.x;
    double s = 0, t = 0;
    for (int b = tid; b < nblk; b += 256) {
        s += part[(long long)b * C + c];
        if (STAGE == 2) t += part[(long long)(nblk + b) * C + c];
    }
    rs[tid] = s;
    rt[tid] = t;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            rs[tid] += rs[tid + o];
            if (STAGE == 2) rt[tid] += rt[tid + o];
        }
        __syncthreads();
    }
    if (tid != 0) return;
    s = rs[0];
    t = rt[0];
    if (STAGE == 2) {
        out0[c] = (float)s;   // dbeta
        out1[c] = (float)t;   // dgamma
    }
    if (STAGE == 3) out0[c] = (float)s;
}

// BN forward statistics from MODE 3 partials (Chan et al. pairwise combination in double): mean = S / M (the sums of
// the former two-pass path, same partials, same order: the same mean), M2 = sum_b M2_b + n_b (mean_b - mean)^2,
// biased var = M2 / M (Keras 2.0.x), inv = 1 / sqrt(var + eps), moving stats <- m * 0.99 + batch * 0.01
__global__ __launch_bounds__(256) void k_bnstat_finish(const float* __restrict__ part, int nblk, int C, long long M,
                                                       long long rpb, float* __restrict__ mean, float* __restrict__ inv,
                                                       float* __restrict__ mm, float* __restrict__ mv) {
    __shared__ double rs[256], rt[256];
    const int c = blockIdx.x, tid = threadIdx.x;
    double s = 0;
    for (int b = tid; b < nblk; b += 256) s += part[(long long)b * C + c];
    rs[tid] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) rs[tid] += rs[tid + o];
        __syncthreads();
    }
    const double mu = rs[0] / (double)M;
    __syncthreads();
    double t = 0;
    for (int b = tid; b < nblk; b += 256) {
        const double nb = (double)min(rpb, M - (long long)b * rpb);
        const double d = (double)part[(long long)b * C + c] / nb - mu;
        t += (double)part[(long long)(nblk + b) * C + c] + nb * d * d;
    }
    rt[tid] = t;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) rt[tid] += rt[tid + o];
        __syncthreads();
    }
    if (tid != 0) return;
    const float m = (float)mu;
    const double var = rt[0] / (double)M;
    mean[c] = m;
    inv[c] = (float)(1.0 / std::sqrt(var + (double)kBnEps));
    mm[c] = mm[c] * BN_MOMENTUM + m * (1.f - BN_MOMENTUM);
    mv[c] = mv[c] * BN_MOMENTUM + (float)var * (1.f - BN_MOMENTUM);
}

struct ActArgs {
    const float* z;          // [N][Hq][Wq][C] pre-BN conv output
    int N, Hq, Wq, C;
    const float* mean;
    const float* inv;
    const float* gamma;
    const float* beta;
    int pool;
    float drop;              // dropout rate (0 = none)
    uint32_t seed, layer;
    float* out;              // layer output (pooled grid when pool)
    long long out_clip;
    int out_pix, out_c;
};

__device__ __forceinline__ float bn_lrelu(const ActArgs& a, long long zi, int c, float& yhat) {
    yhat = fmaf(a.gamma[c], (a.z[zi] - a.mean[c]) * a.inv[c], a.beta[c]);
    return yhat >= 0.f ? yhat : LRELU * yhat;
}

__device__ __forceinline__ float drop_scale(const ActArgs& a, long long idx) {
    if (a.drop <= 0.f) return 1.f;
    const uint32_t h = drop_hash(a.seed, a.layer, (uint32_t)idx);
    return ((float)(h >> 8) * (1.f / 16777216.f)) >= a.drop ? 1.f / (1.f - a.drop) : 0.f;
}

// forward: y = LeakyReLU(BN(z)) [-> 2x2 max pool -> dropout], one thread per output element
__global__ void k_act_fwd(ActArgs a) {
    const int Ho = a.pool ? a.Hq / 2 : a.Hq, Wo = a.pool ? a.Wq / 2 : a.Wq;
    const long long total = (long long)a.N * Ho * Wo * a.C;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        // 32-bit decomposition (every activation tensor < 2^31 elements: avse_trainer_create caps the batch)
        const int ii = (int)i, c = ii % a.C, p = ii / a.C, ox = p % Wo, t2 = p / Wo, oy = t2 % Ho, n = t2 / Ho;
        float y, yh;
        if (a.pool) {
            y = -INFINITY;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const long long zi = (((long long)n * a.Hq + 2 * oy + (e >> 1)) * a.Wq + 2 * ox + (e & 1)) * a.C + c;
                y = fmaxf(y, bn_lrelu(a, zi, c, yh));
            }
        } else {
            y = bn_lrelu(a, i, c, yh);
        }
        y *= drop_scale(a, i);
        a.out[n * a.out_clip + (long long)(oy * Wo + ox) * a.out_pix + a.out_c + c] = y;
    }
}

// backward: g_hat = dL/d(BN output) at full resolution from dL/d(layer output); pool: the window's first maximum
__global__ void k_act_bwd(ActArgs a, const float* __restrict__ gout, long long g_clip, int g_pix, int g_c,
                          float* __restrict__ ghat) {
    const int Ho = a.pool ? a.Hq / 2 : a.Hq, Wo = a.pool ? a.Wq / 2 : a.Wq;
    const long long total = (long long)a.N * Ho * Wo * a.C;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        // 32-bit decomposition (every activation tensor < 2^31 elements: avse_trainer_create caps the batch)
        const int ii = (int)i, c = ii % a.C, p = ii / a.C, ox = p % Wo, t2 = p / Wo, oy = t2 % Ho, n = t2 / Ho;
        const float g = gout[n * g_clip + (long long)(oy * Wo + ox) * g_pix + g_c + c] * drop_scale(a, i);
        if (a.pool) {
            float best = -INFINITY, bh = 0.f;
            int be = 0;
            long long zis[4];
            float yhs[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                zis[e] = (((long long)n * a.Hq + 2 * oy + (e >> 1)) * a.Wq + 2 * ox + (e & 1)) * a.C + c;
                const float y = bn_lrelu(a, zis[e], c, yhs[e]);
                if (y > best) { best = y; be = e; bh = yhs[e]; }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) ghat[zis[e]] = (e == be) ? g * (bh >= 0.f ? 1.f : LRELU) : 0.f;
        } else {
            float yh;
            (void)bn_lrelu(a, i, c, yh);
            ghat[i] = g * (yh >= 0.f ? 1.f : LRELU);
        }
    }
}

// dz = gamma * inv * (g - dbeta / M - xhat * dgamma / M), rounded step by step (explicit fmas and _rn products) so
// the compiler's contraction / hoisting choices cannot make k_bn_bwd and k_bn_bwd_colsum disagree
__device__ __forceinline__ float bn_bwd_dz(float gv, float xh, float ga, float iv, float db, float dg, float rM) {
    const float t = fmaf(-__fmul_rn(xh, dg), rM, fmaf(-db, rM, gv));
    return __fmul_rn(__fmul_rn(ga, iv), t);
}

// in place over g
__global__ void k_bn_bwd(const float* __restrict__ z, float* __restrict__ g, long long M, int C, const float* __restrict__ mean,
                         const float* __restrict__ inv, const float* __restrict__ gamma, const float* __restrict__ dbeta,
                         const float* __restrict__ dgamma) {
    const long long total = M * C;
    const float rM = 1.f / (float)M;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)i % C;   // < 2^31 elements (trainer batch cap)
        const float xh = (z[i] - mean[c]) * inv[c];
        g[i] = bn_bwd_dz(g[i], xh, gamma[c], inv[c], dbeta[c], dgamma[c], rM);
    }
}

// k_bn_bwd fused with the bias gradient's column sums (layers whose BN channels are the conv's output channels): the
// grid, row partition and summation order of k_colreduce<0> over the dz it writes, so the partials (and, after
// k_colfinish<3>, the bias gradient) are those of the two-pass path without dz's second read.
__global__ __launch_bounds__(256) void k_bn_bwd_colsum(const float* __restrict__ z, float* __restrict__ g, long long M, int C,
                                                       const float* __restrict__ mean, const float* __restrict__ inv,
                                                       const float* __restrict__ gamma, const float* __restrict__ dbeta,
                                                       const float* __restrict__ dgamma, long long rows_per_blk,
                                                       float* __restrict__ part) {
    __shared__ float s0[4][64];
    const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
    const int c = blockIdx.x * 64 + cl;
    const long long r0 = blockIdx.y * rows_per_blk, r1 = min(M, r0 + rows_per_blk);
    const float rM = 1.f / (float)M;
    float a0 = 0.f;
    if (c < C) {
        const float mu = mean[c], iv = inv[c], ga = gamma[c], db = dbeta[c], dg = dgamma[c];
        for (long long gr = r0 + rg; gr < r1; gr += 256) {
            float p0 = 0.f;
            const long long ge = min(r1, gr + 256);
            for (long long r = gr; r < ge; r += 4) {
                const long long i = r * C + c;
                const float xh = (z[i] - mu) * iv;
                const float v = bn_bwd_dz(g[i], xh, ga, iv, db, dg, rM);
                g[i] = v;
                p0 = __fadd_rn(p0, v);
            }
            a0 += p0;
        }
    }
    s0[rg][cl] = a0;
    __syncthreads();
    if (rg == 0 && c < C) part[(long long)blockIdx.y * C + c] = s0[0][cl] + s0[1][cl] + s0[2][cl] + s0[3][cl];
}

// mean squared error (network.py:36, Keras mean over every element): per-block partial loss + dL/dy (channel stride gcs)
__global__ __launch_bounds__(256) void k_mse(const float* __restrict__ y, const float* __restrict__ t, long long n, int gcs,
                                             float* __restrict__ g, float* __restrict__ part) {
    __shared__ float red[256];
    float acc = 0.f;
    const float s = 2.f / (float)n;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float d = y[i * gcs] - t[i];
        acc = fmaf(d, d, acc);
        g[i * gcs] = s * d;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_mse_finish(const float* __restrict__ part, int nblk, long long n, float* __restrict__ loss) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double s = 0;
    for (int b = 0; b < nblk; ++b) s += part[b];
    *loss = (float)(s / (double)n);
}

// Weight gradient dW[tap][a][b] = sum over (n, y, x) of G[n][y*sy + dy_t][x*sx + dx_t][a] * H[n][y][x][b]
// (conv: G = input, H = dz; transposed conv: G = dz, H = input; dense: 1 x 1 grids).  Block = 64 a x 64 b of one tap
// over one split of the rows; 256 threads x 4 x 4 outputs; 16-row chunks of G and H staged in LDS.
struct WgArgs {
    const float* G;
    int Hg, Wg, gcs;
    long long g_clip;
    const float* H;
    int Hh, Wh, hcs;
    long long h_clip;
    int N, sy, sx;
    int A, B;
    int ntaps;
    const int2* taps;
    long long rows_per_split;
    float* part;             // [splits][ntaps][A][B]
};

// row r of the reduction -> (n, y, x) on an Hh x Wh grid in 32-bit arithmetic (R < 2^31: host-checked); the
// 64-bit div / mod sequences it replaces were ~a third of k_wgrad's instructions
__device__ __forceinline__ void row_nyx(long long r, int Hh, int Wh, int& n, int& y, int& x) {
    const int ri = (int)r, hw = Hh * Wh;
    n = ri / hw;
    const int rem = ri - n * hw;
    y = rem / Wh;
    x = rem - y * Wh;
}

// Row sums of the weight gradients and column statistics are two-level: a thread sums kWgGroup rows into a partial that
// is then added to its running total, so no fp32 sum runs sequentially over more than ~kWgGroup + rows / kWgGroup
// terms.  BN-backed gradients are small differences of large sums (dz has zero column mean): a one-level sum over the
// ~5,000 rows per split of a 1023-clip batch left ~1.5e-2 relative RMS in every gradient (profiles/r03a_gputest.log).
constexpr int kWgGroup = 256;
template <int A, int B>
__device__ __forceinline__ void flush_partial(float (&acc)[A][B], float (&p)[A][B]) {
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < B; ++j) {
            acc[i][j] += p[i][j];
            p[i][j] = 0.f;
        }
}

// Block = 64 a x 64 b of one tap over one split of the rows: 4 waves of 32 a x 32 b, each 2 x 2 exact-fp32 MFMAs
// (v_mfma_f32_16x16x4_f32: M = a, N = b, K = 4 rows) per 4-row step of a WG_CH-row chunk staged in LDS; the next chunk's
// global loads are issued before the current chunk's MFMAs.  (Round 2's VALU form — 4 x 4 FMAs per thread — ran at
// ~55 TFLOP/s: 0.97 ms of a 8.4-ms batch-16 step for v_conv2's gradient alone.)
constexpr int WG_P = 80;   // LDS row pitch (floats): rows k and k + 1 of an operand read land 16 banks apart
constexpr int WG_CH = 32;   // rows per LDS chunk (two barriers per chunk; 16 measured the same)
__global__ __launch_bounds__(256) void k_wgrad(WgArgs w) {
    __shared__ __attribute__((aligned(16))) float gs[WG_CH][WG_P], hs[WG_CH][WG_P];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nbt = (w.B + 63) / 64;
    const int a0 = (blockIdx.x / nbt) * 64, b0 = (blockIdx.x % nbt) * 64;
    const int tap = blockIdx.y;
    const int2 t = w.taps[tap];
    const long long R = (long long)w.N * w.Hh * w.Wh;
    const long long r0 = blockIdx.z * w.rows_per_split, r1 = min(R, r0 + w.rows_per_split);
    const int lr = tid >> 4, lc = (tid & 15) * 4;   // loader: row lr of the chunk, 4 columns lc..lc+3
    // the tile's columns inside A / B: whole-float4 loads without per-lane edge tests (wave-uniform branch)
    const bool full = a0 + 64 <= w.A && b0 + 64 <= w.B;
    auto load = [&](long long r, int n, int y, int x, float4& gv, float4& hv) {
        gv = make_float4(0.f, 0.f, 0.f, 0.f);
        hv = gv;
        if (r >= r1) return;
        const float* hp = w.H + n * w.h_clip + (long long)(y * w.Wh + x) * w.hcs + b0 + lc;
        const int gy = y * w.sy + t.x, gx = x * w.sx + t.y;
        const bool gin = gy >= 0 && gy < w.Hg && gx >= 0 && gx < w.Wg;
        const float* gp = w.G + n * w.g_clip + (long long)(gy * w.Wg + gx) * w.gcs + a0 + lc;
        if (full) {
            hv = *reinterpret_cast<const float4*>(hp);
            if (gin) gv = *reinterpret_cast<const float4*>(gp);
            return;
        }
        if (b0 + lc + 3 < w.B) hv = make_float4(hp[0], hp[1], hp[2], hp[3]);
        else {
            if (b0 + lc < w.B) hv.x = hp[0];
            if (b0 + lc + 1 < w.B) hv.y = hp[1];
            if (b0 + lc + 2 < w.B) hv.z = hp[2];
        }
        if (gin) {
            if (a0 + lc + 3 < w.A) gv = make_float4(gp[0], gp[1], gp[2], gp[3]);
            else {
                if (a0 + lc < w.A) gv.x = gp[0];
                if (a0 + lc + 1 < w.A) gv.y = gp[1];
                if (a0 + lc + 2 < w.A) gv.z = gp[2];
            }
        }
    };
    // MFMA operands: lane l reads row 4 ks + (l >> 4) of the chunk, column (l & 15) of its 16-wide a / b block
    const int wa = (wave >> 1) * 32, wb = (wave & 1) * 32, kr = lane >> 4, kc = lane & 15;
    f32x4 acc[2][2], p[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = p[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    constexpr int LPT = WG_CH / 16;   // rows each thread stages per chunk
    // a thread's rows advance by WG_CH per chunk: (n, y, x) stepped in place when a grid row holds >= WG_CH pixels
    // (at most one wrap), else re-derived by division (the divisions were most of the loader's instructions)
    const bool step_in_place = w.Wh >= WG_CH;
    float4 gv[LPT], hv[LPT];
    int cn[LPT], cy[LPT], cx[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
        const long long r = r0 + lr + 16 * u;
        if (r < r1) row_nyx(r, w.Hh, w.Wh, cn[u], cy[u], cx[u]);
        else cn[u] = cy[u] = cx[u] = 0;
        load(r, cn[u], cy[u], cx[u], gv[u], hv[u]);
    }
    for (long long rc = r0; rc < r1; rc += WG_CH) {
        if (((rc - r0) & (kWgGroup - 1)) == 0 && rc != r0) {   // two-level row sums (see kWgGroup)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] += p[i][j];
                    p[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
                }
        }
        __syncthreads();   // the previous chunk's operand reads are done
#pragma unroll
        for (int u = 0; u < LPT; ++u) {
            *reinterpret_cast<float4*>(&gs[lr + 16 * u][lc]) = gv[u];
            *reinterpret_cast<float4*>(&hs[lr + 16 * u][lc]) = hv[u];
        }
        __syncthreads();
        if (rc + WG_CH < r1)
#pragma unroll
            for (int u = 0; u < LPT; ++u) {
                const long long r = rc + WG_CH + lr + 16 * u;
                if (step_in_place) {
                    cx[u] += WG_CH;
                    if (cx[u] >= w.Wh) {
                        cx[u] -= w.Wh;
                        if (++cy[u] == w.Hh) {
                            cy[u] = 0;
                            ++cn[u];
                        }
                    }
                } else if (r < r1) {
                    row_nyx(r, w.Hh, w.Wh, cn[u], cy[u], cx[u]);
                }
                load(r, cn[u], cy[u], cx[u], gv[u], hv[u]);
            }
#pragma unroll
        for (int ks = 0; ks < WG_CH / 4; ++ks) {
            const float* gr = &gs[4 * ks + kr][0];
            const float* hr = &hs[4 * ks + kr][0];
            const float av[2] = {gr[wa + kc], gr[wa + 16 + kc]}, bv[2] = {hr[wb + kc], hr[wb + 16 + kc]};
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) p[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], p[i][j], 0, 0, 0);
        }
    }
    float* out = w.part + ((long long)blockIdx.z * w.ntaps + tap) * w.A * w.B;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const f32x4 v = acc[i][j] + p[i][j];
            const int b = b0 + wb + 16 * j + kc;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int a = a0 + wa + 16 * i + 4 * kr + e;   // D row 4 (l >> 4) + e, column l & 15
                if (a < w.A && b < w.B) out[(long long)a * w.B + b] = v[e];
            }
        }
}

// Narrow-A variant (A <= 8: v_conv1's 5 input frames, d_deconv6's single output channel): block tile 8 a x 128 b,
// thread = 4 a x 1 b, 32-row chunks (the 64 x 64 tile computed 92 % padding for v_conv1: 1.9 ms of a 19.7-ms step).
__global__ __launch_bounds__(256) void k_wgrad_na(WgArgs w) {
    __shared__ float gs[32][8], hs[32][132];
    const int tid = threadIdx.x, ta = tid >> 7, tb = tid & 127;
    const int b0 = blockIdx.x * 128;
    const int tap = blockIdx.y;
    const int2 t = w.taps[tap];
    const long long R = (long long)w.N * w.Hh * w.Wh;
    const long long r0 = blockIdx.z * w.rows_per_split, r1 = min(R, r0 + w.rows_per_split);
    float acc[1][4] = {{0.f, 0.f, 0.f, 0.f}}, p[1][4] = {{0.f, 0.f, 0.f, 0.f}};
    for (long long rc = r0; rc < r1; rc += 32) {
        if (((rc - r0) & (kWgGroup - 1)) == 0) flush_partial(acc, p);
        float gv = 0.f;
        {   // G: row tid / 8, channel tid % 8
            const long long r = rc + (tid >> 3);
            const int a = tid & 7;
            if (r < r1 && a < w.A) {
                int n, y, x;
                row_nyx(r, w.Hh, w.Wh, n, y, x);
                const int gy = y * w.sy + t.x, gx = x * w.sx + t.y;
                if (gy >= 0 && gy < w.Hg && gx >= 0 && gx < w.Wg) gv = w.G[n * w.g_clip + (long long)(gy * w.Wg + gx) * w.gcs + a];
            }
        }
        float hv[16];
        {   // H: row (tid / 128) + 2 q, channel b0 + tid % 128; (n, y, x) advanced by 2 rows per q (no divisions)
            const long long r = rc + (tid >> 7);
            int n, y, x;
            row_nyx(r, w.Hh, w.Wh, n, y, x);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                hv[q] = 0.f;
                if (rc + (tid >> 7) + 2 * q < r1 && b0 + tb < w.B)
                    hv[q] = w.H[n * w.h_clip + (long long)(y * w.Wh + x) * w.hcs + b0 + tb];
                x += 2;
                while (x >= w.Wh) {
                    x -= w.Wh;
                    if (++y == w.Hh) { y = 0; ++n; }
                }
            }
        }
        __syncthreads();
        gs[tid >> 3][tid & 7] = gv;
#pragma unroll
        for (int q = 0; q < 16; ++q) hs[(tid >> 7) + 2 * q][tb] = hv[q];
        __syncthreads();
#pragma unroll 8
        for (int k = 0; k < 32; ++k) {
            const float hb = hs[k][tb];
#pragma unroll
            for (int i = 0; i < 4; ++i) p[0][i] = fmaf(gs[k][ta * 4 + i], hb, p[0][i]);
        }
    }
    flush_partial(acc, p);
    float* out = w.part + ((long long)blockIdx.z * w.ntaps + tap) * w.A * w.B;
    const int b = b0 + tb;
    if (b < w.B)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int a = ta * 4 + i;
            if (a < w.A) out[(long long)a * w.B + b] = acc[0][i];
        }
}

// All-taps narrow-A variant (A <= 8, 25 taps, H dense NHWC with B and its channel stride multiples of 4): one
// block walks a row range ONCE for every tap, so the wide operand H (v_conv1's 128-channel dz, 134 MB at batch
// 16) is read once instead of once per tap (k_wgrad_na reads it 25 times: ~1 ms per step).  The chunk's 8-channel
// G rows are gathered per tap into LDS.  Thread = 7 taps (tap group tid / 64) x 4 a x 4 b: per row 8
// ds_read_b128 for 112 FMAs (a 4 a x 1 b x 25 tap thread needed one broadcast read per 4 FMAs: LDS-bound).
constexpr int NAT_TAPS = 25, NAT_TG = 7;   // taps, taps per group (4 groups, the last one 4 taps)
__global__ __launch_bounds__(256) void k_wgrad_nat(WgArgs w) {
    __shared__ float4 hs[32][33];                 // [row][b / 4] (+1 float4 pad)
    __shared__ float4 gs[4 * NAT_TG][32][2];      // [tap][row][a / 4]
    __shared__ int2 tl[NAT_TAPS];
    const int tid = threadIdx.x, tg = tid >> 6, ag = (tid >> 5) & 1, bq = tid & 31;
    const int b0 = blockIdx.x * 128;
    const long long R = (long long)w.N * w.Hh * w.Wh;
    const long long r0 = blockIdx.z * w.rows_per_split, r1 = min(R, r0 + w.rows_per_split);
    if (tid < NAT_TAPS) tl[tid] = w.taps[tid];
    float4 acc[NAT_TG][4];                        // [tap j][a] x 4 b
#pragma unroll
    for (int j = 0; j < NAT_TG; ++j)
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[j][a] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int hr = tid >> 5, hc = (tid & 31) * 4;   // H loader: rows hr + 8 q, columns b0 + hc .. +3
    const int gr = tid >> 3, ga = tid & 7;          // G loader: row gr, channel ga, every tap
    const bool hcol = b0 + hc < w.B;
    __syncthreads();
    for (long long rc = r0; rc < r1; rc += 32) {
        float4 hv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const long long r = rc + hr + 8 * q;
            hv[q] = (r < r1 && hcol) ? *reinterpret_cast<const float4*>(w.H + r * w.hcs + b0 + hc)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float gv[NAT_TAPS];
        {
            const long long r = rc + gr;
            const bool ok = r < r1 && ga < w.A;
            const long long rr = ok ? r : 0;
            int n, y, x;
            row_nyx(rr, w.Hh, w.Wh, n, y, x);
            const float* gb = w.G + n * w.g_clip + ga;
#pragma unroll
            for (int t = 0; t < NAT_TAPS; ++t) {
                const int2 tp = tl[t];
                const int gy = y * w.sy + tp.x, gx = x * w.sx + tp.y;
                gv[t] = (ok && gy >= 0 && gy < w.Hg && gx >= 0 && gx < w.Wg) ? gb[(long long)(gy * w.Wg + gx) * w.gcs] : 0.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) hs[hr + 8 * q][hc >> 2] = hv[q];
#pragma unroll
        for (int t = 0; t < NAT_TAPS; ++t) reinterpret_cast<float*>(&gs[t][gr][0])[ga] = gv[t];
        __syncthreads();
#pragma unroll 2
        for (int k = 0; k < 32; ++k) {
            const float4 h4 = hs[k][bq];
#pragma unroll
            for (int j = 0; j < NAT_TG; ++j) {
                if (tg * NAT_TG + j >= NAT_TAPS) break;   // the last group's 3 missing taps (wave-uniform)
                const float4 g4 = gs[tg * NAT_TG + j][k][ag];
                const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    acc[j][a].x = fmaf(gg[a], h4.x, acc[j][a].x);
                    acc[j][a].y = fmaf(gg[a], h4.y, acc[j][a].y);
                    acc[j][a].z = fmaf(gg[a], h4.z, acc[j][a].z);
                    acc[j][a].w = fmaf(gg[a], h4.w, acc[j][a].w);
                }
            }
        }
    }
    const int b = b0 + 4 * bq;
    if (b < w.B)
#pragma unroll
        for (int j = 0; j < NAT_TG; ++j) {
            const int t = tg * NAT_TG + j;
            if (t >= NAT_TAPS) break;
            float* out = w.part + ((long long)blockIdx.z * NAT_TAPS + t) * w.A * w.B;
#pragma unroll
            for (int a = 0; a < 4; ++a)
                if (4 * ag + a < w.A) *reinterpret_cast<float4*>(out + (long long)(4 * ag + a) * w.B + b) = acc[j][a];
        }
}

// out[i] = sum over z of part[z][i], z in increasing order within each of the 4 waves' strided subsets (z = w mod 4),
// then wave 0 + 1 + 2 + 3: deterministic.  One wave per z subset keeps 4x the loads in flight of a thread that
// walks all splits (the all-taps wgrad writes ~500 splits of 16,000 floats)
__global__ __launch_bounds__(256) void k_sum_splits(const float* __restrict__ part, int splits, long long n,
                                                    float* __restrict__ out) {
    __shared__ float red[3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (long long i0 = blockIdx.x * 64LL; i0 < n; i0 += gridDim.x * 64LL) {
        const long long i = i0 + lane;
        float s = 0.f;
        if (i < n) {
            int z = w;
            for (; z + 12 < splits; z += 16) {   // four independent loads in flight
                const float a = part[(long long)z * n + i], b = part[(long long)(z + 4) * n + i];
                const float c = part[(long long)(z + 8) * n + i], d = part[(long long)(z + 12) * n + i];
                s += a; s += b; s += c; s += d;
            }
            for (; z < splits; z += 4) s += part[(long long)z * n + i];
        }
        if (w) red[w - 1][lane] = s;
        __syncthreads();
        if (w == 0 && i < n) out[i] = ((s + red[0][lane]) + red[1][lane]) + red[2][lane];
        __syncthreads();
    }
}

// Keras 2.0 Adam (optimizers.py): m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2; p -= lr_t m / (sqrt(v) + eps)
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                       long long n, float lr_t, float b1, float b2, float eps) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float gi = g[i];
        const float mi = b1 * m[i] + (1.f - b1) * gi;
        const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        p[i] -= lr_t * mi / (sqrtf(vi) + eps);
    }
}

// ------------------------------------------------------------------------------------------------------------
// host plan
// ------------------------------------------------------------------------------------------------------------
struct TLayer {
    LayerDef L;
    int cin_pad = 0;          // channel stride of this layer's input tensor
    int hq = 1, wq = 1;       // conv output grid (full resolution)
    int ho = 1, wo = 1;       // after pool
    long long o_k = 0, o_b = 0, o_g = -1, o_be = -1, o_mm = -1, o_mv = -1;   // canonical blob offsets
    // forward conv (k_conv), packed [phase][cout][kpad] gathered from the blob
    int nphase = 1;
    ConvPhase ph[MAX_PHASES];
    std::vector<int2> taps;
    long long fw_off = 0;     // offset in the forward packed buffer
    int2* d_taps = nullptr;
    // dgrad
    bool dgrad = false;
    int dg_nphase = 1, dg_hq = 1, dg_wq = 1, dg_sy = 1, dg_sx = 1, dg_oys = 1, dg_oxs = 1, dg_ci = 0;
    ConvPhase dg_ph[MAX_PHASES];
    std::vector<int2> dg_taps;
    long long dg_off = 0;
    int2* d_dg_taps = nullptr;
    // wgrad taps (dy, dx) per Keras tap ky * kw + kx
    std::vector<int2> wg_taps;
    int2* d_wg_taps = nullptr;
    // tensors
    float* in = nullptr;      // this layer's input [N][hin][win][cin_pad] (or a concat view)
    long long in_clip = 0;
    float* z = nullptr;       // [N][hq][wq][cout] pre-BN (the output itself for d_deconv6, channel stride zc)
    int zc = 0;
    float* mean = nullptr;
    float* inv = nullptr;
    float* gin = nullptr;     // dL/d(input), same layout as `in` (only when dgrad)
};

}  // namespace
}  // namespace avse

using namespace avse;

struct avse_trainer {
    int device = 0;
    int64_t max_n = 0;
    int64_t nparams = 0;
    int64_t step = 0;         // Adam iterations done (Keras `iterations`)
    NetPlan plan = kPlan25;   // network shape (netplan.h)
    std::vector<TLayer> layers;
    float *P = nullptr, *Gr = nullptr, *Mo = nullptr, *Vo = nullptr;
    float *wfwd = nullptr, *wdg = nullptr;
    PackTile* pack_tiles = nullptr;   // k_pack work list (forward + dgrad packings)
    long long n_pack_tiles = 0;
    long long n_fwd = 0, n_dg = 0;
    float *ones = nullptr, *zeros = nullptr;
    float *in_audio = nullptr, *in_video = nullptr, *concat = nullptr, *g6 = nullptr, *ghat = nullptr;
    float* red = nullptr;     // column-reduction / loss partials
    long long red_floats = 0;
    float* wpart = nullptr;   // wgrad split partials
    long long wpart_floats = 0;
    float* kpart = nullptr;   // split-K partials of the short-grid convolutions (train_split)
    float* loss = nullptr;
    std::vector<void*> allocs;
};

namespace {

int tfail(int code, const std::string& msg) {
    set_error(msg);
    return code;
}

template <typename T>
int talloc(avse_trainer* t, T** p, size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return tfail(AVSE_ERR_OOM, "hipMalloc failed (trainer)");
    if (hipMemset(q, 0, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return tfail(AVSE_ERR_HIP, "hipMemset failed");
    t->allocs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
}

long long kpad_of(int ntaps, int cp) { return ((long long)ntaps * cp + 31) / 32 * 32; }

// Keras kernel element index for (ky, kx, in-channel c_in, out-channel c_out) of layer L
long long kidx(const LayerDef& L, int ky, int kx, int ci, int co) {
    if (L.kind == DENSE) return (long long)ci * L.cout + co;
    if (L.kind == CONV) return (((long long)ky * L.kw + kx) * L.cin + ci) * L.cout + co;
    return (((long long)ky * L.kw + kx) * L.cout + co) * L.cin + ci;   // transposed conv (kh, kw, cout, cin)
}

// k_pack tiles of one (layer, phase, tap) block: rows x cols, dst row stride dld, source element (r, c) at
// src + r sr + c sc (Keras kernel strides from kidx)
void add_pack_tiles(std::vector<PackTile>& v, int which, long long dst, int dld, long long src, long long sr, long long sc,
                    int rows, int cols) {
    for (int r0 = 0; r0 < rows; r0 += 64)
        for (int c0 = 0; c0 < cols; c0 += 64)
            v.push_back(PackTile{dst + (long long)r0 * dld + c0, src + r0 * sr + c0 * sc, std::min(64, rows - r0),
                                 std::min(64, cols - c0), dld, (int)sr, (int)sc, which});
}

// the packings the tiles write must be exactly the index maps (entries -1: padding, left at the allocation's zero)
int check_pack_tiles(const std::vector<PackTile>& v, int which, const std::vector<int>& map) {
    std::vector<int> got(map.size(), -1);
    for (const PackTile& T : v) {
        if (T.which != which) continue;
        for (int r = 0; r < T.R; ++r)
            for (int c = 0; c < T.C; ++c) {
                const long long d = T.dst + (long long)r * T.dld + c;
                if (d < 0 || d >= (long long)map.size() || got[d] != -1) return tfail(AVSE_ERR_INVALID, "pack tiles overlap");
                got[d] = (int)(T.src + (long long)r * T.sr + (long long)c * T.sc);
            }
    }
    if (got != map) return tfail(AVSE_ERR_INVALID, "pack tiles disagree with the packing map");
    return 0;
}

int build_plan(avse_trainer* t, const float* host_blob) {
    t->layers.resize(kNumLayers);
    long long off = 0;
    std::vector<int> mf, md;   // forward / dgrad gather maps (the reference the k_pack tiles are checked against)
    std::vector<PackTile> tiles;
    for (int i = 0; i < kNumLayers; ++i) {
        TLayer& T = t->layers[i];
        const LayerDef& L = t->plan.L[i];
        T.L = L;
        T.cin_pad = (L.kind == DENSE) ? L.cin : ((L.cin + 7) / 8) * 8;
        T.o_k = off;
        off += (long long)L.kh * L.kw * L.cin * L.cout;
        T.o_b = off;
        off += L.cout;
        if (L.bn) {
            T.o_g = off; T.o_be = off + L.bn_channels; T.o_mm = off + 2 * L.bn_channels; T.o_mv = off + 3 * L.bn_channels;
            off += 4LL * L.bn_channels;
        }
        const int pt = (L.kind == CONV) ? same_pad_before(L.hin, L.kh, L.sh) : std::max(L.kh - L.sh, 0) / 2;
        const int pl = (L.kind == CONV) ? same_pad_before(L.win, L.kw, L.sw) : std::max(L.kw - L.sw, 0) / 2;
        // ---- forward phases / taps (as capi.hip build_layer) ----
        std::vector<std::vector<std::pair<int, int>>> ptaps;
        if (L.kind == DENSE) {
            T.nphase = 1;
            ptaps.push_back({{0, 0}});
            T.taps.push_back(make_int2(0, 0));
            T.ph[0] = ConvPhase{0, 0, 1, 0, 0, 0};
        } else if (L.kind == CONV) {
            T.hq = same_out(L.hin, L.sh);
            T.wq = same_out(L.win, L.sw);
            T.nphase = 1;
            std::vector<std::pair<int, int>> pl_;
            for (int ky = 0; ky < L.kh; ++ky)
                for (int kx = 0; kx < L.kw; ++kx) {
                    pl_.push_back({ky, kx});
                    T.taps.push_back(make_int2(ky - pt, kx - pl));
                }
            ptaps.push_back(pl_);
            T.ph[0] = ConvPhase{0, 0, (int)pl_.size(), 0, 0, 0};
        } else {
            T.hq = L.hin * L.sh;
            T.wq = L.win * L.sw;
            T.nphase = L.sh * L.sw;
            if (T.nphase > MAX_PHASES) return tfail(AVSE_ERR_UNSUPPORTED, "deconv stride too large");
            for (int py = 0; py < L.sh; ++py)
                for (int px = 0; px < L.sw; ++px) {
                    std::vector<std::pair<int, int>> pl_;
                    const int toff = (int)T.taps.size();
                    for (int ky = 0; ky < L.kh; ++ky) {
                        const int ry = py + pt - ky;
                        if (((ry % L.sh) + L.sh) % L.sh) continue;
                        for (int kx = 0; kx < L.kw; ++kx) {
                            const int rx = px + pl - kx;
                            if (((rx % L.sw) + L.sw) % L.sw) continue;
                            pl_.push_back({ky, kx});
                            T.taps.push_back(make_int2(ry / L.sh, rx / L.sw));
                        }
                    }
                    T.ph[py * L.sw + px] = ConvPhase{py, px, (int)pl_.size(), 0, 0, toff};
                    ptaps.push_back(pl_);
                }
        }
        T.ho = L.pool ? T.hq / 2 : T.hq;
        T.wo = L.pool ? T.wq / 2 : T.wq;
        T.fw_off = (long long)mf.size();
        long long woff = 0;
        for (int p = 0; p < T.nphase; ++p) {
            const int cp = T.cin_pad;
            const long long kp = kpad_of((int)ptaps[p].size(), cp);
            T.ph[p].kpad = (int)kp;
            T.ph[p].w_off = woff;
            const size_t base = mf.size();
            mf.resize(base + (size_t)(L.cout * kp), -1);
            for (int n = 0; n < L.cout; ++n)
                for (size_t j = 0; j < ptaps[p].size(); ++j)
                    for (int c = 0; c < L.cin; ++c)
                        mf[base + (size_t)n * kp + j * cp + c] =
                            (int)(T.o_k + kidx(L, ptaps[p][j].first, ptaps[p][j].second, c, n));
            for (size_t j = 0; j < ptaps[p].size(); ++j) {
                const int ky = ptaps[p][j].first, kx = ptaps[p][j].second;
                const long long s0 = kidx(L, ky, kx, 0, 0);
                add_pack_tiles(tiles, 0, (long long)base + (long long)j * cp, (int)kp, T.o_k + s0,
                               kidx(L, ky, kx, 0, 1) - s0, kidx(L, ky, kx, 1, 0) - s0, L.cout, L.cin);
            }
            woff += (long long)L.cout * kp;
        }
        // ---- weight-gradient taps: Keras tap order, offsets (ky - pt, kx - pl) on the strided grid ----
        for (int ky = 0; ky < L.kh; ++ky)
            for (int kx = 0; kx < L.kw; ++kx) T.wg_taps.push_back(make_int2(ky - (L.kind == DENSE ? 0 : pt), kx - (L.kind == DENSE ? 0 : pl)));
        // ---- dgrad: not for the first layer of a branch (its input is data) ----
        T.dgrad = !(i == 0 || std::strcmp(L.name, "v_conv1") == 0);
        if (T.dgrad) {
            const int cpi = (L.cout % 8) ? ((L.cout + 7) / 8) * 8 : L.cout;   // dz channel stride (d_deconv6: 8)
            T.dg_ci = (L.kind == DENSE) ? L.cout : cpi;
            std::vector<std::vector<std::pair<int, int>>> dtaps;
            if (L.kind == DENSE) {
                T.dg_nphase = 1;
                dtaps.push_back({{0, 0}});
                T.dg_taps.push_back(make_int2(0, 0));
                T.dg_ph[0] = ConvPhase{0, 0, 1, 0, 0, 0};
            } else if (L.kind == CONV) {
                // dx[iy], iy = q s + r: taps ky = r + pt (mod s), dz row q + (r + pt - ky) / s
                if (L.hin % L.sh || L.win % L.sw) return tfail(AVSE_ERR_UNSUPPORTED, "conv dgrad needs input dims divisible by the stride");
                T.dg_nphase = L.sh * L.sw;
                T.dg_hq = L.hin / L.sh;
                T.dg_wq = L.win / L.sw;
                T.dg_oys = L.sh;
                T.dg_oxs = L.sw;
                for (int ry = 0; ry < L.sh; ++ry)
                    for (int rx = 0; rx < L.sw; ++rx) {
                        std::vector<std::pair<int, int>> pl_;
                        const int toff = (int)T.dg_taps.size();
                        for (int ky = 0; ky < L.kh; ++ky) {
                            const int dy = ry + pt - ky;
                            if (((dy % L.sh) + L.sh) % L.sh) continue;
                            for (int kx = 0; kx < L.kw; ++kx) {
                                const int dx = rx + pl - kx;
                                if (((dx % L.sw) + L.sw) % L.sw) continue;
                                pl_.push_back({ky, kx});
                                T.dg_taps.push_back(make_int2(dy / L.sh, dx / L.sw));
                            }
                        }
                        if (pl_.empty()) return tfail(AVSE_ERR_UNSUPPORTED, "conv dgrad phase without taps");
                        T.dg_ph[ry * L.sw + rx] = ConvPhase{ry, rx, (int)pl_.size(), 0, 0, toff};
                        dtaps.push_back(pl_);
                    }
            } else {
                // transposed conv: din[iy] = sum_ky dout[iy s + ky - pt] W[ky] (a strided conv of dout)
                T.dg_nphase = 1;
                T.dg_hq = L.hin;
                T.dg_wq = L.win;
                T.dg_sy = L.sh;
                T.dg_sx = L.sw;
                std::vector<std::pair<int, int>> pl_;
                for (int ky = 0; ky < L.kh; ++ky)
                    for (int kx = 0; kx < L.kw; ++kx) {
                        pl_.push_back({ky, kx});
                        T.dg_taps.push_back(make_int2(ky - pt, kx - pl));
                    }
                dtaps.push_back(pl_);
                T.dg_ph[0] = ConvPhase{0, 0, (int)pl_.size(), 0, 0, 0};
            }
            T.dg_off = (long long)md.size();
            long long doff = 0;
            for (int p = 0; p < T.dg_nphase; ++p) {
                const int cp = T.dg_ci;
                const long long kp = kpad_of((int)dtaps[p].size(), cp);
                T.dg_ph[p].kpad = (int)kp;
                T.dg_ph[p].w_off = doff;
                const size_t base = md.size();
                md.resize(base + (size_t)(L.cin * kp), -1);
                for (int n = 0; n < L.cin; ++n)          // output channel of dgrad = the layer's input channel
                    for (size_t j = 0; j < dtaps[p].size(); ++j)
                        for (int c = 0; c < L.cout; ++c)   // reduction channel = the layer's output channel
                            md[base + (size_t)n * kp + j * cp + c] =
                                (int)(T.o_k + kidx(L, dtaps[p][j].first, dtaps[p][j].second, n, c));
                for (size_t j = 0; j < dtaps[p].size(); ++j) {
                    const int ky = dtaps[p][j].first, kx = dtaps[p][j].second;
                    const long long s0 = kidx(L, ky, kx, 0, 0);
                    add_pack_tiles(tiles, 1, (long long)base + (long long)j * cp, (int)kp, T.o_k + s0,
                                   kidx(L, ky, kx, 1, 0) - s0, kidx(L, ky, kx, 0, 1) - s0, L.cin, L.cout);
                }
                doff += (long long)L.cin * kp;
            }
        }
    }
    if (off != blob_floats(t->plan)) return tfail(AVSE_ERR_INVALID, "trainer plan / blob size mismatch");
    t->nparams = off;
    t->n_fwd = (long long)mf.size();
    t->n_dg = (long long)md.size();
    if (int rc = check_pack_tiles(tiles, 0, mf)) return rc;
    if (int rc = check_pack_tiles(tiles, 1, md)) return rc;
    t->n_pack_tiles = (long long)tiles.size();
    if (int rc = talloc(t, &t->pack_tiles, tiles.size())) return rc;
    if (int rc = talloc(t, &t->wfwd, mf.size())) return rc;   // zeroed: the packings' padding is never written
    if (int rc = talloc(t, &t->wdg, md.size())) return rc;
    AVSE_HIP_CHECK(hipMemcpy(t->pack_tiles, tiles.data(), tiles.size() * sizeof(PackTile), hipMemcpyHostToDevice));
    for (auto& T : t->layers) {
        if (int rc = talloc(t, &T.d_taps, T.taps.size())) return rc;
        AVSE_HIP_CHECK(hipMemcpy(T.d_taps, T.taps.data(), T.taps.size() * sizeof(int2), hipMemcpyHostToDevice));
        if (int rc = talloc(t, &T.d_wg_taps, T.wg_taps.size())) return rc;
        AVSE_HIP_CHECK(hipMemcpy(T.d_wg_taps, T.wg_taps.data(), T.wg_taps.size() * sizeof(int2), hipMemcpyHostToDevice));
        if (T.dgrad) {
            if (int rc = talloc(t, &T.d_dg_taps, T.dg_taps.size())) return rc;
            AVSE_HIP_CHECK(hipMemcpy(T.d_dg_taps, T.dg_taps.data(), T.dg_taps.size() * sizeof(int2), hipMemcpyHostToDevice));
        }
    }
    // parameters, gradients, Adam moments
    if (int rc = talloc(t, &t->P, off)) return rc;
    if (int rc = talloc(t, &t->Gr, off)) return rc;
    if (int rc = talloc(t, &t->Mo, off)) return rc;
    if (int rc = talloc(t, &t->Vo, off)) return rc;
    AVSE_HIP_CHECK(hipMemcpy(t->P, host_blob, off * sizeof(float), hipMemcpyHostToDevice));
    return 0;
}

// k_wgrad_nat applies: A <= 8, 5 x 5 taps, a conv whose H (dz on the conv grid) is dense with 4-aligned rows
bool wg_all_taps(const TLayer& T) {
    const LayerDef& L = T.L;
    return L.kind == CONV && L.cin <= 8 && L.kh * L.kw == 25 && L.cout % 4 == 0 && T.zc % 4 == 0;
}

// wgrad work split over the reduction rows: ~2048 blocks in total, >= 256 rows per split (k_wgrad_nat: ~512
// blocks of >= 256 rows, each covering every tap: its partials are 25 taps deep)
constexpr long long kNatMaxRows = 2048;
constexpr long long kSplitTiles = 2048;   // train_split: tiles x splits per launch (its workspace: 128 x 128 floats each)
long long wg_splits(const TLayer& T, int64_t N) {
    const LayerDef& L = T.L;
    const int A = (L.kind == DECONV) ? L.cout : L.cin, B = (L.kind == DECONV) ? L.cin : L.cout;
    const long long R = N * (long long)((L.kind == DECONV) ? L.hin * L.win : T.hq * T.wq);
    if (wg_all_taps(T)) {
        // its per-thread row sums are one-level (112 accumulators leave no registers for a second set), so a split
        // never exceeds kNatMaxRows rows (more, smaller partial slabs at large batches; 16,000 floats each)
        const long long bt = (B + 127) / 128;
        return std::max({1LL, std::min((512 + bt - 1) / bt, (R + 255) / 256), (R + kNatMaxRows - 1) / kNatMaxRows});
    }
    const long long tiles = (A <= 8 ? (long long)((B + 127) / 128) : (long long)((A + 63) / 64) * ((B + 63) / 64)) * L.kh * L.kw;
    return std::max(1LL, std::min((2048 + tiles - 1) / tiles, (R + 255) / 256));
}

int alloc_tensors(avse_trainer* t) {
    const long long N = t->max_n;
    // unit scale / zero shift of the bias-only and dgrad convolutions: one entry per output channel (the widest
    // is enc_dense's input gradient, 5248 channels)
    int cmax = 0;
    for (int i = 0; i < kNumLayers; ++i) cmax = std::max({cmax, t->plan.L[i].cin, t->plan.L[i].cout});
    std::vector<float> one(cmax, 1.f);
    if (int rc = talloc(t, &t->ones, cmax)) return rc;
    if (int rc = talloc(t, &t->zeros, cmax)) return rc;
    AVSE_HIP_CHECK(hipMemcpy(t->ones, one.data(), cmax * sizeof(float), hipMemcpyHostToDevice));
    const long long spec = (long long)kMels * t->plan.T;
    if (int rc = talloc(t, &t->in_audio, N * spec * 8)) return rc;
    if (int rc = talloc(t, &t->in_video, N * 128 * 128 * 8)) return rc;
    if (int rc = talloc(t, &t->concat, N * t->plan.cat)) return rc;
    if (int rc = talloc(t, &t->g6, N * spec * 8)) return rc;
    long long zmax = 0, red = 0, wmax = 0;
    for (int i = 0; i < kNumLayers; ++i) {
        TLayer& T = t->layers[i];
        const LayerDef& L = T.L;
        T.zc = (L.cout % 8 && L.kind != DENSE) ? ((L.cout + 7) / 8) * 8 : L.cout;
        const long long zel = N * T.hq * T.wq * T.zc;
        zmax = std::max(zmax, zel);
        if (int rc = talloc(t, &T.z, zel)) return rc;
        if (L.bn) {
            if (int rc = talloc(t, &T.mean, L.bn_channels)) return rc;
            if (int rc = talloc(t, &T.inv, L.bn_channels)) return rc;
        }
        const long long rows = N * T.hq * T.wq * (L.kind == DENSE ? L.cout / std::max(L.bn_channels, 1) : 1);
        red = std::max(red, 2 * ((rows + 4095) / 4096 + 1) * (long long)std::max(L.cout, 64));
    }
    for (int i = 0; i < kNumLayers; ++i) {   // after zc: wg_splits reads the grids
        const TLayer& T = t->layers[i];
        long long mx = 0;
        for (int64_t n = 1; n <= N; n = (n < N && 2 * n > N) ? N : 2 * n) mx = std::max(mx, wg_splits(T, n));
        wmax = std::max(wmax, (long long)T.L.kh * T.L.kw * T.L.cin * T.L.cout * mx);
    }
    if (int rc = talloc(t, &t->ghat, zmax)) return rc;
    t->red_floats = std::max(red, 2LL * (2048 + 64) * 64 + 4096);   // colred's nblk * C <= (2048 + 64) * 64 (x2 MODE 2)
    if (int rc = talloc(t, &t->red, t->red_floats)) return rc;
    if (int rc = talloc(t, &t->kpart, kSplitTiles * 128LL * 128)) return rc;
    t->wpart_floats = wmax;
    if (int rc = talloc(t, &t->wpart, wmax)) return rc;
    if (int rc = talloc(t, &t->loss, 1)) return rc;
    // layer inputs: the previous layer's output tensor; the first layers read the prepared inputs
    for (int i = 0; i < kNumLayers; ++i) {
        TLayer& T = t->layers[i];
        const LayerDef& L = T.L;
        if (i == 0) { T.in = t->in_audio; T.in_clip = (long long)kMels * t->plan.T * 8; }
        else if (std::strcmp(L.name, "v_conv1") == 0) { T.in = t->in_video; T.in_clip = 128 * 128 * 8; }
        else if (std::strcmp(L.name, "enc_dense") == 0) { T.in = t->concat; T.in_clip = t->plan.cat; }
        else {
            const long long el = (long long)L.hin * L.win * T.cin_pad;
            if (int rc = talloc(t, &T.in, N * el)) return rc;
            T.in_clip = el;
        }
        if (T.dgrad) {
            if (int rc = talloc(t, &T.gin, N * T.in_clip)) return rc;
        }
    }
    return 0;
}

// where layer i's output goes (and its gradient comes from): next input, or the concat buffer
void out_view(avse_trainer* t, int i, float** buf, float** gbuf, long long* clip, int* pix, int* coff) {
    const TLayer& T = t->layers[i];
    const char* nm = T.L.name;
    *pix = std::strcmp(nm, "dec_dense2") == 0 ? 128 : T.L.cout;   // dec_dense2: Reshape(5, 5, 128) (network.py:76)
    if (std::strcmp(nm, "a_conv5") == 0 || std::strcmp(nm, "v_conv6") == 0) {
        const TLayer& E = t->layers[11];   // enc_dense
        *buf = t->concat;
        *gbuf = E.gin;
        *clip = t->plan.cat;
        *coff = std::strcmp(nm, "a_conv5") == 0 ? 0 : t->plan.aemb;
        return;
    }
    const TLayer& Nx = t->layers[i + 1];
    *buf = Nx.in;
    *gbuf = Nx.gin;
    *clip = Nx.in_clip;
    *coff = 0;
}

ConvArgs fwd_args(avse_trainer* t, const TLayer& T, int64_t N) {
    const LayerDef& L = T.L;
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.in = T.in;
    a.out = T.z;
    a.w = t->wfwd + T.fw_off;
    a.scale = t->ones;
    a.shift = t->P + T.o_b;
    a.taps = T.d_taps;
    a.N = (int)N;
    a.Hi = L.hin;
    a.Wi = L.win;
    a.Ci = T.cin_pad;
    a.in_clip_stride = T.in_clip;
    a.Hq = (L.kind == DECONV) ? L.hin : T.hq;
    a.Wq = (L.kind == DECONV) ? L.win : T.wq;
    a.sy = (L.kind == CONV) ? L.sh : 1;
    a.sx = (L.kind == CONV) ? L.sw : 1;
    a.oys = (L.kind == DECONV) ? L.sh : 1;
    a.oxs = (L.kind == DECONV) ? L.sw : 1;
    a.Ho = T.hq;
    a.Wo = T.wq;
    a.Co = L.cout;
    a.out_clip_stride = (long long)T.hq * T.wq * T.zc;
    a.out_pix_stride = T.zc;
    a.out_c_off = 0;
    a.pool = 0;
    a.act = 0;
    a.nphase = T.nphase;
    a.ksplit = 1;
    for (int p = 0; p < T.nphase; ++p) a.ph[p] = T.ph[p];
    return a;
}

ConvArgs dgrad_args(avse_trainer* t, const TLayer& T, const float* dz, int64_t N) {
    const LayerDef& L = T.L;
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.in = dz;
    a.out = T.gin;
    a.w = t->wdg + T.dg_off;
    a.scale = t->ones;
    a.shift = t->zeros;
    a.taps = T.d_dg_taps;
    a.N = (int)N;
    a.Hi = T.hq;
    a.Wi = T.wq;
    a.Ci = T.dg_ci;
    a.in_clip_stride = (long long)T.hq * T.wq * T.zc;
    a.Hq = (L.kind == DENSE) ? 1 : T.dg_hq;
    a.Wq = (L.kind == DENSE) ? 1 : T.dg_wq;
    a.sy = T.dg_sy;
    a.sx = T.dg_sx;
    a.oys = T.dg_oys;
    a.oxs = T.dg_oxs;
    a.Ho = L.hin;
    a.Wo = L.win;
    a.Co = L.cin;
    a.out_clip_stride = T.in_clip;
    a.out_pix_stride = T.cin_pad;
    a.out_c_off = 0;
    a.pool = 0;
    a.act = 0;
    a.nphase = T.dg_nphase;
    a.ksplit = 1;
    for (int p = 0; p < T.dg_nphase; ++p) a.ph[p] = T.dg_ph[p];
    return a;
}

// row blocks of a column reduction (k_colreduce, k_bn_bwd_colsum): ~2048 blocks of 64 columns x >= 64 rows
// (v_conv1's 262k-row reductions ran on 128 blocks: 10 of 19.7 ms/step)
void colred_grid(long long M, int C, long long* nblk_out, long long* rpb_out) {
    const long long cblk = (C + 63) / 64;
    long long nblk = std::min(std::max(1LL, 2048 / cblk), std::max(1LL, (M + 63) / 64));
    const long long rpb = (M + nblk - 1) / nblk;
    *nblk_out = (M + rpb - 1) / rpb;
    *rpb_out = rpb;
}

// column reduction + finish; returns status
template <int MODE, int STAGE>
int colred(avse_trainer* t, const float* x, int ld, const float* z, const float* mean, const float* inv, long long M, int C,
           float* fmean, float* finv, float* mm, float* mv, float* o0, float* o1, hipStream_t s) {
    long long nblk, rpb;
    colred_grid(M, C, &nblk, &rpb);
    if ((MODE == 2 ? 2 : 1) * nblk * (long long)C > t->red_floats) return tfail(AVSE_ERR_INVALID, "reduction workspace too small");
    hipLaunchKernelGGL(k_colreduce<MODE>, dim3((C + 63) / 64, (unsigned)nblk), dim3(256), 0, s, x, ld, z, mean, inv, M, C, rpb, t->red);
    AVSE_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_colfinish<STAGE>, dim3(C), dim3(256), 0, s, t->red, (int)nblk, C, M, fmean, finv, mm, mv, o0, o1);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

// Split-K for the short grids of a training batch (fp32): at batch 16 the forward and input-gradient launches of
// v_conv4..v_conv6 and the dense layers ran 11-64 workgroups (one 128-row tile of 16 clips for enc_dense) over K up to
// 5,248.  Each split is exactly one block of k_conv's blocked fp32 summation (kFp32Block slabs) and
// k_splitk_reduce_tiles adds the splits in order, so every sum is the unsplit kernel's bit for bit: ((0 + b0) + b1)
// + ... either way.  (A split on the inference planner's rule — a few long splits — moved forward values within
// rounding of a LeakyReLU kink or pool tie to the other side: 1.7e-2 on the upstream video gradients of the
// test_gradients_match_oracle fixture)  Launches with >= 256 tiles, more than kSplitTiles
// tile-splits, or a slab count whose even split is not exactly one block stay unsplit.
void train_split(avse_trainer* t, ConvArgs& a) {
    if (a.nphase != 1) return;
    const long long M = (long long)a.N * a.Hq * a.Wq;
    const int BN = a.Co <= 64 ? 64 : 128;
    const long long tiles = ((M + 127) / 128) * ((a.Co + BN - 1) / BN);
    if (tiles >= 256) return;
    const int nslab = a.ph[0].kpad / 16;
    const int ks = (nslab + kFp32Block - 1) / kFp32Block;
    if (ks < 2 || (nslab + ks - 1) / ks != kFp32Block || tiles * ks > kSplitTiles) return;
    a.ksplit = ks;
    a.partial = t->kpart;
}

int wgrad(avse_trainer* t, const TLayer& T, const float* dz, int64_t N, hipStream_t s) {
    const LayerDef& L = T.L;
    WgArgs w;
    std::memset(&w, 0, sizeof(w));
    w.N = (int)N;
    w.ntaps = L.kh * L.kw;
    w.taps = T.d_wg_taps;
    if (L.kind == DECONV) {   // G = dz on the output grid (stride s), H = input
        w.G = dz; w.Hg = T.hq; w.Wg = T.wq; w.gcs = T.zc; w.g_clip = (long long)T.hq * T.wq * T.zc;
        w.H = T.in; w.Hh = L.hin; w.Wh = L.win; w.hcs = T.cin_pad; w.h_clip = T.in_clip;
        w.sy = L.sh; w.sx = L.sw;
        w.A = L.cout; w.B = L.cin;
    } else {                  // G = input (stride s), H = dz on the conv grid
        w.G = T.in; w.Hg = L.hin; w.Wg = L.win; w.gcs = T.cin_pad; w.g_clip = T.in_clip;
        w.H = dz; w.Hh = T.hq; w.Wh = T.wq; w.hcs = T.zc; w.h_clip = (long long)T.hq * T.wq * T.zc;
        w.sy = (L.kind == CONV) ? L.sh : 1; w.sx = (L.kind == CONV) ? L.sw : 1;
        w.A = L.cin; w.B = L.cout;
    }
    const long long R = N * (long long)w.Hh * w.Wh;
    if (R >= (1LL << 31)) return tfail(AVSE_ERR_UNSUPPORTED, "wgrad: batch x grid exceeds 2^31 rows");
    const long long tiles = (long long)((w.A + 63) / 64) * ((w.B + 63) / 64) * w.ntaps;
    long long splits = wg_splits(T, N);
    const long long per = (long long)w.ntaps * w.A * w.B;
    if (splits * per > t->wpart_floats) return tfail(AVSE_ERR_INVALID, "wgrad workspace too small");
    w.rows_per_split = ((R + splits - 1) / splits + 31) / 32 * 32;
    splits = (R + w.rows_per_split - 1) / w.rows_per_split;
    w.part = t->wpart;
    if (wg_all_taps(T))
        hipLaunchKernelGGL(k_wgrad_nat, dim3((unsigned)((w.B + 127) / 128), 1, (unsigned)splits), dim3(256), 0, s, w);
    else if (w.A <= 8)
        hipLaunchKernelGGL(k_wgrad_na, dim3((unsigned)((w.B + 127) / 128), (unsigned)w.ntaps, (unsigned)splits), dim3(256), 0, s, w);
    else
        hipLaunchKernelGGL(k_wgrad, dim3((unsigned)(tiles / w.ntaps), (unsigned)w.ntaps, (unsigned)splits), dim3(256), 0, s, w);
    AVSE_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_sum_splits, dim3((unsigned)std::min<long long>((per + 63) / 64, 8192)), dim3(256), 0, s,
                       (const float*)t->wpart, (int)splits, per, t->Gr + T.o_k);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int step_impl(avse_trainer* t, const float* audio, const float* video, const float* target, const float* vmean,
              const float* vstd, int64_t N, float lr, float drop, uint32_t seed, int flags, float* loss, hipStream_t s) {
    // ---- weight packings from the current parameters ----
    hipLaunchKernelGGL(k_pack, dim3((unsigned)t->n_pack_tiles), dim3(256), 0, s, t->wfwd, t->wdg, (const float*)t->P,
                       (const PackTile*)t->pack_tiles);
    AVSE_HIP_CHECK(hipGetLastError());
    AVSE_HIP_CHECK(hipMemsetAsync(t->Gr, 0, sizeof(float) * t->nparams, s));
    // ---- inputs ----
    const long long spec = (long long)kMels * t->plan.T;
    hipLaunchKernelGGL(k_prep_audio, dim3(grid_for(N * spec)), dim3(256), 0, s, audio, t->in_audio, (long long)N * spec);
    hipLaunchKernelGGL(k_prep_video, dim3(grid_for(N * 16384)), dim3(256), 0, s, video, vmean, vstd, t->in_video,
                       (long long)N * 16384, 16384, t->plan.F);
    AVSE_HIP_CHECK(hipGetLastError());
    // ---- forward ----
    for (int i = 0; i < kNumLayers; ++i) {
        TLayer& T = t->layers[i];
        const LayerDef& L = T.L;
        ConvArgs a = fwd_args(t, T, N);
        train_split(t, a);
        if (int rc = launch_conv(a, AVSE_F32, s)) return rc;
        if (!L.bn) continue;
        const int C = L.bn_channels;
        const long long M = N * (long long)T.hq * T.wq * (L.cout / C);
        float* P = t->P;
        {   // batch statistics in one pass over z (per-block sums + deviations about the block mean) + one finish
            long long nblk, rpb;
            colred_grid(M, C, &nblk, &rpb);
            if (2 * nblk * (long long)C > t->red_floats) return tfail(AVSE_ERR_INVALID, "reduction workspace too small");
            hipLaunchKernelGGL(k_colreduce<3>, dim3((C + 63) / 64, (unsigned)nblk), dim3(256), 0, s, (const float*)T.z, C,
                               nullptr, nullptr, nullptr, M, C, rpb, t->red);
            AVSE_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_bnstat_finish, dim3(C), dim3(256), 0, s, (const float*)t->red, (int)nblk, C, M, rpb, T.mean,
                               T.inv, P + T.o_mm, P + T.o_mv);
            AVSE_HIP_CHECK(hipGetLastError());
        }
        ActArgs aa;
        std::memset(&aa, 0, sizeof(aa));
        aa.z = T.z; aa.N = (int)N; aa.C = C;
        aa.Hq = (L.kind == DENSE) ? ((std::strcmp(L.name, "dec_dense2") == 0) ? 5 : 1) : T.hq;
        aa.Wq = (L.kind == DENSE) ? ((std::strcmp(L.name, "dec_dense2") == 0) ? t->plan.W5 : 1) : T.wq;
        aa.mean = T.mean; aa.inv = T.inv; aa.gamma = P + T.o_g; aa.beta = P + T.o_be;
        aa.pool = L.pool ? 1 : 0;
        aa.drop = L.pool ? drop : 0.f;   // Dropout(0.25) follows each video pooling (network.py:142-174)
        aa.seed = seed; aa.layer = (uint32_t)i;
        float* gdummy;
        out_view(t, i, &aa.out, &gdummy, &aa.out_clip, &aa.out_pix, &aa.out_c);
        const long long total = N * (long long)aa.Hq * aa.Wq * C / (aa.pool ? 4 : 1);
        hipLaunchKernelGGL(k_act_fwd, dim3(grid_for(total)), dim3(256), 0, s, aa);
        AVSE_HIP_CHECK(hipGetLastError());
    }
    // ---- loss ----
    TLayer& D6 = t->layers[kNumLayers - 1];
    const long long nout = N * spec;
    const unsigned lb = grid_for(nout, 256, 1024);
    hipLaunchKernelGGL(k_mse, dim3(lb), dim3(256), 0, s, (const float*)D6.z, target, nout, D6.zc, t->g6, t->red);
    hipLaunchKernelGGL(k_mse_finish, dim3(1), dim3(64), 0, s, (const float*)t->red, (int)lb, nout, t->loss);
    AVSE_HIP_CHECK(hipGetLastError());
    if (loss) AVSE_HIP_CHECK(hipMemcpyAsync(loss, t->loss, sizeof(float), hipMemcpyDeviceToDevice, s));
    // ---- backward ----
    for (int i = kNumLayers - 1; i >= 0; --i) {
        TLayer& T = t->layers[i];
        const LayerDef& L = T.L;
        float* dz;
        const long long Mfull = N * (long long)T.hq * T.wq;
        bool bias_fused = false;
        if (!L.bn) {
            dz = t->g6;   // dL/dy with the output's 8-channel stride
        } else {
            const int C = L.bn_channels;
            const long long M = Mfull * (L.cout / C);
            ActArgs aa;
            std::memset(&aa, 0, sizeof(aa));
            aa.z = T.z; aa.N = (int)N; aa.C = C;
            aa.Hq = (L.kind == DENSE) ? ((std::strcmp(L.name, "dec_dense2") == 0) ? 5 : 1) : T.hq;
            aa.Wq = (L.kind == DENSE) ? ((std::strcmp(L.name, "dec_dense2") == 0) ? t->plan.W5 : 1) : T.wq;
            aa.mean = T.mean; aa.inv = T.inv; aa.gamma = t->P + T.o_g; aa.beta = t->P + T.o_be;
            aa.pool = L.pool ? 1 : 0;
            aa.drop = L.pool ? drop : 0.f;
            aa.seed = seed; aa.layer = (uint32_t)i;
            float *obuf, *gbuf;
            long long gclip;
            int gpix, gc;
            out_view(t, i, &obuf, &gbuf, &gclip, &gpix, &gc);
            const long long total = N * (long long)aa.Hq * aa.Wq * C / (aa.pool ? 4 : 1);
            hipLaunchKernelGGL(k_act_bwd, dim3(grid_for(total)), dim3(256), 0, s, aa, (const float*)gbuf, gclip, gpix, gc, t->ghat);
            AVSE_HIP_CHECK(hipGetLastError());
            if (int rc = colred<2, 2>(t, t->ghat, C, T.z, T.mean, T.inv, M, C, nullptr, nullptr, nullptr, nullptr,
                                      t->Gr + T.o_be, t->Gr + T.o_g, s)) return rc;
            bias_fused = (L.cout == C && T.zc == C);
            if (bias_fused) {   // dz and the bias gradient's column partials in one pass
                long long nblk, rpb;
                colred_grid(M, C, &nblk, &rpb);
                if (nblk * (long long)C > t->red_floats) return tfail(AVSE_ERR_INVALID, "reduction workspace too small");
                hipLaunchKernelGGL(k_bn_bwd_colsum, dim3((C + 63) / 64, (unsigned)nblk), dim3(256), 0, s, (const float*)T.z,
                                   t->ghat, M, C, (const float*)T.mean, (const float*)T.inv, (const float*)(t->P + T.o_g),
                                   (const float*)(t->Gr + T.o_be), (const float*)(t->Gr + T.o_g), rpb, t->red);
                AVSE_HIP_CHECK(hipGetLastError());
                hipLaunchKernelGGL(k_colfinish<3>, dim3(C), dim3(256), 0, s, (const float*)t->red, (int)nblk, C, M, nullptr,
                                   nullptr, nullptr, nullptr, t->Gr + T.o_b, nullptr);
            } else {
                hipLaunchKernelGGL(k_bn_bwd, dim3(grid_for(M * C)), dim3(256), 0, s, (const float*)T.z, t->ghat, M, C,
                                   (const float*)T.mean, (const float*)T.inv, (const float*)(t->P + T.o_g),
                                   (const float*)(t->Gr + T.o_be), (const float*)(t->Gr + T.o_g));
            }
            AVSE_HIP_CHECK(hipGetLastError());
            dz = t->ghat;
            if ((flags & AVSE_TRAIN_DEBUG_STOP) && (flags >> 8) == i) return 0;   // debug: dz of layer i in ghat
        }
        // bias: sum of dz over every pixel (per output channel)
        if (!bias_fused)
            if (int rc = colred<0, 3>(t, dz, T.zc, nullptr, nullptr, nullptr, Mfull, L.cout, nullptr, nullptr, nullptr, nullptr,
                                      t->Gr + T.o_b, nullptr, s)) return rc;
        if (int rc = wgrad(t, T, dz, N, s)) return rc;
        if (T.dgrad) {
            ConvArgs a = dgrad_args(t, T, dz, N);
            train_split(t, a);
            if (int rc = launch_conv(a, AVSE_F32, s)) return rc;
            if ((flags & AVSE_TRAIN_DEBUG_GIN) && (flags >> 8) == i) {   // debug: dL/d(input) of layer i in the scratch
                AVSE_HIP_CHECK(hipMemcpyAsync(t->ghat, T.gin, sizeof(float) * N * T.in_clip, hipMemcpyDeviceToDevice, s));
                return 0;
            }
        }
    }
    if (flags & 1) return 0;   // gradients only
    // ---- Adam ----
    t->step += 1;
    const double b1 = 0.9, b2 = 0.999;
    const double lr_t = (double)lr * std::sqrt(1.0 - std::pow(b2, (double)t->step)) / (1.0 - std::pow(b1, (double)t->step));
    hipLaunchKernelGGL(k_adam, dim3(grid_for(t->nparams)), dim3(256), 0, s, t->P, (const float*)t->Gr, t->Mo, t->Vo,
                       (long long)t->nparams, (float)lr_t, (float)b1, (float)b2, 1e-8f);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int avse_trainer_create(avse_ctx* c, const float* host_blob, int64_t n_floats, int64_t max_batch, avse_trainer** out) {
    return avse_trainer_create_shape(c, host_blob, n_floats, max_batch, kPlan25.T, kPlan25.F, out);
}

int avse_trainer_create_shape(avse_ctx* c, const float* host_blob, int64_t n_floats, int64_t max_batch, int spec_frames,
                              int video_frames, avse_trainer** out) {
    if (!c || !host_blob || !out) return tfail(AVSE_ERR_INVALID, "NULL argument");
    if (!plan_valid(spec_frames, video_frames)) return tfail(AVSE_ERR_UNSUPPORTED, "unsupported network shape");
    const NetPlan plan = make_plan(spec_frames, video_frames);
    if (n_floats != blob_floats(plan)) return tfail(AVSE_ERR_INVALID, "weight blob has the wrong size");
    // <= 1023 keeps every activation tensor (v_conv1's pre-pool z: 128 x 128 x 128 per clip) below 2^31 elements,
    // so the element-wise kernels index in 32 bits
    if (max_batch < 1 || max_batch > 1023) return tfail(AVSE_ERR_INVALID, "max_batch must be in [1, 1023]");
    auto* t = new avse_trainer();
    t->plan = plan;
    t->device = ctx_device_index(c);
    t->max_n = max_batch;
    int rc = hipSetDevice(t->device) == hipSuccess ? 0 : tfail(AVSE_ERR_HIP, "hipSetDevice failed");
    if (!rc) rc = build_plan(t, host_blob);
    if (!rc) rc = alloc_tensors(t);
    if (rc) {
        avse_trainer_destroy(t);
        return rc;
    }
    *out = t;
    return 0;
}

void avse_trainer_destroy(avse_trainer* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    for (void* p : t->allocs) (void)hipFree(p);
    delete t;
}

int avse_trainer_step(avse_trainer* t, const float* audio, const float* video, const float* target, const float* vnorm_mean,
                      const float* vnorm_std, int64_t N, float lr, float dropout_rate, uint32_t dropout_seed, int flags,
                      float* loss, void* stream) {
    if (!t || !audio || !video || !target) return tfail(AVSE_ERR_INVALID, "NULL argument");
    if (N < 1 || N > t->max_n) return tfail(AVSE_ERR_INVALID, "batch size outside [1, max_batch]");
    if ((vnorm_mean == nullptr) != (vnorm_std == nullptr)) return tfail(AVSE_ERR_INVALID, "vnorm_mean / vnorm_std: both or neither");
    if (!(dropout_rate >= 0.f && dropout_rate < 1.f)) return tfail(AVSE_ERR_INVALID, "dropout_rate must be in [0, 1)");
    AVSE_HIP_CHECK(hipSetDevice(t->device));
    return step_impl(t, audio, video, target, vnorm_mean, vnorm_std, N, lr, dropout_rate, dropout_seed, flags, loss,
                     (hipStream_t)stream);
}

int avse_trainer_read(avse_trainer* t, int what, float* host_blob, int64_t n_floats) {
    if (!t || !host_blob) return tfail(AVSE_ERR_INVALID, "NULL argument");
    if (n_floats != t->nparams && !(what == AVSE_TRAIN_DEBUG_DZ && n_floats <= t->nparams))
        return tfail(AVSE_ERR_INVALID, "blob size mismatch");
    const float* src = what == AVSE_TRAIN_PARAMS ? t->P : what == AVSE_TRAIN_GRADS ? t->Gr : what == AVSE_TRAIN_ADAM_M ? t->Mo
                       : what == AVSE_TRAIN_ADAM_V ? t->Vo : nullptr;
    if (what == AVSE_TRAIN_DEBUG_DZ) {   // debug: the head of the dz scratch (see AVSE_TRAIN_DEBUG_STOP)
        AVSE_HIP_CHECK(hipSetDevice(t->device));
        AVSE_HIP_CHECK(hipDeviceSynchronize());
        AVSE_HIP_CHECK(hipMemcpy(host_blob, t->ghat, sizeof(float) * n_floats, hipMemcpyDeviceToHost));
        return 0;
    }
    if (!src) return tfail(AVSE_ERR_INVALID, "unknown trainer buffer");
    AVSE_HIP_CHECK(hipSetDevice(t->device));
    AVSE_HIP_CHECK(hipDeviceSynchronize());
    AVSE_HIP_CHECK(hipMemcpy(host_blob, src, sizeof(float) * n_floats, hipMemcpyDeviceToHost));
    return 0;
}

int avse_trainer_iterations(avse_trainer* t, int64_t* iterations) {
    if (!t || !iterations) return tfail(AVSE_ERR_INVALID, "NULL argument");
    *iterations = t->step;
    return 0;
}

}  // extern "C"
