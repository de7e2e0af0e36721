// Prototype (not in the library): a windowed form of the generic split-pair layer kernel at d_deconv4's shape, to
// measure what DESIGN.md §8 item 3 proposes.  k_conv (conv.hip) gathers its A operand per tap from global memory (the
// im2col re-reads: 41 % of its time at this shape, tools/kconv_ablate.hip); here each 128-row M tile stages, per
// 16-channel pair chunk, the input window its rows need for all 16 taps in LDS once, and every tap's A fragments are
// read from it at a per-lane base + a uniform tap offset.  B (weights) as in k_conv: register-staged slabs through an
// LDS ring, one barrier per slab; the K order is chunk-outer, tap-inner; fp32 blocked summation over 8-slab blocks.
// Compares its output with k_conv's on the same inputs (different summation order: relative RMS ~1e-7) and times both.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/win_proto.bin tools/conv_win_proto.hip && tools/win_proto.bin
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/conv.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
}  // namespace avse

using namespace avse;

namespace {
constexpr int H = 40, W = 10, HWc = H * W, CI = 128, CO = 64, NT = 16, NCH = CI / 16;   // 16-ch pair chunks
constexpr int CIH = 2 * CI, KPH = NT * CIH;           // halves per pixel / per weight row
constexpr int WP = 14;                                 // window pitch (13 columns: x - 2 .. x + 1 over 0..9, + 1)
constexpr int BNW = 64, BSL = BNW * 64;                // B slab bytes
// TM-row tiles (128: 4 waves, 256: 8 waves sharing every weight slab): window rows capacity = the tile's image rows
// (<= TM / W + 2 over two clips) + 2 x 4 halo rows
template <int TM> struct WinGeom {
    static constexpr int NTH = TM * 2, WROWS = TM / W + 2 + 8, WIN = WROWS * WP * 64;
    static constexpr int NPIECE = (WROWS * WP * 4 + NTH - 1) / NTH, LDS = 2 * WIN + 3 * BSL;
};

__device__ __forceinline__ int bswz(int row) { return ((row >> 3) & 1) * 3; }
// window pixel p's 16-B slots rotate every 4 pixels: 16 lanes reading 16 neighbouring pixels hit 16 distinct bank quads
#ifndef WIN_SWZ
#define WIN_SWZ 0
#endif
__device__ __forceinline__ int wsw(int p) { return WIN_SWZ ? (p >> 2) & 3 : 0; }

// grid: ceil(M / TM) tiles; TM / 32 waves (TM / 64 x 2: 64 rows x 32 columns each)
template <int TM>
__global__ __launch_bounds__(TM * 2, TM == 128 ? 3 : 2) void k_win4(ConvArgs a) {
    using G = WinGeom<TM>;
    constexpr int NTH = G::NTH, WROWS = G::WROWS, WIN = G::WIN, NPIECE = G::NPIECE;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char* const win = lds;                 // [2][WIN]
    char* const bs = lds + 2 * WIN;        // [3][BSL]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
    const int fr = lane & 15, fg = lane >> 4;
    const int M = a.N * HWc;
    const int m0 = blockIdx.x * TM;
    // the tile's rows span clip c0 (pixels p0 ..) and possibly c0 + 1
    const int c0 = m0 / HWc, p0 = m0 - c0 * HWc;
    const int last = min(m0 + TM - 1, M - 1);
    const int c1 = last / HWc;
    const int ylo0 = p0 / W, yhi0 = (c1 == c0) ? (last - c0 * HWc) / W : H - 1;
    const int n0 = yhi0 - ylo0 + 4;                              // window rows of region 0: ylo0 - 2 .. yhi0 + 1
    const int yhi1 = (c1 != c0) ? (last - c1 * HWc) / W : -1;
    const int n1 = c1 != c0 ? yhi1 + 4 : 0;                      // region 1: -2 .. yhi1 + 1
    const long long clip_b = (long long)HWc * CIH * 2;
    const __amdgpu_buffer_rsrc_t rsA = make_rsrc(reinterpret_cast<const char*>(a.in) + c0 * clip_b, (a.N - c0) * clip_b);
    const __amdgpu_buffer_rsrc_t rsB = make_rsrc(a.w, (long long)CO * KPH * 2);

    // window pieces of this thread (source byte offset for chunk 0, or kOOB), destination offsets
    int psrc[NPIECE], pdst[NPIECE];
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) {
        const int q = tid + NTH * k, p = q >> 2, qq = q & 3;
        const int wrow = p / WP, wcol = p - wrow * WP;
        int src = kOOB;
        if (wrow < n0 + n1) {
            const int R = wrow < n0 ? 0 : 1;
            const int iy = (R == 0 ? ylo0 - 2 + wrow : -2 + wrow - n0), ix = wcol - 2;
            if (iy >= 0 && iy < H && ix >= 0 && ix < W && wcol < 13)
                src = (int)((R * clip_b) + ((long long)(iy * W + ix) * CIH + qq * 8) * 2);
        }
        psrc[k] = wrow < WROWS ? src : kOOB;
        pdst[k] = wrow < WROWS ? p * 64 + ((qq ^ wsw(p)) << 4) : -1;
    }
    // per-lane A base of fragment i (tap-independent): window pixel of (y + 2, x + 2) in the row's region
    int abase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int m = m0 + wm * 64 + 16 * i + fr;
        m = min(m, M - 1);
        const int c = m / HWc, pp = m - c * HWc, y = pp / W, x = pp - y * W;
        const int wrow = c == c0 ? (y - ylo0 + 2) : (n0 + y + 2);
        abase[i] = wrow * WP + x + 2;   // window pixel at tap (0, 0)
    }
    // B: thread's 16-B piece of the slab: row tid >> 2, chunk tid & 3
    const int brow = (tid & 255) >> 2, bg = tid & 3;
    const int bsrc = brow * KPH * 2 + bg * 16, bdst = brow * 64 + ((bg ^ bswz(brow)) << 4);
    auto bslab_off = [](int s) { const int c = s / NT, t = s - c * NT; return t * CIH * 2 + c * 64; };
    constexpr int NS = NCH * NT;   // 128 slabs

    float esc[2], esh[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = wn * 32 + 16 * j + fr;
        esc[j] = a.scale[n];
        esh[j] = a.shift[n];
    }

    // prologue: window of chunk 0 -> buffer 0, B slabs 0, 1, 2 in registers, slab 0 -> LDS
    {
        i32x4 pc[NPIECE];
#pragma unroll
        for (int k = 0; k < NPIECE; ++k) pc[k] = __builtin_amdgcn_raw_buffer_load_b128(rsA, psrc[k], 0, 0);
#pragma unroll
        for (int k = 0; k < NPIECE; ++k)
            if (pdst[k] >= 0) *reinterpret_cast<i32x4*>(win + pdst[k]) = pc[k];
    }
    i32x4 rb[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) rb[p] = __builtin_amdgcn_raw_buffer_load_b128(rsB, bsrc + bslab_off(p), 0, 0);
    const bool bl = tid < 256;   // the weight slab (4 KB) is 256 x 16 B
    if (bl) *reinterpret_cast<i32x4*>(bs + bdst) = rb[0];
    rb[0] = __builtin_amdgcn_raw_buffer_load_b128(rsB, bl ? bsrc + bslab_off(3) : kOOB, 0, 0);
    __syncthreads();

    f32x4 acc[4][2], part[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int nblk = 0;
    i32x4 pw[NPIECE];   // next chunk's window pieces
    auto step = [&](auto qidx, int s) {
        constexpr int q = decltype(qidx)::value, qn = (q + 1) % 3;
        const int c = s / NT, t = s - c * NT;
        const int dy = 1 - t / 4, dx = 1 - t % 4;
        const char* wb = win + (c & 1) * WIN;
        const int toff = dy * WP + dx;
        if (t == 0 && c + 1 < NCH) {
#pragma unroll
            for (int k = 0; k < NPIECE; ++k) pw[k] = __builtin_amdgcn_raw_buffer_load_b128(rsA, psrc[k], (c + 1) * 64, 0);
        }
        i32x4 fa[4], fb[2], fl[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = abase[i] + toff;
            fa[i] = *reinterpret_cast<const i32x4*>(wb + p * 64 + ((fg ^ wsw(p)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = wn * 32 + 16 * j + fr;
            fb[j] = *reinterpret_cast<const i32x4*>(bs + q * BSL + row * 64 + (((fg & 1) ^ bswz(row)) << 4));
            fl[j] = *reinterpret_cast<const i32x4*>(bs + q * BSL + row * 64 + (((2 + (fg & 1)) ^ bswz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa[i]),
                                                                    __builtin_bit_cast(f16x8, fb[j]), part[i][j], 0, 0, 0);
                part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa[i]),
                                                                    __builtin_bit_cast(f16x8, fl[j]), part[i][j], 0, 0, 0);
            }
        if (++nblk == 8) {
            nblk = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] += part[i][j];
                    part[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
                }
        }
        // B slab s + 1 -> LDS (buffer qn held slab s - 2, read before the barrier of step s - 2); refill with s + 4
        if (bl) *reinterpret_cast<i32x4*>(bs + qn * BSL + bdst) = rb[qn];
        rb[qn] = __builtin_amdgcn_raw_buffer_load_b128(rsB, bl ? bsrc + bslab_off(min(s + 4, NS - 1)) : kOOB, 0, 0);
        if (t == NT - 1 && c + 1 < NCH) {   // next chunk's window -> the other buffer (read last during chunk c - 1)
#pragma unroll
            for (int k = 0; k < NPIECE; ++k)
                if (pdst[k] >= 0) *reinterpret_cast<i32x4*>(win + ((c + 1) & 1) * WIN + pdst[k]) = pw[k];
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
        for (int j = 0; j < 2; ++j) acc[i][j] += part[i][j];
    // epilogue: BN + LeakyReLU, split pair store (as k_conv's store_val with out_s16)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int mb = m0 + wm * 64 + 16 * i + 4 * fg;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = mb + r;
            if (m >= M) continue;
            const int c = m / HWc, pp = m - c * HWc;
            const long long rowbase = c * a.out_clip_stride + (long long)pp * a.out_pix_stride + a.out_c_off;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = wn * 32 + 16 * j + fr;
                float x = acc[i][j][r] * esc[j] + esh[j];
                x = x >= 0.f ? x : 0.3f * x;
                _Float16* o = reinterpret_cast<_Float16*>(a.out) + rowbase + 32 * (n >> 4) + (n & 15);
                const _Float16 h = (_Float16)x;
                o[0] = h;
                o[16] = (_Float16)(x - (float)h);
            }
        }
    }
}
}  // namespace

int main() {
    const int N = 512;
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.N = N; a.Hi = H; a.Wi = W; a.Ci = CIH; a.in_clip_stride = (long long)HWc * CIH;
    a.Hq = H; a.Wq = W; a.sy = a.sx = 1; a.oys = a.oxs = 1; a.Ho = H; a.Wo = W; a.Co = CO;
    a.out_clip_stride = (long long)HWc * 2 * CO; a.out_pix_stride = 2 * CO; a.out_c_off = 0;
    a.act = 1; a.nphase = 1; a.ksplit = 1; a.out_s16 = 1;
    a.ph[0].ntaps = NT; a.ph[0].kpad = KPH; a.ph[0].w_off = 0; a.ph[0].tap_off = 0;
    std::vector<int2> taps;
    for (int t = 0; t < NT; ++t) taps.push_back(make_int2(1 - t / 4, 1 - t % 4));
    void *in, *out, *out2, *w, *tp;
    float *sc, *sh;
    const size_t in_b = (size_t)N * HWc * CIH * 2, w_b = (size_t)CO * KPH * 2, out_b = (size_t)N * HWc * 2 * CO * 2;
    (void)hipMalloc(&in, in_b);
    (void)hipMalloc(&out, out_b);
    (void)hipMalloc(&out2, out_b);
    (void)hipMalloc(&w, w_b);
    (void)hipMalloc(&tp, NT * sizeof(int2));
    (void)hipMalloc(&sc, CO * 4);
    (void)hipMalloc(&sh, CO * 4);
    // inputs: fp32 values split into [h | l] pairs per 16 channels; weights likewise (magnitudes of a BN'd layer)
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xffff) / 65536.0f - 0.5f; };
    auto split_fill = [&](std::vector<_Float16>& v, size_t rows, int cols, float scale) {
        for (size_t r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c) {
                const float x = rnd() * scale;
                const _Float16 hh = (_Float16)x, ll = (_Float16)(x - (float)hh);
                const size_t base = r * 2 * cols + 32 * (c / 16) + c % 16;
                v[base] = hh;
                v[base + 16] = ll;
            }
    };
    std::vector<_Float16> hin(in_b / 2), hw(w_b / 2);
    split_fill(hin, (size_t)N * HWc, CI, 4.f);
    split_fill(hw, (size_t)CO * NT, CI, 2048.f);   // weight rows [co][tap][ci pairs]
    (void)hipMemcpy(in, hin.data(), in_b, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw.data(), w_b, hipMemcpyHostToDevice);
    (void)hipMemcpy(tp, taps.data(), NT * sizeof(int2), hipMemcpyHostToDevice);
    std::vector<float> scv(CO, 1.f / 2048.f), shv(CO, 0.01f);
    (void)hipMemcpy(sc, scv.data(), CO * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(sh, shv.data(), CO * 4, hipMemcpyHostToDevice);
    a.in = in; a.w = w; a.taps = reinterpret_cast<const int2*>(tp); a.scale = sc; a.shift = sh;
    (void)hipFuncSetAttribute((const void*)k_win4<128>, hipFuncAttributeMaxDynamicSharedMemorySize, WinGeom<128>::LDS);
    (void)hipFuncSetAttribute((const void*)k_win4<256>, hipFuncAttributeMaxDynamicSharedMemorySize, WinGeom<256>::LDS);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto time_it = [&](auto&& f) {
        for (int r = 0; r < 5; ++r) f();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 30; ++r) f();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 30;
    };
    ConvArgs a1 = a, a2 = a;
    a1.out = out;
    a2.out = out2;
    const float t_conv = time_it([&] { launch_conv(a1, kConvSplitPairs, 0); });
    const float t_win = time_it([&] {
        hipLaunchKernelGGL(k_win4<128>, dim3((N * HWc + 127) / 128), dim3(256), WinGeom<128>::LDS, 0, a2); });
    (void)hipDeviceSynchronize();
    std::vector<_Float16> o128(out_b / 2);
    (void)hipMemcpy(o128.data(), out2, out_b, hipMemcpyDeviceToHost);
    const float t_win256 = time_it([&] {
        hipLaunchKernelGGL(k_win4<256>, dim3((N * HWc + 255) / 256), dim3(512), WinGeom<256>::LDS, 0, a2); });
    const float t_conv2 = time_it([&] { launch_conv(a1, kConvSplitPairs, 0); });
    (void)hipDeviceSynchronize();
    std::vector<_Float16> o1(out_b / 2), o2(out_b / 2);
    (void)hipMemcpy(o1.data(), out, out_b, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o2.data(), out2, out_b, hipMemcpyDeviceToHost);
    double num = 0, den = 0, mx = 0;
    for (size_t px = 0; px < (size_t)N * HWc; ++px)
        for (int c = 0; c < CO; ++c) {
            const size_t b = px * 2 * CO + 32 * (c / 16) + c % 16;
            const double v1 = (double)(float)o1[b] + (double)(float)o1[b + 16];
            const double v2 = (double)(float)o2[b] + (double)(float)o2[b + 16];
            num += (v1 - v2) * (v1 - v2);
            den += v1 * v1;
            mx = std::fmax(mx, std::fabs(v1 - v2));
        }
    const double flop = 2.0 * N * HWc * CO * (double)CI * NT;
    std::printf("k_conv   %.4f / %.4f ms  %.1f TF/s\n", t_conv, t_conv2, flop / (t_conv * 1e-3) / 1e12);
    std::printf("k_win4<128> %.4f ms  %.1f TF/s  (LDS %d B)\n", t_win, flop / (t_win * 1e-3) / 1e12, WinGeom<128>::LDS);
    std::printf("k_win4<256> %.4f ms  %.1f TF/s  (LDS %d B); outputs bitwise equal to <128>: %s\n", t_win256,
                flop / (t_win256 * 1e-3) / 1e12, WinGeom<256>::LDS,
                std::memcmp(o128.data(), o2.data(), out_b) == 0 ? "yes" : "NO");
    std::printf("outputs: rel RMS %.3e, max abs diff %.3e, RMS %.3e  %s\n", std::sqrt(num / den), mx,
                std::sqrt(den / ((double)N * HWc * CO)), hipGetErrorString(hipGetLastError()));
    return 0;
}
