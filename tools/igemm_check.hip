// Standalone check of k_igemm's split-K partial sums (igemm.hip) on a dense-layer-shaped GEMM against a
// CPU reference: out[m][n] = sum_k A[m][k] * W[n][k] per K-split.   hipcc ... -o _igemm_check igemm_check.hip
#include <cmath>
#include <cstring>
#include <cstdio>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/igemm.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int launch_splitk_reduce(const ConvArgs&, int, hipStream_t) { return 0; }   // partials checked directly
}  // namespace avse
using namespace avse;

static uint16_t f2bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return u >> 16; }
static float bf2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; std::memcpy(&f, &u, 4); return f; }

int main() {
    const int M = 300, K = 640, Co = 200, KS = 4;
    std::vector<uint16_t> A((size_t)M * K), W((size_t)Co * K);
    uint32_t st = 1;
    auto rnd = [&] { st = st * 1664525u + 1013904223u; return ((st >> 9) & 0xffff) / 32768.f - 1.f; };
    for (auto& v : A) v = f2bf(rnd());
    for (auto& v : W) v = f2bf(rnd());
    void *dA, *dW, *dP, *dT, *dO;
    float *dS, *dH;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dW, W.size() * 2);
    hipMalloc(&dP, (size_t)KS * M * Co * 4); hipMalloc(&dT, 8); hipMalloc(&dO, (size_t)M * Co * 2);
    hipMalloc(&dS, Co * 4); hipMalloc(&dH, Co * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW, W.data(), W.size() * 2, hipMemcpyHostToDevice);
    hipMemset(dP, 0xff, (size_t)KS * M * Co * 4);
    hipMemset(dT, 0, 8);
    ConvArgs a{};
    a.in = dA; a.out = dO; a.w = dW; a.scale = dS; a.shift = dH; a.taps = (const int2*)dT;
    a.N = M; a.Hi = a.Wi = 1; a.Ci = K; a.in_clip_stride = K; a.Hq = a.Wq = 1; a.sy = a.sx = 1; a.oys = a.oxs = 1;
    a.Ho = a.Wo = 1; a.Co = Co; a.out_clip_stride = Co; a.out_pix_stride = Co; a.act = 1; a.nphase = 1;
    a.ksplit = KS; a.partial = (float*)dP;
    a.ph[0] = ConvPhase{0, 0, 1, K, 0, 0};
    if (launch_igemm(a, 0)) return 1;
    hipDeviceSynchronize();
    std::vector<float> P((size_t)KS * M * Co);
    hipMemcpy(P.data(), dP, P.size() * 4, hipMemcpyDeviceToHost);
    const int nst = (K + 63) / 64, sps = (nst + KS - 1) / KS;   // 64-deep steps per split
    for (int z = 0; z < KS; ++z) {
        double e2 = 0, r2 = 0;
        int bad = 0;
        for (int m = 0; m < M; ++m)
            for (int n = 0; n < Co; ++n) {
                double ref = 0;
                for (int k = std::min(K, z * sps * 64); k < std::min(K, (z + 1) * sps * 64); ++k)
                    ref += (double)bf2f(A[(size_t)m * K + k]) * bf2f(W[(size_t)n * K + k]);
                const double got = P[((size_t)z * M + m) * Co + n];
                e2 += (got - ref) * (got - ref);
                r2 += ref * ref;
                if (std::fabs(got - ref) > 1e-2 * (1 + std::fabs(ref)) && bad++ < 3)
                    std::printf("  z=%d m=%d n=%d got %g ref %g\n", z, m, n, got, ref);
            }
        std::printf("split %d: rel rms %.3e, bad %d\n", z, std::sqrt(e2 / r2), bad);
    }
    // which reference row does each computed row of split 0 match?
    for (int m = 0; m < 40; ++m) {
        int best = -1;
        double be = 1e30;
        for (int mr = 0; mr < M; ++mr) {
            double e = 0;
            for (int n = 0; n < 8; ++n) {
                double ref = 0;
                for (int k = 0; k < std::min(K, sps * 64); ++k) ref += (double)bf2f(A[(size_t)mr * K + k]) * bf2f(W[(size_t)n * K + k]);
                const double d = P[(size_t)m * Co + n] - ref;
                e += d * d;
            }
            if (e < be) { be = e; best = mr; }
        }
        std::printf("row %d ~ ref row %d (err %.2e)\n", m, best, be);
    }
    return 0;
}
