// Numerics probe for fp32-accurate split-operand MFMA products on gfx950 (DESIGN.md §3 "split fp16"):
//   1. do f16 MFMA operands keep subnormals (the lo piece of a small value is an f16 subnormal)?
//   2. does one v_mfma_f32_16x16x32_f16 round once per product (an fmaf chain) or sum its 32 products first?
//   3. relative RMS error of a K = 3200 dot-product tile against float64, for exact-f32 MFMA (16x16x4),
//      2x2-split f16 (x = hi + lo in f16, all four products), 2x2-split f16 with the three small products in a
//      second accumulator, and 3x3-split bf16 (six products).
// Build + run (GPU box):  hipcc --offload-arch=gfx950 -O3 -o /tmp/split_probe tools/split_probe.hip && /tmp/split_probe
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// one wave: C[16][16] = A[16][K] B[K][16] (A row-major [16][K], B stored [16][K] = B^T), K % 32 == 0
// mode 0: f32 MFMA 16x16x4; 1: f16 2x2 split one accumulator; 2: f16 2x2 split, small products separate;
// 3: bf16 3x3 split, six products; 4: f16 hi only (plain f16)
__global__ void k_dot(const float* A, const float* B, int K, int mode, float* C) {
    const int l = threadIdx.x, r = l & 15, kg = l >> 4;
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    if (mode == 0) {
        for (int k = 0; k < K; k += 4)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[r * K + k + kg], B[r * K + k + kg], acc, 0, 0, 0);
    } else if (mode == 3) {
        for (int k = 0; k < K; k += 32) {
            bf16x8 a[3], b[3];
            for (int e = 0; e < 8; ++e) {
                float x = A[r * K + k + 8 * kg + e], y = B[r * K + k + 8 * kg + e];
                for (int p = 0; p < 3; ++p) {
                    __bf16 hx = (__bf16)x, hy = (__bf16)y;
                    a[p][e] = hx; b[p][e] = hy;
                    x -= (float)hx; y -= (float)hy;
                }
            }
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc2, 0, 0, 0);
        }
    } else {
        for (int k = 0; k < K; k += 32) {
            f16x8 ah, al, bh, bl;
            for (int e = 0; e < 8; ++e) {
                const float x = A[r * K + k + 8 * kg + e], y = B[r * K + k + 8 * kg + e];
                const _Float16 hx = (_Float16)x, hy = (_Float16)y;
                ah[e] = hx; bh[e] = hy;
                al[e] = (_Float16)(x - (float)hx); bl[e] = (_Float16)(y - (float)hy);
            }
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
            if (mode == 4) continue;
            f32x4& s = mode == 2 ? acc2 : acc;
            s = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bl, s, 0, 0, 0);
        }
    }
    for (int i = 0; i < 4; ++i) C[(4 * kg + i) * 16 + r] = acc[i] + acc2[i];
}

// probe 1/2: one f16 MFMA on given operands (all rows/cols equal), returns C[0][0]
__global__ void k_one(const _Float16* a, const _Float16* b, float c0, float* out) {
    const int l = threadIdx.x, kg = l >> 4;
    f16x8 av, bv;
    for (int e = 0; e < 8; ++e) { av[e] = a[8 * kg + e]; bv[e] = b[8 * kg + e]; }
    f32x4 acc = {c0, c0, c0, c0};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
    if (l == 0) out[0] = acc[0];
}

int one(std::vector<_Float16> a, std::vector<_Float16> b, float c0, float* res) {
    _Float16 *da, *db; float* dout;
    CK(hipMalloc(&da, 64)); CK(hipMalloc(&db, 64)); CK(hipMalloc(&dout, 4));
    CK(hipMemcpy(da, a.data(), 64, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), 64, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
    CK(hipMemcpy(res, dout, 4, hipMemcpyDeviceToHost));
    CK(hipFree(da)); CK(hipFree(db)); CK(hipFree(dout));
    return 0;
}

int main() {
    // 1. subnormals: a = 2^-20 (f16 subnormal), b = 1
    {
        std::vector<_Float16> a(32, (_Float16)0.f), b(32, (_Float16)0.f);
        a[0] = (_Float16)std::ldexp(1.f, -20);
        b[0] = (_Float16)1.f;
        float r = 0;
        if (one(a, b, 0.f, &r)) return 1;
        printf("subnormal f16 operand 2^-20 x 1 -> %.9g (kept: %s)\n", r, r == std::ldexp(1.f, -20) ? "yes" : "NO");
        a[0] = (_Float16)std::ldexp(1.f, -14);   // min normal x 2^-10 (smallest subnormal 2^-24)
        a[0] = (_Float16)std::ldexp(1.f, -24);
        if (one(a, b, 0.f, &r)) return 1;
        printf("subnormal f16 operand 2^-24 x 1 -> %.9g\n", r);
    }
    // 2. internal accumulation: C = 2^24, 32 products of 1 x 1: fmaf chain -> 2^24, exact sum -> 2^24 + 32
    {
        std::vector<_Float16> a(32, (_Float16)1.f), b(32, (_Float16)1.f);
        float r = 0;
        if (one(a, b, 16777216.f, &r)) return 1;
        printf("C = 2^24 + 32 x (1 x 1) -> %.1f (2^24 = 16777216: per-product rounding; 16777248: one rounding)\n", r);
        // 16 products of +1 and 16 of 2^-12 onto C = 1: exact = 1 + 16 + 16 * 2^-12
        for (int i = 16; i < 32; ++i) a[i] = (_Float16)std::ldexp(1.f, -12);
        if (one(a, b, 1.f, &r)) return 1;
        printf("C = 1 + 16 x 1 + 16 x 2^-12 -> %.9g (exact %.9g)\n", r, 17.0 + 16 * std::ldexp(1.0, -12));
        // tiny products under a big one: 2^11 * 2^11 + 31 x (2^-11 x 2^-4)
        for (int i = 0; i < 32; ++i) { a[i] = (_Float16)std::ldexp(1.f, -11); b[i] = (_Float16)std::ldexp(1.f, -4); }
        a[0] = (_Float16)2048.f; b[0] = (_Float16)2048.f;
        if (one(a, b, 0.f, &r)) return 1;
        printf("2^22 + 31 x 2^-15 -> %.9g (exact %.12g, f32 sum order-dependent)\n", r, 4194304.0 + 31 * std::ldexp(1.0, -15));
    }
    // 3. K = 3200 dot tiles, activation-like A (|N(0, 20)| mixed sign), weight-like B (U(-0.03, 0.03) x 2^9)
    const int K = 3200;
    std::mt19937_64 g(7);
    std::normal_distribution<double> nd(0, 20);
    std::uniform_real_distribution<double> ud(-0.03, 0.03);
    std::vector<float> A(16 * K), B(16 * K), C(256);
    for (auto& x : A) { double v = nd(g); x = (float)(v < 0 ? 0.3 * v : v); }
    for (auto& x : B) x = (float)(ud(g) * 512.0);
    std::vector<double> ref(256);
    double rr = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0;
            for (int k = 0; k < K; ++k) s += (double)A[i * K + k] * (double)B[j * K + k];
            ref[i * 16 + j] = s;
            rr += s * s;
        }
    rr = std::sqrt(rr / 256);
    float *dA, *dB, *dC;
    CK(hipMalloc(&dA, A.size() * 4)); CK(hipMalloc(&dB, B.size() * 4)); CK(hipMalloc(&dC, 1024));
    CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    const char* names[5] = {"f32 MFMA 16x16x4", "f16 2x2 split, one acc", "f16 2x2 split, small products apart",
                            "bf16 3x3 split, 6 products", "f16 hi only"};
    for (int m = 0; m < 5; ++m) {
        hipLaunchKernelGGL(k_dot, dim3(1), dim3(64), 0, 0, dA, dB, K, m, dC);
        CK(hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost));
        double e = 0;
        for (int i = 0; i < 256; ++i) e += (C[i] - ref[i]) * (C[i] - ref[i]);
        printf("K=%d %-38s rel RMS err %.3e\n", K, names[m], std::sqrt(e / 256) / rr);
    }
    return 0;
}
