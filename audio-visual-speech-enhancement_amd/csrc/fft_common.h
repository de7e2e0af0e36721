// Small in-register DFT building blocks shared by the STFT (stft.hip) and ISTFT (istft.hip) kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace avse {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
// multiply by -i
__device__ __forceinline__ float2 cmni(float2 a) { return make_float2(a.y, -a.x); }

// forward 4-point DFT, in place
__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
    float2 a = cadd(x0, x2), b = csub(x0, x2), c = cadd(x1, x3), d = cmni(csub(x1, x3));
    x0 = cadd(a, c);
    x2 = csub(a, c);
    x1 = cadd(b, d);
    x3 = csub(b, d);
}

// forward 5-point DFT (W = e^{-2 pi i / 5}), in place
__device__ __forceinline__ void dft5(float2& x0, float2& x1, float2& x2, float2& x3, float2& x4) {
    const float c1 = 0.30901699437494745f, c2 = -0.8090169943749475f;
    const float s1 = 0.9510565162951535f, s2 = 0.5877852522924731f;
    float2 t1 = cadd(x1, x4), t2 = cadd(x2, x3), t3 = csub(x1, x4), t4 = csub(x2, x3);
    float2 a1 = make_float2(x0.x + c1 * t1.x + c2 * t2.x, x0.y + c1 * t1.y + c2 * t2.y);
    float2 a2 = make_float2(x0.x + c2 * t1.x + c1 * t2.x, x0.y + c2 * t1.y + c1 * t2.y);
    // p = s1 t3 + s2 t4 ; q = s2 t3 - s1 t4 ; -i p, -i q
    float2 p = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);
    float2 q = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
    float2 y0 = cadd(x0, cadd(t1, t2));
    float2 mp = cmni(p), mq = cmni(q);
    x0 = y0;
    x1 = cadd(a1, mp);
    x4 = csub(a1, mp);
    x2 = cadd(a2, mq);
    x3 = csub(a2, mq);
}

// 20-point forward DFT of v[n2] (n2 = 5a + b, k2 = c + 4d) in registers; result Y[c + 4d] in v[5c + d].
// tw = W640^k table (W20^{bc} = W640^{32 bc}).
__device__ __forceinline__ void dft20(float2 (&v)[20], const float2* __restrict__ tw) {
#pragma unroll
    for (int b = 0; b < 5; ++b) dft4(v[b], v[5 + b], v[10 + b], v[15 + b]);
#pragma unroll
    for (int b = 1; b < 5; ++b)
#pragma unroll
        for (int c = 1; c < 4; ++c) v[5 * c + b] = cmul(v[5 * c + b], tw[32 * b * c]);
#pragma unroll
    for (int c = 0; c < 4; ++c) dft5(v[5 * c], v[5 * c + 1], v[5 * c + 2], v[5 * c + 3], v[5 * c + 4]);
}

// 16-point forward DFT of v[n1] (n1 = 4a + b, k1 = c + 4d); result Z[c + 4d] in v[4c + d].
// tw = W640^k table (W16^{bc} = W640^{40 bc}).
__device__ __forceinline__ void dft16(float2 (&v)[16], const float2* __restrict__ tw) {
#pragma unroll
    for (int b = 0; b < 4; ++b) dft4(v[b], v[4 + b], v[8 + b], v[12 + b]);
#pragma unroll
    for (int b = 1; b < 4; ++b)
#pragma unroll
        for (int c = 1; c < 4; ++c) v[4 * c + b] = cmul(v[4 * c + b], tw[40 * b * c]);
#pragma unroll
    for (int c = 0; c < 4; ++c) dft4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
}

// ---- packed-fp32 forms (v_pk_add / v_pk_mul / v_pk_fma: one instruction per complex add, two per complex product) ----
// A complex value is one 64-bit register pair (re, im).  Auto-vectorised float2 code pairs values across different
// complex numbers and spends ~40 % of its instructions on v_mov re-pairing (r03, K1 step 1: 211 of 532); these
// helpers keep (re, im) together and fold the quarter turns into the op_sel / neg modifiers.
typedef float v2f __attribute__((ext_vector_type(2)));

// b + (-i) e = (b.x + e.y, b.y - e.x) as one v_pk_fma_f32: the swapped e times (1, -1) (inline 1.0, neg_hi) plus b.
// Not v_pk_add_f32 with a half-swapping op_sel (op_sel:[0,1] op_sel_hi:[1,0]): on gfx950 that form returned wrong
// values in lanes 48..63 whenever matrix-core work of another kernel shared the CU (tools/pk_probe.py: 12 of 12 runs,
// every run of the STFT beside an MFMA loop; 0 runs alone), while v_pk_fma_f32 with op_sel and v_pk_add_f32 without it
// measured clean.  (Round 5; the v_pk_add form is kept out of every kernel: DESIGN.md §3 K1.)
__device__ __forceinline__ v2f pk_add_mi(v2f b, v2f e) {
    v2f r;
    asm("v_pk_fma_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(e), "v"(b));
    return r;
}
// b - (-i) e = (b.x - e.y, b.y + e.x): the swapped e times (-1, 1) plus b
__device__ __forceinline__ v2f pk_sub_mi(v2f b, v2f e) {
    v2f r;
    asm("v_pk_fma_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(e), "v"(b));
    return r;
}
// b + conj(e), b - conj(e)
__device__ __forceinline__ v2f pk_add_conj(v2f b, v2f e) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(b), "v"(e));
    return r;
}
__device__ __forceinline__ v2f pk_sub_conj(v2f b, v2f e) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(b), "v"(e));
    return r;
}
// a * w, with wq = i w = (-w.y, w.x) supplied (a table entry or a constant): v_pk_mul + v_pk_fma
__device__ __forceinline__ v2f pk_cmul(v2f a, v2f w, v2f wq) {
    return __builtin_elementwise_fma(__builtin_shufflevector(a, a, 1, 1), wq, __builtin_shufflevector(a, a, 0, 0) * w);
}
__device__ __forceinline__ v2f pk_cmul_c(v2f a, float wr, float wi) { return pk_cmul(a, v2f{wr, wi}, v2f{-wi, wr}); }
// a * w from w alone: (a.x w.x, a.x w.y) by v_pk_mul, then + (a.y (-w.y), a.y w.x) by one v_pk_fma whose op_sel swaps
// w's halves and whose neg_lo negates the swapped-in w.y (twiddle tables stay float2: half the LDS bytes of (w, i w))
__device__ __forceinline__ v2f pk_cmul_t(v2f a, v2f w) {
    const v2f t = __builtin_shufflevector(a, a, 0, 0) * w;
    v2f r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}

// W20^m, W16^m = e^{-2 pi i m / N} (double literals rounded to float)
__device__ constexpr float kW20[13][2] = {
    {1.0, 0.0}, {0.9510565162951535, -0.3090169943749474}, {0.8090169943749475, -0.5877852522924731},
    {0.5877852522924731, -0.8090169943749475}, {0.30901699437494745, -0.9510565162951535}, {0.0, -1.0},
    {-0.30901699437494734, -0.9510565162951536}, {-0.587785252292473, -0.8090169943749475},
    {-0.8090169943749473, -0.5877852522924732}, {-0.9510565162951535, -0.3090169943749475}, {-1.0, 0.0},
    {-0.9510565162951538, 0.3090169943749469}, {-0.8090169943749476, 0.587785252292473}};
__device__ constexpr float kW16[10][2] = {
    {1.0, 0.0}, {0.9238795325112867, -0.3826834323650898}, {0.7071067811865476, -0.7071067811865475},
    {0.38268343236508984, -0.9238795325112867}, {0.0, -1.0}, {-0.3826834323650897, -0.9238795325112867},
    {-0.7071067811865475, -0.7071067811865476}, {-0.9238795325112867, -0.3826834323650899}, {-1.0, 0.0},
    {-0.9238795325112868, 0.38268343236508967}};

__device__ __forceinline__ void pk_dft4(v2f& x0, v2f& x1, v2f& x2, v2f& x3) {
    const v2f a = x0 + x2, b = x0 - x2, c = x1 + x3, e = x1 - x3;
    x0 = a + c;
    x2 = a - c;
    x1 = pk_add_mi(b, e);
    x3 = pk_sub_mi(b, e);
}

__device__ __forceinline__ void pk_dft5(v2f& x0, v2f& x1, v2f& x2, v2f& x3, v2f& x4) {
    const float c1 = 0.30901699437494745f, c2 = -0.8090169943749475f;
    const float s1 = 0.9510565162951535f, s2 = 0.5877852522924731f;
    const v2f t1 = x1 + x4, t2 = x2 + x3, t3 = x1 - x4, t4 = x2 - x3;
    const v2f a1 = __builtin_elementwise_fma(v2f(c2), t2, __builtin_elementwise_fma(v2f(c1), t1, x0));
    const v2f a2 = __builtin_elementwise_fma(v2f(c1), t2, __builtin_elementwise_fma(v2f(c2), t1, x0));
    const v2f p = __builtin_elementwise_fma(v2f(s2), t4, v2f(s1) * t3);
    const v2f q = __builtin_elementwise_fma(v2f(-s1), t4, v2f(s2) * t3);
    x0 = x0 + (t1 + t2);
    x1 = pk_add_mi(a1, p);
    x4 = pk_sub_mi(a1, p);
    x2 = pk_add_mi(a2, q);
    x3 = pk_sub_mi(a2, q);
}

// dft20 / dft16 above in packed form, twiddles as constants
__device__ __forceinline__ void pk_dft20(v2f (&v)[20]) {
#pragma unroll
    for (int b = 0; b < 5; ++b) pk_dft4(v[b], v[5 + b], v[10 + b], v[15 + b]);
#pragma unroll
    for (int b = 1; b < 5; ++b)
#pragma unroll
        for (int c = 1; c < 4; ++c) v[5 * c + b] = pk_cmul_c(v[5 * c + b], kW20[b * c][0], kW20[b * c][1]);
#pragma unroll
    for (int c = 0; c < 4; ++c) pk_dft5(v[5 * c], v[5 * c + 1], v[5 * c + 2], v[5 * c + 3], v[5 * c + 4]);
}

__device__ __forceinline__ void pk_dft16(v2f (&v)[16]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) pk_dft4(v[b], v[4 + b], v[8 + b], v[12 + b]);
#pragma unroll
    for (int b = 1; b < 4; ++b)
#pragma unroll
        for (int c = 1; c < 4; ++c) v[4 * c + b] = pk_cmul_c(v[4 * c + b], kW16[b * c][0], kW16[b * c][1]);
#pragma unroll
    for (int c = 0; c < 4; ++c) pk_dft4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
}

}  // namespace avse
