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

}  // namespace avse
