// Diagnostic (tools/pk_probe.py, never the library): does a packed-FP32 VALU chain (v_pk_fma_f32) give the same
// result when matrix-core work from another kernel shares its compute units?  k_pk_victim: 448 threads (7 waves, the
// STFT kernels' shape) with a 72-KB LDS footprint (two blocks per CU, like k_spec_seg), each lane iterating
// x = x * a + b on a float2 `iters` times — kind 0 as v_pk_fma_f32 (inline asm), kind 1 as two v_fma_f32 — and storing
// x (kinds 16.. : one packed-FP32 op_sel / neg form each, every form the built library contains — the allow-list of
// tests/test_isa_guard.py; `x = FORM(x / 2, a, b) + b`); k_mfma_busy: a grid of 256-thread workgroups issuing v_mfma_f32_16x16x32_f16 back to back.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/pk_probe.hip -o tools/_stress/libpk_probe.so
#include <hip/hip_runtime.h>

#include "../audio-visual-speech-enhancement_amd/csrc/fft_common.h"
using avse::pk_add_mi;
using avse::pk_sub_conj;
using avse::pk_cmul_t;
using avse::v2f;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(448) void k_pk_victim(const float* in, float* out, int iters) {
    __shared__ float pad[18432];   // 72 KB
    const int tid = threadIdx.x;
    const size_t g = (size_t)blockIdx.x * 448 + tid;
    pad[tid] = in[g & 4095];
    __syncthreads();
    v2f x = {in[(g * 7) & 4095], in[(g * 13 + 1) & 4095]};
    const v2f a = {0.999f + 1e-4f * pad[(tid + 1) % 448], 1.0001f - 1e-4f * pad[(tid + 2) % 448]};
    const v2f b = {1e-3f * pad[(tid + 3) % 448], -1e-3f * pad[(tid + 5) % 448]};
    const int lane = tid & 63, wave = tid >> 6;
    float* wr = pad + 4096 + wave * 2048;   // the wave's own 8-KB LDS region (past the coefficients at 0..447)
    for (int it = 0; it < iters; ++it) {
        if constexpr (KIND == 8) {          // pk_add_mi / pk_sub_mi as v_pk_fma_f32 (fft_common.h, round 5)
            x = avse::pk_sub_mi(avse::pk_add_mi(x * v2f{0.25f, 0.25f}, b), a * v2f{0.25f, 0.25f});
        } else if constexpr (KIND == 4) {          // v_pk_fma_f32 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0] (pk_cmul_t)
            x = pk_cmul_t(x, a) * v2f{0.5f, 0.5f} + b;
        } else if constexpr (KIND == 5) {   // v_pk_add_f32 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1] (round-4 pk_add_mi)
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(h), "v"(b));
            x = r;
        } else if constexpr (KIND == 6) {   // v_pk_add_f32 neg_lo:[0,1] (pk_sub_conj: no op_sel)
            x = pk_sub_conj(x * v2f{0.5f, 0.5f}, b);
        } else if constexpr (KIND == 7) {   // v_pk_add_f32 with op_sel only, no neg
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(h), "v"(b));
            x = r;
        } else if constexpr (KIND == 16) {   // v_pk_fma_f32 op_sel_hi:[1,0,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 17) {   // v_pk_fma_f32 op_sel_hi:[1,0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 18) {   // v_pk_fma_f32 op_sel_hi:[1,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 19) {   // v_pk_fma_f32 op_sel_hi:[0,1,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 20) {   // v_pk_fma_f32 op_sel_hi:[0,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 21) {   // v_pk_fma_f32 op_sel:[1,0,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 22) {   // v_pk_fma_f32 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 23) {   // v_pk_fma_f32 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 24) {   // v_pk_fma_f32 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 25) {   // v_pk_fma_f32 op_sel:[1,0,0] op_sel_hi:[1,0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 26) {   // v_pk_fma_f32 op_sel:[1,0,0] op_sel_hi:[1,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 27) {   // v_pk_fma_f32 op_sel:[0,0,1] op_sel_hi:[1,1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 28) {   // v_pk_fma_f32 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 29) {   // v_pk_fma_f32 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 30) {   // v_pk_mul_f32 op_sel_hi:[1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 31) {   // v_pk_mul_f32 op_sel_hi:[0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 32) {   // v_pk_add_f32 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 33) {   // v_pk_add_f32 
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 " : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 34) {   // v_pk_add_f32 neg_hi:[0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 35) {   // v_pk_add_f32 neg_lo:[0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 36) {   // v_pk_add_f32 neg_lo:[0,1] neg_hi:[0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 37) {   // v_pk_add_f32 neg_lo:[1,1] neg_hi:[1,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[1,1] neg_hi:[1,1]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 38) {   // v_pk_fma_f32 
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 " : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 39) {   // v_pk_fma_f32 neg_lo:[0,0,1] neg_hi:[0,0,1]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[0,0,1] neg_hi:[0,0,1]" : "=v"(r) : "v"(h), "v"(a), "v"(b));
            x = r + b;
        } else if constexpr (KIND == 40) {   // v_pk_mul_f32 
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_mul_f32 %0, %1, %2 " : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 41) {   // v_pk_add_f32 op_sel_hi:[1,0]
            v2f r;
            const v2f h = x * v2f{0.5f, 0.5f};
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(h), "v"(a));
            x = r + b;
        } else if constexpr (KIND == 3) {
            // the STFT's op_sel / neg packed-fp32 helpers (fft_common.h): a rotation, a -i add and a conjugate add
            const v2f t = pk_cmul_t(x, a);
            const v2f u = pk_add_mi(t, b);
            x = pk_sub_conj(u, t) * v2f{0.25f, 0.25f} + x * v2f{0.25f, 0.25f};
        } else if constexpr (KIND == 2) {
            // LDS round trip inside the wave: store x, read the partner lane's (lane ^ 32) value, pk_fma with it
            reinterpret_cast<v2f*>(wr)[(it & 15) * 64 + lane] = x;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const v2f y = reinterpret_cast<const v2f*>(wr)[(it & 15) * 64 + (lane ^ 32)];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(y), "v"(a), "v"(b));
        } else if constexpr (KIND == 0) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
        } else {
            float x0 = x.x, x1 = x.y;
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(a.x), "v"(b.x));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(a.y), "v"(b.y));
            x = v2f{x0, x1};
        }
    }
    out[2 * g] = x.x;
    out[2 * g + 1] = x.y;
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_mfma_busy(float* out, int iters) {
    __shared__ float st[4096];
    if constexpr (LDS) {
        for (int i = threadIdx.x; i < 4096; i += 256) st[i] = 0.001f * i;
        __syncthreads();
    }
    f16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = (_Float16)(0.001f * (threadIdx.x + e));
        b[e] = (_Float16)(0.002f * (threadIdx.x - e));
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
        if constexpr (LDS) {
            if ((it & 7) == 0) {
                a[0] = (_Float16)st[(threadIdx.x + it) & 4095];
                st[(threadIdx.x * 5 + it) & 4095] = acc[1];
            }
        }
    }
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

extern "C" int pk_victim(int kind, const float* in, float* out, int blocks, int iters, void* stream) {
    if (kind == 0) hipLaunchKernelGGL(k_pk_victim<0>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 1) hipLaunchKernelGGL(k_pk_victim<1>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 3) hipLaunchKernelGGL(k_pk_victim<3>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 4) hipLaunchKernelGGL(k_pk_victim<4>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 5) hipLaunchKernelGGL(k_pk_victim<5>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 6) hipLaunchKernelGGL(k_pk_victim<6>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 7) hipLaunchKernelGGL(k_pk_victim<7>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 8) hipLaunchKernelGGL(k_pk_victim<8>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 16) hipLaunchKernelGGL(k_pk_victim<16>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 17) hipLaunchKernelGGL(k_pk_victim<17>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 18) hipLaunchKernelGGL(k_pk_victim<18>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 19) hipLaunchKernelGGL(k_pk_victim<19>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 20) hipLaunchKernelGGL(k_pk_victim<20>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 21) hipLaunchKernelGGL(k_pk_victim<21>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 22) hipLaunchKernelGGL(k_pk_victim<22>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 23) hipLaunchKernelGGL(k_pk_victim<23>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 24) hipLaunchKernelGGL(k_pk_victim<24>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 25) hipLaunchKernelGGL(k_pk_victim<25>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 26) hipLaunchKernelGGL(k_pk_victim<26>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 27) hipLaunchKernelGGL(k_pk_victim<27>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 28) hipLaunchKernelGGL(k_pk_victim<28>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 29) hipLaunchKernelGGL(k_pk_victim<29>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 30) hipLaunchKernelGGL(k_pk_victim<30>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 31) hipLaunchKernelGGL(k_pk_victim<31>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 32) hipLaunchKernelGGL(k_pk_victim<32>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 33) hipLaunchKernelGGL(k_pk_victim<33>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 34) hipLaunchKernelGGL(k_pk_victim<34>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 35) hipLaunchKernelGGL(k_pk_victim<35>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 36) hipLaunchKernelGGL(k_pk_victim<36>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 37) hipLaunchKernelGGL(k_pk_victim<37>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 38) hipLaunchKernelGGL(k_pk_victim<38>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 39) hipLaunchKernelGGL(k_pk_victim<39>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 40) hipLaunchKernelGGL(k_pk_victim<40>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else if (kind == 41) hipLaunchKernelGGL(k_pk_victim<41>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    else hipLaunchKernelGGL(k_pk_victim<2>, dim3(blocks), dim3(448), 0, (hipStream_t)stream, in, out, iters);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
extern "C" int mfma_busy(int lds, float* out, int blocks, int iters, void* stream) {
    if (lds) hipLaunchKernelGGL(k_mfma_busy<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
    else hipLaunchKernelGGL(k_mfma_busy<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
