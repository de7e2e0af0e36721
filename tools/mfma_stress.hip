// Diagnostic (tools/overlap_probe.py "stress" mode, never the library): a grid of small workgroups that run only
// matrix-core loops of one kind on register operands, with a 16-KB LDS footprint and 2-byte or 4-byte global stores
// of their results, to be co-scheduled beside the spectrogram kernels on another stream.
//   kind 0: v_mfma_f32_16x16x32_f16, f16 2-byte stores of the results
//   kind 1: v_mfma_f32_16x16x32_bf16, bf16 2-byte stores
//   kind 2: v_mfma_f32_16x16x32_f16, fp32 4-byte stores
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_stress.hip -o tools/_stress/libmfma_stress.so
#include <hip/hip_runtime.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(256) void k_stress(void* out, int iters, float seed) {
    __shared__ float stage[4096];   // 16 KB, written and read so the allocation is real
    const int tid = threadIdx.x;
    for (int i = tid; i < 4096; i += 256) stage[i] = seed + i;
    __syncthreads();
    f32x4 acc = {stage[tid], stage[tid + 256], 0.f, 0.f};
    f16x8 a, b;
    bf16x8 c, d;
    for (int e = 0; e < 8; ++e) {
        a[e] = (_Float16)(stage[(tid + e) & 4095] * 1e-3f);
        b[e] = (_Float16)(stage[(tid * 3 + e) & 4095] * 1e-3f);
        c[e] = (__bf16)(stage[(tid + e) & 4095] * 1e-3f);
        d[e] = (__bf16)(stage[(tid * 3 + e) & 4095] * 1e-3f);
    }
    for (int it = 0; it < iters; ++it) {
        if constexpr (KIND == 1)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, d, acc, 0, 0, 0);
        else
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    }
    const size_t o = ((size_t)blockIdx.x * 256 + tid) * 4;
    if constexpr (KIND == 2) {
        for (int r = 0; r < 4; ++r) reinterpret_cast<float*>(out)[o + r] = acc[r];
    } else if constexpr (KIND == 1) {
        for (int r = 0; r < 4; ++r) reinterpret_cast<__bf16*>(out)[o + r] = (__bf16)acc[r];
    } else {
        for (int r = 0; r < 4; ++r) reinterpret_cast<_Float16*>(out)[o + r] = (_Float16)acc[r];
    }
}

extern "C" int mfma_stress(int kind, void* out, int n_wg, int iters, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0) hipLaunchKernelGGL(k_stress<0>, dim3(n_wg), dim3(256), 0, s, out, iters, 1.f);
    else if (kind == 1) hipLaunchKernelGGL(k_stress<1>, dim3(n_wg), dim3(256), 0, s, out, iters, 1.f);
    else hipLaunchKernelGGL(k_stress<2>, dim3(n_wg), dim3(256), 0, s, out, iters, 1.f);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
