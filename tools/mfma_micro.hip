// Micro-benchmark: cycles per v_mfma_f32_16x16x32_bf16 for one wave per SIMD with 28 accumulators (the fused
// decoder kernel's step), optionally with the step's 7 ds_read_b128 and 4 buffer loads.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/mfma_micro.hip -o /tmp/mfma_micro && /tmp/mfma_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(const i32x4* wsrc, float* out, unsigned long long* cyc, int steps) {
    __shared__ i32x4 lds[8192];
    const int tid = threadIdx.x;
    for (int i = tid; i < 8192; i += 256) lds[i] = wsrc[(i * 7) & 65535];   // random bf16 pairs from the host
    __syncthreads();
    f32x4 acc[7][4];
    for (int i = 0; i < 7; ++i) for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0, 0, 0, 0};
    i32x4 fa[2][7], fb[4][4];
    for (int i = 0; i < 7; ++i) fa[0][i] = fa[1][i] = lds[(tid * 7 + i) & 8191];
    for (int r = 0; r < 4; ++r) for (int j = 0; j < 4; ++j) fb[r][j] = wsrc[(tid + 256 * j) & 1023];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<i32x4*>(wsrc), (short)0, 1 << 20, 0x00020000);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; s += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (MODE & 1) {
#pragma unroll
                for (int i = 0; i < 7; ++i) fa[(q + 1) & 1][i] = lds[((tid & 63) * 2 + i * 130 + q * 64 + (s & 7)) & 8191];
            }
            if constexpr (MODE & 2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) fb[(q + 3) & 3][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((tid * 16 + j * 4096 + q * 64) & 0x3ffff), 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 7; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[q & 1][i]),
                                                                         __builtin_bit_cast(bf16x8, fb[q][j]), acc[i][j], 0, 0, 0);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0;
    for (int i = 0; i < 7; ++i) for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][3];
    out[blockIdx.x * 256 + tid] = sum;
    if ((tid & 63) == 0) cyc[blockIdx.x * 4 + tid / 64] = t1 - t0;
}

int main() {
    i32x4* w; float* out; unsigned long long* cyc;
    hipMalloc(&w, 1 << 20); hipMalloc(&out, 512 * 256 * 4); hipMalloc(&cyc, 512 * 4 * 8);
    std::vector<int> hw(1 << 18);
    unsigned st = 12345;
    auto rnd_bf16 = [&]() { st = st * 1664525u + 1013904223u; const float f = ((st >> 8) & 0xffff) / 65536.f - 0.5f;
                            unsigned u; memcpy(&u, &f, 4); return u >> 16; };
    for (size_t i = 0; i < hw.size(); ++i) hw[i] = (int)(rnd_bf16() | (rnd_bf16() << 16));
    hipMemcpy(w, hw.data(), 1 << 20, hipMemcpyHostToDevice);
    const int steps = 1024;
    for (int mode = 0; mode < 4; ++mode) {
        for (int nb : {256, 512}) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nb), dim3(256), 0, 0, w, out, cyc, steps);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(nb), dim3(256), 0, 0, w, out, cyc, steps);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(nb), dim3(256), 0, 0, w, out, cyc, steps);
                if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(nb), dim3(256), 0, 0, w, out, cyc, steps);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms; hipEventElapsedTime(&ms, e0, e1);
            std::vector<unsigned long long> h(nb * 4);
            hipMemcpy(h.data(), cyc, nb * 4 * 8, hipMemcpyDeviceToHost);
            double a = 0; for (auto v : h) a += v; a /= h.size();
            const double nm = (double)steps * 28;
            printf("mode %d (lds %d, vmem %d) blocks %d: %.1f cycles/MFMA (s_memtime), %.3f ms, %.0f TFLOP/s\n", mode, mode & 1, (mode >> 1) & 1,
                   nb, a / nm, ms, nb * 4 * nm * 16384.0 / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
