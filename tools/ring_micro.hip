// Micro-benchmark of the per-clip fused kernels' slab step (conv_dec.hip / conv_aud.hip / gemm.hip shape):
// 8 waves (two per SIMD), per slab 4 A + 4 B ds_read_b128 fragments, 16 v_mfma_f32_16x16x32_bf16 per wave,
// a weight ring (8 B per lane per slab: buffer_load_dwordx2 8 slabs ahead, ds_write_b64 4 ahead) and one
// barrier per 4 slabs.  MODE bits remove parts: 1 no barrier, 2 no ring (load + store), 4 no fragment reads,
// 8 ring stores as ds_write_b128 (16 B per lane).  Prints cycles per MFMA (s_memtime) and TFLOP/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ring_micro.hip -o tools/_ring_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void k(const int* wsrc, float* out, unsigned long long* cyc, int steps) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, kg = lane >> 4;
    for (int i = tid; i < 147456 / 16; i += 512) reinterpret_cast<i32x4*>(lds)[i] = reinterpret_cast<const i32x4*>(wsrc)[i & 4095];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(wsrc), (short)0, 1 << 20, 0x00020000);
    const int BOFF = 115584;
    const int bst = BOFF + (tid >> 3) * 64 + (((tid >> 1) & 3) << 4) + (tid & 1) * 8;
    const int bfr = BOFF + r16 * 64 + (kg << 4);
    int vb[4];
    for (int i = 0; i < 4; ++i) vb[i] = ((w + 8 * i) * 16 * 96 + r16 * 96 + kg * 16) % 100000;
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0, 0, 0, 0};
    i32x4 fa[2][4], fb[2][4];
    for (int i = 0; i < 4; ++i) { fa[0][i] = fa[1][i] = *reinterpret_cast<i32x4*>(lds + vb[i]); fb[0][i] = fb[1][i] = *reinterpret_cast<i32x4*>(lds + bfr + 1024 * i); }
    i32x2 pb[4];
    i32x4 pb4[4];
    for (int q = 0; q < 4; ++q) { pb[q] = (i32x2){q, tid}; pb4[q] = (i32x4){q, tid, 0, 0}; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s0 = 0; s0 < steps; s0 += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int s = s0 + q;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!(MODE & 2)) {
                if constexpr (MODE & 8) {
                    *reinterpret_cast<i32x4*>(lds + bst + (((s >> 2) + 1) & 1) * 16384 + q * 4096) = pb4[q];
                    pb4[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid * 16 + (s & 63) * 8192) & 0xfffff, 0, 0);
                } else {
                    *reinterpret_cast<i32x2*>(lds + bst + (((s >> 2) + 1) & 1) * 16384 + q * 4096) = pb[q];
                    pb[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, (tid * 8 + (s & 63) * 4096) & 0xfffff, 0, 0);
                }
            }
            if constexpr (!(MODE & 1)) { if (q == 3) __syncthreads(); }
            if constexpr (!(MODE & 4)) {
                const int imm = ((s + 1) % 16) * 96;
#pragma unroll
                for (int i = 0; i < 4; ++i) fa[(q + 1) & 1][i] = *reinterpret_cast<i32x4*>(lds + vb[i] + imm);
#pragma unroll
                for (int j = 0; j < 4; ++j) fb[(q + 1) & 1][j] = *reinterpret_cast<i32x4*>(lds + bfr + (((s + 1) >> 2) & 1) * 16384 + ((s + 1) & 3) * 4096 + 1024 * j);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[q & 1][i]),
                                                                         __builtin_bit_cast(bf16x8, fb[q & 1][j]), acc[i][j], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][3];
    for (int q = 0; q < 4; ++q) sum += pb[q][0] + pb4[q][1];
    out[blockIdx.x * 512 + tid] = sum;
    if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int MODE>
void run(const int* w, float* out, unsigned long long* cyc, int nb, int steps) {
    hipFuncSetAttribute((const void*)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 148352);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<MODE>, dim3(nb), dim3(512), 148352, 0, w, out, cyc, steps);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    std::vector<unsigned long long> h(nb * 8);
    hipMemcpy(h.data(), cyc, nb * 8 * 8, hipMemcpyDeviceToHost);
    double a = 0; for (auto v : h) a += v; a /= h.size();
    const double nm = (double)steps * 16;   // MFMAs per wave
    printf("mode %2d (no-barrier %d no-ring %d no-reads %d ring16B %d): %.1f cycles per MFMA per wave pair-SIMD, %.3f ms, %.0f TFLOP/s\n",
           MODE, MODE & 1, (MODE >> 1) & 1, (MODE >> 2) & 1, (MODE >> 3) & 1, a / nm / 2, ms, nb * 8 * nm * 16384.0 / (ms * 1e-3) / 1e12);
}

int main() {
    int* w; float* out; unsigned long long* cyc;
    hipMalloc(&w, 1 << 20); hipMalloc(&out, 512 * 512 * 4); hipMalloc(&cyc, 512 * 8 * 8);
    std::vector<int> hw(1 << 18);
    unsigned st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; const float f = ((st >> 8) & 0xffff) / 65536.f - 0.5f; unsigned u; memcpy(&u, &f, 4); return u >> 16; };
    for (auto& v : hw) v = (int)(rnd() | (rnd() << 16));
    hipMemcpy(w, hw.data(), 1 << 20, hipMemcpyHostToDevice);
    const int nb = 512, steps = 512;
    run<0>(w, out, cyc, nb, steps);
    run<1>(w, out, cyc, nb, steps);
    run<2>(w, out, cyc, nb, steps);
    run<3>(w, out, cyc, nb, steps);
    run<4>(w, out, cyc, nb, steps);
    run<6>(w, out, cyc, nb, steps);
    run<7>(w, out, cyc, nb, steps);
    run<8>(w, out, cyc, nb, steps);
    return 0;
}
