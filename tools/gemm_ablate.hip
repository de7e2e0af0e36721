// Timing of k_gemm<0> (gemm.hip) at the bench's dense-layer shapes (M = 512 clips): enc_dense 5248 -> 1312,
// dec_dense1 1312 -> 1312, dec_dense2 1312 -> 3200, for every split-K factor, with and without the last
// workgroup's partial reads (ABL 1: outputs meaningless).  Measured (round 2): enc_dense 21.9 / 18.5 us at
// ksplit 5, dec_dense1 14.4 / 10.2 us, dec_dense2 16.4 / 14.5 us at ksplit 2; a distributed reduction (every
// workgroup of a tile spins until all partials have landed, then sums 1/ksplit of the tile; bit-identical
// outputs) was slower at every ksplit (enc 30.5, dec1 19.7, dec2 20.2 us): the spin waits for the slowest.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o _gemm_ablate gemm_ablate.hip
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/gemm.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int ensure_lds_attr(const void* fn, int bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 2;
}
}  // namespace avse

using namespace avse;

template <int ABL>
float run(const GemmArgs& g, int reps) {
    (void)hipFuncSetAttribute((const void*)k_gemm<0, ABL>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    const dim3 grid((g.M + 127) / 128, (g.N + 127) / 128, g.ksplit);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_gemm<0, ABL>), grid, dim3(NT), LDS_BYTES, 0, g);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_gemm<0, ABL>), grid, dim3(NT), LDS_BYTES, 0, g);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int M = 512;
    const int shapes[3][2] = {{5248, 1312}, {1312, 1312}, {1312, 3200}};
    const char* names[3] = {"enc_dense", "dec_dense1", "dec_dense2"};
    void *a, *w, *out, *part;
    float *sc, *sh;
    int* cnt;
    (void)hipMalloc(&a, (size_t)M * 5248 * 2);
    (void)hipMalloc(&w, (size_t)5248 * 3200 * 2);
    (void)hipMalloc(&out, (size_t)M * 3200 * 2);
    (void)hipMalloc(&part, (size_t)256 * 128 * 128 * 4);
    (void)hipMalloc(&sc, 3200 * 4);
    (void)hipMalloc(&sh, 3200 * 4);
    (void)hipMalloc(&cnt, 4096 * 4);
    {
        std::vector<uint16_t> h((size_t)5248 * 3200);
        uint32_t st = 12345;
        for (auto& v : h) { st = st * 1664525u + 1013904223u; v = (uint16_t)(0x3c00 + (st >> 22)) ^ (uint16_t)((st >> 7 & 1) << 15); }
        (void)hipMemcpy(w, h.data(), h.size() * 2, hipMemcpyHostToDevice);
        (void)hipMemcpy(a, h.data(), (size_t)M * 5248 * 2, hipMemcpyHostToDevice);
    }
    {
        std::vector<float> one(3200, 0.01f);
        (void)hipMemcpy(sc, one.data(), 3200 * 4, hipMemcpyHostToDevice);
        (void)hipMemset(sh, 0, 3200 * 4);
    }
    (void)hipMemset(cnt, 0, 4096 * 4);
    for (int l = 0; l < 3; ++l) {
        GemmArgs g{};
        g.a = (const bf16_t*)a; g.lda = shapes[l][0]; g.w = (const bf16_t*)w;
        g.M = M; g.N = shapes[l][1]; g.kpad = shapes[l][0];
        g.scale = sc; g.shift = sh; g.act = 1; g.out = (bf16_t*)out; g.ldo = shapes[l][1]; g.out_off = 0;
        g.partial = (float*)part; g.counters = cnt;
        const int ks0 = gemm_ksplit(M, g.N, g.kpad, 0);
        std::printf("%s (default ksplit %d)\n", names[l], ks0);
        for (int ks = 1; ks <= 8; ++ks) {
            const int tiles = ((M + 127) / 128) * ((g.N + 127) / 128);
            if (tiles * ks > 256 || g.kpad / 32 < ks) break;
            g.ksplit = ks;
            const float t0 = run<0>(g, 20), t1 = ks > 1 ? run<1>(g, 20) : t0;
            std::printf("  ksplit %d: %7.2f us   no partial reads %7.2f us\n", ks, t0 * 1e3, t1 * 1e3);
        }
    }
    return 0;
}
