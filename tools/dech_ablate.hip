// Ablation timing of the fused decoder head (k_dec_head<ABL>, conv_dech.hip) at the bench shape (N = 512).
// Timing only: outputs are meaningless for ABL != 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o _dech_ablate dech_ablate.hip
#include <cstdio>
#include <string>

#include "../audio-visual-speech-enhancement_amd/csrc/conv_dech.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int ensure_lds_attr(const void* fn, int bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 2;
}
}  // namespace avse

using namespace avse;

template <int ABL>
float run(const DecHeadArgs& a, int reps) {
    (void)hipFuncSetAttribute((const void*)k_dec_head<ABL>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const dim3 grid((a.N + NC - 1) / NC);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_dec_head<ABL>, grid, dim3(NT), LDS_BYTES, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_dec_head<ABL>, grid, dim3(NT), LDS_BYTES, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int N = 512;
    DecHeadArgs a{};
    a.N = N;
    a.in_clip_stride = 3200;
    a.out_clip_stride = 400 * 128;
    void *in, *out, *w1, *w2, *w3;
    float *sc, *sh;
    (void)hipMalloc(&in, (size_t)N * 3200 * 2);
    (void)hipMalloc(&out, (size_t)N * 400 * 128 * 2);
    (void)hipMalloc(&w1, 2 * 128 * 256 * 2);
    (void)hipMalloc(&w2, 2 * 128 * 256 * 2);
    (void)hipMalloc(&w3, 4 * 128 * 512 * 2);
    (void)hipMalloc(&sc, 3 * 128 * 4);
    (void)hipMalloc(&sh, 3 * 128 * 4);
    (void)hipMemset(in, 0, (size_t)N * 3200 * 2);
    (void)hipMemset(w1, 0, 2 * 128 * 256 * 2);
    (void)hipMemset(w2, 0, 2 * 128 * 256 * 2);
    (void)hipMemset(w3, 0, 4 * 128 * 512 * 2);
    (void)hipMemset(sc, 0, 3 * 128 * 4);
    (void)hipMemset(sh, 0, 3 * 128 * 4);
    a.in = (const bf16_t*)in; a.out = (bf16_t*)out;
    a.w1 = (const bf16_t*)w1; a.w2 = (const bf16_t*)w2; a.w3 = (const bf16_t*)w3;
    for (int k = 0; k < 3; ++k) { a.sc[k] = sc + 128 * k; a.sh[k] = sh + 128 * k; }
    const int reps = 20;
    auto rep = [&](const char* name, float ms) { std::printf("%-36s %8.4f ms\n", name, ms); };
    rep("full", run<0>(a, reps));
    rep("no MFMA (1)", run<1>(a, reps));
    rep("no epilogue stores (2)", run<2>(a, reps));
    rep("no slab barriers (4)", run<4>(a, reps));
    rep("no weight loads (8)", run<8>(a, reps));
    rep("no MFMA, no stores (3)", run<3>(a, reps));
    rep("only MFMA + LDS reads (2|4|8)", run<14>(a, reps));
    rep("nothing but ring / reads (1|2|4|8)", run<15>(a, reps));
    rep("full (again)", run<0>(a, reps));
    return 0;
}
