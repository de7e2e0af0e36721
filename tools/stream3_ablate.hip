// Ablation timing of k_conv_stream<3,16,16,1> (conv_stream.hip) at the v_conv3 and v_conv4 bench shapes (N = 512:
// 32x32x128 -> 256 and 16x16x256 -> 256, 3x3, pooled).  Timing only: outputs are meaningless for ABL != 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o _stream3_ablate stream3_ablate.hip
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/conv_stream.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int ensure_lds_attr(const void* fn, int bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 2;
}
}  // namespace avse

using namespace avse;

// warm-up: 200 launches (~40 ms) — with 10 the clock was still settling through the whole list of variants
template <int ABL, int BP = 1, int LAT = 6>
float run(const HaloArgs& a, int reps) {
    using G = StreamGeom<3, 16, 16, 1, LAT, BP>;
    auto k = k_conv_stream<3, 16, 16, 1, true, G::LAT, ABL, BP>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS + 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int cob = a.Co / 128, gx = 256 / cob;
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k, dim3(gx, cob), dim3(512), G::LDS + 1024, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(gx, cob), dim3(512), G::LDS + 1024, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int N = 512;
    for (int shape = 0; shape < 2; ++shape) {
        const int H = shape == 0 ? 32 : 16, Ci = shape == 0 ? 128 : 256, Co = 256;
        HaloArgs a{};
        a.variant = HALO_K3_16;
        a.N = N; a.Hc = H; a.Wc = H; a.Ci = Ci; a.Co = Co;
        a.out_clip_stride = (long long)(H / 2) * (H / 2) * Co;
        a.out_pix_stride = Co;
        void *in, *out, *w;
        float *sc, *sh;
        (void)hipMalloc(&in, (size_t)N * H * H * Ci * 2);
        (void)hipMalloc(&out, (size_t)N * (H / 2) * (H / 2) * Co * 2);
        (void)hipMalloc(&w, (size_t)9 * Ci * Co * 2);
        (void)hipMalloc(&sc, Co * 4);
        (void)hipMalloc(&sh, Co * 4);
        // AVSE_ABL_RANDOM=1: random bf16 activations / weights (MFMA power, hence clock, depends on data)
        const char* rnd = std::getenv("AVSE_ABL_RANDOM");
        if (rnd && rnd[0] == '1') {
            std::vector<uint16_t> h((size_t)N * H * H * Ci);
            uint32_t st = 12345;
            auto next = [&] { st = st * 1664525u + 1013904223u; return st; };
            for (auto& v : h) v = (uint16_t)(0x3c00 + (next() >> 22)) ^ (uint16_t)((next() >> 31) << 15);
            (void)hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
            (void)hipMemcpy(w, h.data(), (size_t)9 * Ci * Co * 2, hipMemcpyHostToDevice);
        } else {
            (void)hipMemset(in, 0, (size_t)N * H * H * Ci * 2);
            (void)hipMemset(w, 0, (size_t)9 * Ci * Co * 2);
        }
        (void)hipMemset(sc, 0, Co * 4);
        (void)hipMemset(sh, 0, Co * 4);
        a.in = in; a.out = out; a.w = w; a.scale = sc; a.shift = sh;
        const double flop = 2.0 * N * H * H * Co * Ci * 9;
        const int reps = 20;
        std::printf("%s\n", shape == 0 ? "v_conv3 32x32x128 -> 256" : "v_conv4 16x16x256 -> 256");
        auto rep = [&](const char* name, float ms) {
            std::printf("  %-30s %8.4f ms  %7.1f TF/s\n", name, ms, flop / (ms * 1e-3) / 1e12);
        };
        rep("full", run<0>(a, reps));
        rep("full, LAT 3 (again)", run<0, 1, 3>(a, reps));
        rep("full, LAT 3", run<0, 1, 3>(a, reps));
        rep("full", run<0>(a, reps));
        rep("full, LAT 3 (again)", run<0, 1, 3>(a, reps));
        rep("full, barrier period 2", run<0, 2>(a, reps));
        rep("no halo pieces (1)", run<1>(a, reps));
        rep("no weight streaming (2)", run<2>(a, reps));
        rep("no loads at all (3)", run<3>(a, reps));
        rep("no wait/barrier (4)", run<4>(a, reps));
        rep("no frag reads (8)", run<8>(a, reps));
        rep("MFMA only (15)", run<15>(a, reps));
        rep("full (again)", run<0>(a, reps));
        (void)hipFree(in); (void)hipFree(out); (void)hipFree(w); (void)hipFree(sc); (void)hipFree(sh);
    }
    return 0;
}
