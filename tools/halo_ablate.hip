// Ablation timing of the halo-tiled v_conv2 kernel (k_conv_halo<5,16,16,1,false,true,ABL>) at the
// bench shape (N=512, 64x64x128 -> 128, 5x5): each ABL bit removes one part of the K loop so the
// time it costs shows up as the difference.  Timing only — the outputs are meaningless for ABL != 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../audio-visual-speech-enhancement_amd/csrc halo_ablate.hip
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/conv_halo.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int launch_conv_stream(const HaloArgs&, hipStream_t) { return 3; }   // conv_stream.hip is not linked here
}  // namespace avse

using namespace avse;

template <int ABL>
float run(const HaloArgs& a, int reps) {
    constexpr size_t shm = 400 * 256 + 256 + 3 * HALO_NT * 8192;
    (void)hipFuncSetAttribute((const void*)k_conv_halo<5, 16, 16, 1, false, true, ABL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    const int tiles = a.N * 16;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 2; ++r)
        hipLaunchKernelGGL((k_conv_halo<5, 16, 16, 1, false, true, ABL>), dim3(tiles, 1), dim3(512), shm, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_conv_halo<5, 16, 16, 1, false, true, ABL>), dim3(tiles, 1), dim3(512), shm, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int N = 512, H = 64, C = 128;
    HaloArgs a{};
    a.variant = HALO_K5;
    a.N = N; a.Hc = H; a.Wc = H; a.Ci = C; a.Co = C;
    a.out_clip_stride = (long long)(H / 2) * (H / 2) * C;
    a.out_pix_stride = C;
    a.out_c_off = 0;
    void *in, *out, *w;
    float *sc, *sh;
    (void)hipMalloc(&in, (size_t)N * H * H * C * 2);
    (void)hipMalloc(&out, (size_t)N * (H / 2) * (H / 2) * C * 2);
    (void)hipMalloc(&w, (size_t)100 * C * 64);
    (void)hipMalloc(&sc, C * 4);
    (void)hipMalloc(&sh, C * 4);
    const char* rnd = std::getenv("AVSE_ABL_RANDOM");
    if (rnd && rnd[0] == '1') {
        std::vector<uint16_t> h((size_t)N * H * H * C);
        uint32_t st = 12345;
        auto next = [&] { st = st * 1664525u + 1013904223u; return st; };
        for (auto& v : h) v = (uint16_t)(0x3c00 + (next() >> 22)) ^ (uint16_t)((next() >> 31) << 15);
        (void)hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
        (void)hipMemcpy(w, h.data(), (size_t)100 * C * 64, hipMemcpyHostToDevice);
    } else {
        (void)hipMemset(in, 0, (size_t)N * H * H * C * 2);
        (void)hipMemset(w, 0, (size_t)100 * C * 64);
    }
    (void)hipMemset(sc, 0, C * 4);
    (void)hipMemset(sh, 0, C * 4);
    a.in = in; a.out = out; a.w = w; a.scale = sc; a.shift = sh;
    const double flop = 2.0 * N * H * H * C * C * 25;
    const int reps = 10;
    auto rep = [&](const char* name, float ms) {
        std::printf("%-34s %8.4f ms  %7.1f TF/s\n", name, ms, flop / (ms * 1e-3) / 1e12);
    };
    rep("full", run<0>(a, reps));
    rep("no frag reads (1)", run<1>(a, reps));
    rep("no barrier (2)", run<2>(a, reps));
    rep("no halo staging (4)", run<4>(a, reps));
    rep("no weight stream (8)", run<8>(a, reps));
    rep("no frag reads+weights (9)", run<9>(a, reps));
    rep("no reads+weights+barrier (11)", run<11>(a, reps));
    rep("MFMA only (15)", run<15>(a, reps));
    rep("no MFMA (16)", run<16>(a, reps));
    return 0;
}
