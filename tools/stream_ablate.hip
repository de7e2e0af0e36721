// Ablation timing of the persistent warp-specialised kernel (k_conv_stream<5,16,16,1,M16,LAT,ABL>, conv_stream.hip) at
// the v_conv2 bench shape (N=512, 64x64x128 -> 128, 5x5).  Timing only: outputs are meaningless for
// ABL != 0.   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o _stream_ablate stream_ablate.hip
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <algorithm>

#include "../audio-visual-speech-enhancement_amd/csrc/conv_stream.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int ensure_lds_attr(const void* fn, int bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 2;
}
}  // namespace avse

using namespace avse;

template <int ABL, int LAT = 10, bool M16 = true, int BP = 1>
float run(const HaloArgs& a, int reps, int gx = 256) {
    using G = StreamGeom<5, 16, 16, 1, LAT, BP>;
    (void)hipFuncSetAttribute((const void*)k_conv_stream<5, 16, 16, 1, M16, LAT, ABL, BP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G::LDS + 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 10; ++r)   // warm-up long enough for the clock to settle under MFMA load
        hipLaunchKernelGGL((k_conv_stream<5, 16, 16, 1, M16, LAT, ABL, BP>), dim3(gx, 1), dim3(512), G::LDS + 1024, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_conv_stream<5, 16, 16, 1, M16, LAT, ABL, BP>), dim3(gx, 1), dim3(512), G::LDS + 1024, 0, a);
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
    void *in, *out, *w;
    float *sc, *sh;
    (void)hipMalloc(&in, (size_t)N * H * H * C * 2);
    (void)hipMalloc(&out, (size_t)N * (H / 2) * (H / 2) * C * 2);
    (void)hipMalloc(&w, (size_t)100 * C * 64);
    (void)hipMalloc(&sc, C * 4);
    (void)hipMalloc(&sh, C * 4);
    // AVSE_ABL_RANDOM=1: random bf16 activations / weights (MFMA power, hence clock, depends on data)
    const char* rnd = std::getenv("AVSE_ABL_RANDOM");
    if (rnd && rnd[0] == '1') {
        std::vector<uint16_t> h((size_t)N * H * H * C);
        uint32_t st = 12345;
        auto next = [&] { st = st * 1664525u + 1013904223u; return st; };
        for (auto& v : h) v = (uint16_t)(0x3c00 + (next() >> 22)) ^ (uint16_t)((next() >> 31) << 15);   // +-[0.0078, 0.03)
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
    const int reps = 20;
    auto rep = [&](const char* name, float ms) {
        std::printf("%-34s %8.4f ms  %7.1f TF/s\n", name, ms, flop / (ms * 1e-3) / 1e12);
    };
    rep("full, 32x32x16 compute waves", run<0, 10, false>(a, reps));
    rep("MFMA only, 32x32x16 (15)", run<15, 10, false>(a, reps));
    rep("full", run<0, 10>(a, reps));
    rep("full, 240 workgroups", run<0, 10>(a, reps, 240));
    rep("full, 224 workgroups", run<0, 10>(a, reps, 224));
    rep("full", run<0, 10>(a, reps));
    rep("full, 240 workgroups", run<0, 10>(a, reps, 240));
    rep("full, barrier every step (BP 1)", run<0, 10, true, 1>(a, reps));
    rep("full", run<0, 10>(a, reps));
    rep("full, barrier every step (BP 1)", run<0, 10, true, 1>(a, reps));
    rep("no halo pieces (1)", run<1, 10>(a, reps));
    rep("no weight streaming (2)", run<2, 10>(a, reps));
    rep("no loads at all (3)", run<3, 10>(a, reps));
    rep("no wait/barrier (4)", run<4, 10>(a, reps));
    rep("no frag reads (8)", run<8, 10>(a, reps));
    rep("MFMA only (15)", run<15, 10>(a, reps));
    rep("L2-resident input (64)", run<64, 10>(a, reps));
    rep("LAT5", run<0, 5>(a, reps));
    rep("full (again: clock drift check)", run<0, 10>(a, reps));
    // per-step cycle split (s_memtime; the counters add a few instructions per step)
    unsigned long long* prof;
    (void)hipMalloc(&prof, 256 * 8 * 4 * 8);
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    a.prof = prof;
    rep("instrumented (128, 32x32x16)", run<128, 10, false>(a, reps));
    auto split = [&](const char* title) {
    std::vector<unsigned long long> hp(256 * 8 * 4);
    (void)hipMemcpy(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost);
    double s[2][3] = {}, steps[2] = {};
    for (int b = 0; b < 256; ++b)
        for (int wv = 0; wv < 8; ++wv) {
            const int role = wv >= 4;
            for (int k = 0; k < 3; ++k) s[role][k] += (double)hp[(b * 8 + wv) * 4 + k];
            steps[role] += (double)hp[(b * 8 + wv) * 4 + 3];
        }
    const char* names[2] = {"compute", "loader"};
    for (int r = 0; r < 2; ++r)
        std::printf("%s %-8s cycles/step: work %7.1f  wait(vm/lgkm) %7.1f  barrier %7.1f\n", title, names[r],
                    s[r][0] / steps[r], s[r][1] / steps[r], s[r][2] / steps[r]);
    };
    split("LAT10");
    rep("instrumented, no pieces (129)", run<129, 10, false>(a, reps));
    split("nopc ");
    rep("instrumented, L2 input (192)", run<192, 10, false>(a, reps));
    split("L2in ");
    rep("instrumented, M16 (128)", run<128, 10>(a, reps));
    split("M16  ");
    rep("instrumented, M16 no pieces (129)", run<129, 10>(a, reps));
    split("M16np");
    rep("instrumented, M16 BP1 (128)", run<128, 10, true, 1>(a, reps));
    split("M16b1");
    rep("instrumented (128, 32x32x16) again", run<128, 10, false>(a, reps));
    split("LAT10");
    {   // per-workgroup busy span (compute wave 0: work + wait + barrier): the persistent grid's tail imbalance
        std::vector<unsigned long long> hp(256 * 8 * 4);
        (void)hipMemcpy(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> tot;
        for (int b = 0; b < 256; ++b) tot.push_back((double)(hp[(b * 8) * 4] + hp[(b * 8) * 4 + 1] + hp[(b * 8) * 4 + 2]));
        std::sort(tot.begin(), tot.end());
        std::printf("per-WG cycles: min %.0f  p10 %.0f  median %.0f  p90 %.0f  max %.0f  (max/median %.3f)\n", tot[0], tot[25],
                    tot[128], tot[230], tot[255], tot[255] / tot[128]);
        for (int x = 0; x < 8; ++x) {   // by XCD (block % 8)
            double s = 0;
            for (int b = x; b < 256; b += 8) s += (double)(hp[(b * 8) * 4] + hp[(b * 8) * 4 + 1] + hp[(b * 8) * 4 + 2]);
            std::printf("  XCD %d mean %.0f\n", x, s / 32);
        }
    }
    return 0;
}
