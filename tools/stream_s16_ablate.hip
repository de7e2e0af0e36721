// Ablation timing of the split-f16 stream kernel (k_conv_stream<5,16,16,1,true,LAT,ABL,BP,true>, conv_stream.hip) at
// the v_conv2 bench shape (N=512, 64x64, 128 -> 128 real channels = 256 halves of [h | l] pairs, 5x5, BP 4).  Timing
// only: outputs are meaningless for ABL != 0.  Random f16 data (MFMA power, hence clock, depends on it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o /tmp/s16abl tools/stream_s16_ablate.hip && /tmp/s16abl
//   (-DAVSE_S16_APLDS=1: the A'-from-LDS form of the third MFMA group)
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

template <int ABL, int LAT = 10, int BP = 4>
float run(const HaloArgs& a, int reps, int gx = 256) {
    using G = StreamGeom<5, 16, 16, 1, LAT, BP, true>;
    constexpr auto kern = k_conv_stream<5, 16, 16, 1, true, LAT, ABL, BP, true>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS + 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 6; ++r) hipLaunchKernelGGL(kern, dim3(gx, 1), dim3(512), G::LDS + 1024, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(gx, 1), dim3(512), G::LDS + 1024, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int N = 512, H = 64, C = 128, CI = 2 * C;
    HaloArgs a{};
    a.variant = HALO_K5;
    a.split = 1;
    a.out_mode = OUT_S16;
    a.N = N; a.Hc = H; a.Wc = H; a.Ci = CI; a.Co = C;
    a.out_pix_stride = 2 * C;
    a.out_clip_stride = (long long)(H / 2) * (H / 2) * 2 * C;
    const size_t in_b = (size_t)N * H * H * CI * 2, w_b = (size_t)(CI / 32) * 25 * C * 64;
    void *in, *out, *w;
    float *sc, *sh;
    (void)hipMalloc(&in, in_b);
    (void)hipMalloc(&out, (size_t)N * (H / 2) * (H / 2) * 2 * C * 2);
    (void)hipMalloc(&w, w_b);
    (void)hipMalloc(&sc, C * 4);
    (void)hipMalloc(&sh, C * 4);
    std::vector<uint16_t> h(in_b / 2);
    uint32_t st = 12345;
    auto next = [&] { st = st * 1664525u + 1013904223u; return st; };
    for (auto& v : h) v = (uint16_t)(0x2000 + (next() >> 21)) ^ (uint16_t)((next() >> 31) << 15);   // +-[2^-7, 2)
    (void)hipMemcpy(in, h.data(), in_b, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, h.data(), w_b, hipMemcpyHostToDevice);
    std::vector<float> one(C, 1.f);
    (void)hipMemcpy(sc, one.data(), C * 4, hipMemcpyHostToDevice);
    (void)hipMemset(sh, 0, C * 4);
    a.in = in; a.out = out; a.w = w; a.scale = sc; a.shift = sh;
    const double flop = 2.0 * N * H * H * C * C * 25;   // fp32 multiply-adds of the layer
    const int reps = 10;
    auto rep = [&](const char* name, float ms) {
        std::printf("%-40s %8.4f ms  %7.1f TF/s (fp32 MAC)\n", name, ms, flop / (ms * 1e-3) / 1e12);
    };
    rep("full", run<0>(a, reps));
    rep("half the B fragment reads (256)", run<256>(a, reps));
    rep("full", run<0>(a, reps));
    rep("half the B fragment reads (256)", run<256>(a, reps));
    rep("no halo pieces (1)", run<1>(a, reps));
    rep("no weight streaming (2)", run<2>(a, reps));
    rep("no loads (3)", run<3>(a, reps));
    rep("no wait/barrier (4)", run<4>(a, reps));
    rep("no frag reads (8)", run<8>(a, reps));
    rep("no frag reads, no loads (11)", run<11>(a, reps));
    rep("MFMA + permlane only (15)", run<15>(a, reps));
    rep("no MFMAs (16)", run<16>(a, reps));
    rep("full again", run<0>(a, reps));
    unsigned long long* prof;
    (void)hipMalloc(&prof, 256 * 8 * 4 * 8);
    a.prof = prof;
    // instrumented variants: cycles per slice of the compute / loader waves, and the effective shader clock =
    // compute-wave cycles per CU (all of its slices) / kernel time
    auto inst = [&](const char* name, float ms) {
        std::vector<unsigned long long> hp(256 * 8 * 4);
        (void)hipMemcpy(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost);
        double s[2][3] = {}, steps[2] = {};
        for (int b = 0; b < 256; ++b)
            for (int wv = 0; wv < 8; ++wv) {
                const int role = wv >= 4;
                for (int k = 0; k < 3; ++k) s[role][k] += (double)hp[(b * 8 + wv) * 4 + k];
                steps[role] += (double)hp[(b * 8 + wv) * 4 + 3];
            }
        const double cyc = (s[0][0] + s[0][1] + s[0][2]) / 4 / 256;   // per compute wave = per CU
        std::printf("%-28s %7.4f ms  clock %.2f GHz | compute work %6.1f wait %5.1f bar %5.1f | loader work %6.1f "
                    "wait %5.1f bar %6.1f (cycles/slice)\n", name, ms, cyc / (ms * 1e6), s[0][0] / steps[0],
                    s[0][1] / steps[0], s[0][2] / steps[0], s[1][0] / steps[1], s[1][1] / steps[1], s[1][2] / steps[1]);
    };
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("full (128)", run<128>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("no pieces (129)", run<129>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("no weights (130)", run<130>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("no loads (131)", run<131>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("no frag reads (136)", run<136>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("L2-resident input (192)", run<192>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("full again (128)", run<128>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("MFMA + permlane only (143)", run<143>(a, 1));
    (void)hipMemset(prof, 0, 256 * 8 * 4 * 8);
    inst("no frag reads, no loads (139)", run<139>(a, 1));
    rep("L2-resident input (64)", run<64>(a, reps));
    return 0;
}
