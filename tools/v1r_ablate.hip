// Ablation timing of the v_conv1 kernel (k_conv_v1r<ABL>, conv_v1r.hip) at the bench shape (N=512,
// 128x128x5 f32 video -> 64x64x128 bf16).  Timing only: outputs are meaningless for ABL != 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o _v1r_ablate v1r_ablate.hip
#include <cstdio>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/conv_v1r.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
int ensure_lds_attr(const void* fn, int bytes) {
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 2;
}
}  // namespace avse

using namespace avse;

template <int ABL>
float run(const HaloArgs& a, int reps) {
    (void)hipFuncSetAttribute((const void*)k_conv_v1r<ABL>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_conv_v1r<ABL>, dim3(256), dim3(512), LDS_BYTES, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_conv_v1r<ABL>, dim3(256), dim3(512), LDS_BYTES, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int N = 512, H = 128, C = 128;
    HaloArgs a{};
    a.variant = HALO_V1;
    a.N = N; a.Hc = H; a.Wc = H; a.Ci = 5; a.Co = C;
    a.out_clip_stride = (long long)(H / 2) * (H / 2) * C;
    a.out_pix_stride = C;
    void *out, *w;
    float *video, *mean, *stdv, *sc, *sh;
    (void)hipMalloc(&video, (size_t)N * H * H * 5 * 4);
    (void)hipMalloc(&mean, (size_t)H * H * 4);
    (void)hipMalloc(&stdv, (size_t)H * H * 4);
    (void)hipMalloc(&out, (size_t)N * (H / 2) * (H / 2) * C * 2);
    (void)hipMalloc(&w, (size_t)C * 160 * 2);
    (void)hipMalloc(&sc, C * 4);
    (void)hipMalloc(&sh, C * 4);
    {   // random data: zero operands let the chip hold a higher clock under MFMA load
        std::vector<float> hv((size_t)N * H * H * 5);
        unsigned s = 12345u;
        for (auto& x : hv) { s = s * 1664525u + 1013904223u; x = (float)(s >> 24); }
        (void)hipMemcpy(video, hv.data(), hv.size() * 4, hipMemcpyHostToDevice);
        std::vector<unsigned short> hw((size_t)C * 160);
        for (auto& x : hw) { s = s * 1664525u + 1013904223u; x = (unsigned short)(0x3c00 + ((s >> 20) & 0x3ff) - 0x200); }
        (void)hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
        std::vector<float> m((size_t)H * H, 128.f), one(C, 1.f);
        (void)hipMemcpy(mean, m.data(), m.size() * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(sc, one.data(), C * 4, hipMemcpyHostToDevice);
        (void)hipMemset(sh, 0, C * 4);
    }
    std::vector<float> ones((size_t)H * H, 1.f);
    (void)hipMemcpy(stdv, ones.data(), ones.size() * 4, hipMemcpyHostToDevice);
    a.video = video; a.vmean = mean; a.vstd = stdv; a.out = out; a.w = w; a.scale = sc; a.shift = sh;
    const double flop = 2.0 * N * H * H * C * 125;
    const int reps = 10;
    auto rep = [&](const char* name, float ms) {
        std::printf("%-34s %8.4f ms  %7.1f TF/s (125-K)\n", name, ms, flop / (ms * 1e-3) / 1e12);
    };
    rep("full", run<0>(a, reps));
    rep("no output pass (1)", run<1>(a, reps));
    rep("no loader window work (2)", run<2>(a, reps));
    rep("no MFMA / frags (4)", run<4>(a, reps));
    rep("no barrier (8)", run<8>(a, reps));
    rep("no output pass, no window (3)", run<3>(a, reps));
    rep("only MFMA+frags: (1|2|8)", run<11>(a, reps));
    rep("full (again)", run<0>(a, reps));
    return 0;
}
