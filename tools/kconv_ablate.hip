// Timing ablations of the generic split-pair layer kernel (k_conv<_Float16, 64, true, true>, conv.hip) at d_deconv4's
// shape in the split dtype: N = 512 clips, 40 x 10 pixels, 128 -> 64 channels (256 halves of [h | l] pairs in), a 4 x 4
// stride-1 tap grid ('same'), fp32 blocked summation, pair output.  Timing only: outputs are meaningless for ABL != 0.
//   for A in 0 1 2 4 8 16 3 6; do hipcc --offload-arch=gfx950 -O3 -std=c++20 -DAVSE_KCONV_ABL=$A \
//       -o tools/kabl_$A.bin tools/kconv_ablate.hip; done      (then run each binary; it prints one line)
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <string>
#include <vector>

#include "../audio-visual-speech-enhancement_amd/csrc/conv.hip"

namespace avse {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
}  // namespace avse

using namespace avse;

int main() {
    const int N = 512, H = 40, W = 10, CI = 128, CO = 64, NT = 16;
    const int CIH = 2 * CI, KPAD = NT * CIH;   // halves
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.N = N; a.Hi = H; a.Wi = W; a.Ci = CIH; a.in_clip_stride = (long long)H * W * CIH;
    a.Hq = H; a.Wq = W; a.sy = a.sx = 1; a.oys = a.oxs = 1; a.Ho = H; a.Wo = W; a.Co = CO;
    a.out_clip_stride = (long long)H * W * 2 * CO; a.out_pix_stride = 2 * CO; a.out_c_off = 0;
    a.act = 1; a.nphase = 1; a.ksplit = 1; a.out_s16 = 1;
    a.ph[0].ntaps = NT; a.ph[0].kpad = KPAD; a.ph[0].w_off = 0; a.ph[0].tap_off = 0;
    std::vector<int2> taps;
    for (int t = 0; t < NT; ++t) taps.push_back(make_int2(t / 4 - 1, t % 4 - 1));
    void *in, *out, *w, *tp;
    float *sc, *sh;
    const size_t in_b = (size_t)N * H * W * CIH * 2, w_b = (size_t)CO * KPAD * 2;
    (void)hipMalloc(&in, in_b);
    (void)hipMalloc(&out, (size_t)N * H * W * 2 * CO * 2);
    (void)hipMalloc(&w, w_b);
    (void)hipMalloc(&tp, NT * sizeof(int2));
    (void)hipMalloc(&sc, CO * 4);
    (void)hipMalloc(&sh, CO * 4);
    std::vector<uint16_t> h(in_b / 2);
    uint32_t st = 12345;
    for (auto& v : h) { st = st * 1664525u + 1013904223u; v = (uint16_t)(0x2000 + (st >> 21)) ^ (uint16_t)(((st >> 7) & 1) << 15); }
    (void)hipMemcpy(in, h.data(), in_b, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, h.data(), w_b, hipMemcpyHostToDevice);
    (void)hipMemcpy(tp, taps.data(), NT * sizeof(int2), hipMemcpyHostToDevice);
    std::vector<float> one(CO, 1.f);
    (void)hipMemcpy(sc, one.data(), CO * 4, hipMemcpyHostToDevice);
    (void)hipMemset(sh, 0, CO * 4);
    a.in = in; a.out = out; a.w = w; a.taps = reinterpret_cast<const int2*>(tp); a.scale = sc; a.shift = sh;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 10; ++r) launch_conv(a, kConvSplitPairs, 0);
    const int reps = 50;
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch_conv(a, kConvSplitPairs, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * N * H * W * CO * (double)CI * NT;
    std::printf("ABL %2d  %8.4f ms  %6.1f TF/s (fp32 MAC)  %s\n", AVSE_KCONV_ABL, ms / reps, flop / (ms / reps * 1e-3) / 1e12,
                hipGetErrorString(hipGetLastError()));
    return 0;
}
