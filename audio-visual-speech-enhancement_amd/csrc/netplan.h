// The layer plan of /root/reference/network.py:17-175 (shared by the inference path, capi.hip, and the
// training step, train.hip): kinds, channel counts, kernel sizes, strides, input grids, BN / pool flags, TF
// 'SAME' geometry, and the canonical weight-blob size (include/avse.h, avse_weights_load).
//
// The reference builds the network from the shapes of its inputs (network.py:17-40, build(audio_spectrogram_shape,
// video_shape)): audio [80, T] with T = spectrogram frames per 200-ms slice (data_processor.py:44-52: 20 at 25 fps,
// 24 at 29.97 / 30 fps) and video [128, 128, F] with F = video frames per slice (data_processor.py:24: 5 at 25 and
// 29.97 fps, 6 at 30 fps).  T fixes the audio embedding (5 x ceil(T / 4) x 128), the concat width and through it
// the dense widths (shared_embedding_size = concat / 4, network.py:55) and the decoder grids; F is v_conv1's Cin.
#pragma once
#include <stdint.h>

namespace avse {

enum Kind { CONV = 0, DECONV = 1, DENSE = 2 };

struct LayerDef {
    const char* name;
    Kind kind;
    int cin, cout, kh, kw, sh, sw;
    int hin, win;   // input spatial dims (1,1 for dense)
    bool bn, pool;
    int bn_channels;  // BN width (dec_dense2: 128 after Reshape)
};

inline constexpr int kNumLayers = 20;
inline constexpr float kBnEps = 1e-3f;
inline constexpr int kMels = 80, kVideoHW = 128;

constexpr int same_out_c(int n, int s) { return (n + s - 1) / s; }
inline int same_out(int n, int s) { return same_out_c(n, s); }
inline int same_pad_before(int n, int k, int s) {
    const int out = same_out(n, s);
    int tot = (out - 1) * s + k - n;
    if (tot < 0) tot = 0;
    return tot / 2;
}

struct NetPlan {
    int T = 0, F = 0;          // spectrogram frames per slice, video frames per slice
    int W5 = 0;                // audio embedding width (5 x W5 x 128)
    int aemb = 0;              // audio embedding size = concat[0 : aemb]
    int cat = 0;               // concat width = aemb + 2048 (video 2 x 2 x 512)
    int emb = 0;               // shared embedding = cat / 4
    LayerDef L[kNumLayers];
};

// The plan Keras builds for build((80, T), (128, 128, F)).  valid() is false for shapes whose decoder output
// (80 x 4 ceil(ceil(T / 2) / 2)) would not be the input's 80 x T (fit / evaluate would fail in the reference too).
constexpr NetPlan make_plan(int T, int F) {
    NetPlan p{};
    p.T = T;
    p.F = F;
    const int w1 = same_out_c(T, 2), w3 = same_out_c(w1, 2);
    p.W5 = w3;
    p.aemb = 5 * w3 * 128;
    p.cat = p.aemb + 2 * 2 * 512;
    p.emb = p.cat / 4;
    const LayerDef L[kNumLayers] = {
        {"a_conv1", CONV, 1, 64, 5, 5, 2, 2, kMels, T, true, false, 64},            // network.py:89
        {"a_conv2", CONV, 64, 64, 4, 4, 1, 1, 40, w1, true, false, 64},             // :93
        {"a_conv3", CONV, 64, 128, 4, 4, 2, 2, 40, w1, true, false, 128},           // :97
        {"a_conv4", CONV, 128, 128, 2, 2, 2, 1, 20, w3, true, false, 128},          // :101
        {"a_conv5", CONV, 128, 128, 2, 2, 2, 1, 10, w3, true, false, 128},          // :105
        {"v_conv1", CONV, F, 128, 5, 5, 1, 1, 128, 128, true, true, 128},           // :139
        {"v_conv2", CONV, 128, 128, 5, 5, 1, 1, 64, 64, true, true, 128},           // :145
        {"v_conv3", CONV, 128, 256, 3, 3, 1, 1, 32, 32, true, true, 256},           // :151
        {"v_conv4", CONV, 256, 256, 3, 3, 1, 1, 16, 16, true, true, 256},           // :157
        {"v_conv5", CONV, 256, 512, 3, 3, 1, 1, 8, 8, true, true, 512},             // :163
        {"v_conv6", CONV, 512, 512, 3, 3, 1, 1, 4, 4, true, true, 512},             // :169
        {"enc_dense", DENSE, p.cat, p.emb, 1, 1, 1, 1, 1, 1, true, false, p.emb},   // :56
        {"dec_dense1", DENSE, p.emb, p.emb, 1, 1, 1, 1, 1, 1, true, false, p.emb},  // :69
        {"dec_dense2", DENSE, p.emb, p.aemb, 1, 1, 1, 1, 1, 1, true, false, 128},   // :75-78
        {"d_deconv1", DECONV, 128, 128, 2, 2, 2, 1, 5, w3, true, false, 128},       // :113
        {"d_deconv2", DECONV, 128, 128, 2, 2, 2, 1, 10, w3, true, false, 128},      // :117
        {"d_deconv3", DECONV, 128, 128, 4, 4, 2, 2, 20, w3, true, false, 128},      // :121
        {"d_deconv4", DECONV, 128, 64, 4, 4, 1, 1, 40, 2 * w3, true, false, 64},    // :125
        {"d_deconv5", DECONV, 64, 64, 5, 5, 2, 2, 40, 2 * w3, true, false, 64},     // :129
        {"d_deconv6", DECONV, 64, 1, 1, 1, 1, 1, kMels, 4 * w3, false, false, 0},   // :133
    };
    for (int i = 0; i < kNumLayers; ++i) p.L[i] = L[i];
    return p;
}

// T <= 64: the range the kernels' 32-bit activation / gather-map indexing is validated for (T = 20 at 25 fps, 24 at
// 29.97 / 30 fps; a 1023-clip training batch keeps every tensor far below 2^31 elements there)
constexpr bool plan_valid(int T, int F) { return T >= 4 && T % 4 == 0 && T <= 64 && F >= 1 && F <= 8; }

// audio 80x20x1, video 128x128x5 (data_processor.py:12, :47-55 at 16 kHz / 25 fps): the benchmarked network
inline constexpr NetPlan kPlan25 = make_plan(20, 5);
static_assert(kPlan25.cat == 5248 && kPlan25.emb == 1312 && kPlan25.aemb == 3200, "25-fps plan");

inline int64_t blob_floats(const NetPlan& p) {
    int64_t n = 0;
    for (int i = 0; i < kNumLayers; ++i) {
        const LayerDef& L = p.L[i];
        n += (int64_t)L.kh * L.kw * L.cin * L.cout + L.cout;
        if (L.bn) n += 4 * (int64_t)L.bn_channels;
    }
    return n;
}

}  // namespace avse
