// The layer plan of /root/reference/network.py:17-175 (shared by the inference path, capi.hip, and the
// training step, train.hip): kinds, channel counts, kernel sizes, strides, input grids, BN / pool flags, TF
// 'SAME' geometry, and the canonical weight-blob size (include/avse.h, avse_weights_load).
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

// audio 80x20x1, video 128x128x5 (data_processor.py:12, :47-55)
inline constexpr LayerDef kLayers[] = {
    {"a_conv1", CONV, 1, 64, 5, 5, 2, 2, 80, 20, true, false, 64},      // network.py:89
    {"a_conv2", CONV, 64, 64, 4, 4, 1, 1, 40, 10, true, false, 64},     // :93
    {"a_conv3", CONV, 64, 128, 4, 4, 2, 2, 40, 10, true, false, 128},   // :97
    {"a_conv4", CONV, 128, 128, 2, 2, 2, 1, 20, 5, true, false, 128},   // :101
    {"a_conv5", CONV, 128, 128, 2, 2, 2, 1, 10, 5, true, false, 128},   // :105
    {"v_conv1", CONV, 5, 128, 5, 5, 1, 1, 128, 128, true, true, 128},   // :139
    {"v_conv2", CONV, 128, 128, 5, 5, 1, 1, 64, 64, true, true, 128},   // :145
    {"v_conv3", CONV, 128, 256, 3, 3, 1, 1, 32, 32, true, true, 256},   // :151
    {"v_conv4", CONV, 256, 256, 3, 3, 1, 1, 16, 16, true, true, 256},   // :157
    {"v_conv5", CONV, 256, 512, 3, 3, 1, 1, 8, 8, true, true, 512},     // :163
    {"v_conv6", CONV, 512, 512, 3, 3, 1, 1, 4, 4, true, true, 512},     // :169
    {"enc_dense", DENSE, 5248, 1312, 1, 1, 1, 1, 1, 1, true, false, 1312},   // :56
    {"dec_dense1", DENSE, 1312, 1312, 1, 1, 1, 1, 1, 1, true, false, 1312},  // :69
    {"dec_dense2", DENSE, 1312, 3200, 1, 1, 1, 1, 1, 1, true, false, 128},   // :75-78
    {"d_deconv1", DECONV, 128, 128, 2, 2, 2, 1, 5, 5, true, false, 128},     // :113
    {"d_deconv2", DECONV, 128, 128, 2, 2, 2, 1, 10, 5, true, false, 128},    // :117
    {"d_deconv3", DECONV, 128, 128, 4, 4, 2, 2, 20, 5, true, false, 128},    // :121
    {"d_deconv4", DECONV, 128, 64, 4, 4, 1, 1, 40, 10, true, false, 64},     // :125
    {"d_deconv5", DECONV, 64, 64, 5, 5, 2, 2, 40, 10, true, false, 64},      // :129
    {"d_deconv6", DECONV, 64, 1, 1, 1, 1, 1, 80, 20, false, false, 0},       // :133
};
inline constexpr int kNumLayers = sizeof(kLayers) / sizeof(kLayers[0]);
inline constexpr float kBnEps = 1e-3f;

inline int same_out(int n, int s) { return (n + s - 1) / s; }
inline int same_pad_before(int n, int k, int s) {
    const int out = same_out(n, s);
    int tot = (out - 1) * s + k - n;
    if (tot < 0) tot = 0;
    return tot / 2;
}

inline int64_t blob_floats() {
    int64_t n = 0;
    for (int i = 0; i < kNumLayers; ++i) {
        const LayerDef& L = kLayers[i];
        n += (int64_t)L.kh * L.kw * L.cin * L.cout + L.cout;
        if (L.bn) n += 4 * (int64_t)L.bn_channels;
    }
    return n;
}

}  // namespace avse
