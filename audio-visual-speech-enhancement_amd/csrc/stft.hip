// K1: fused STFT -> |X| -> Slaney mel -> dB (-> top_db clamp, -> slicing) for gfx950.
//
// Replaces librosa.core.stft / magphase / filters.mel / amplitude_to_db as called by
// signal_to_spectrogram (/root/reference/data_processor.py:77-96) and the slicing of
// preprocess_audio_signal (data_processor.py:49-57).
//
// n_fft = 640 (16 kHz / 25 fps, data_processor.py:44) is not a power of two.  The real
// 640-point frame is packed as a 320-point complex sequence z[n] = x[2n] + i x[2n+1] and
// transformed with a 16 x 20 Cooley-Tukey split, entirely within one wavefront:
//   step 1: lane (frame f, n1 in [0,16)) does a 20-point DFT (4 x 5) over n2 of
//           z[n1 + 16 n2] in registers, multiplies by W320^{n1 k2}, writes LDS
//   step 2: lane (f, k2 in [0,20)) does a 16-point DFT (4 x 4) over n1 -> Z[k2 + 20 k1]
//   step 3: lane (f, k) untangles X[k], X[320-k] from Z[k], Z[320-k]  -> |X| in LDS
//   step 4: lane (f, mel band) sparse Slaney dot (<= max_width bins) -> dB
// Each 448-lane block handles one chunk of up to 21 frames of one utterance, 3 frames per
// wave (48 / 60 active lanes in steps 1 / 2).  When the chunk covers the whole utterance (the
// 200-ms segment case: 3200 samples -> 21 frames) the top_db clamp (max over the WHOLE
// [80, T] array, including the frame the slicing later drops) happens in-kernel; otherwise each
// chunk publishes its max with an ordered-uint atomicMax and a clamp kernel follows.
//
// Other n_fft (e.g. 533 at 29.97 fps) use k_spec_dft: a direct DFT, one block per frame.
#include "avse_common.h"
#include "fft_common.h"

namespace avse {

namespace {

constexpr int FPG = 3;          // frames per pass
constexpr int CHUNK = 21;       // frames per block (7 passes)
constexpr int ZS = 340;         // float2 slots per frame in LDS (20 rows x 17, padded)

__device__ __forceinline__ float sample_at(const float* __restrict__ s, long long L, long long i, int pad_mode) {
    if (i < 0) {
        if (pad_mode != 0) return 0.f;
        i = -i;
    } else if (i >= L) {
        if (pad_mode != 0) return 0.f;
        i = 2 * (L - 1) - i;
    }
    return s[i];
}

__device__ __forceinline__ float2 sample_pair(const float* __restrict__ s, long long L, long long i, int pad_mode) {
    if (i >= 0 && i + 1 < L) return *reinterpret_cast<const float2*>(s + i);
    return make_float2(sample_at(s, L, i, pad_mode), sample_at(s, L, i + 1, pad_mode));
}

__device__ __forceinline__ unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ long long out_index(int spf, int n_slices, int n_mels, int T, long long u, int m, int t) {
    if (spf > 0) {
        int sl = t / spf;
        if (sl >= n_slices) return -1;
        return ((u * n_slices + sl) * n_mels + m) * (long long)spf + (t - sl * spf);
    }
    return (u * n_mels + m) * (long long)T + t;
}

// One block per (chunk of CHUNK frames, utterance): wave w owns frames [3w, 3w + 3) of the chunk, so a
// 21-frame chunk is one pass of 7 waves (was one 64-lane wave walking 7 passes: ~110 us of serial
// latency per utterance).  Twiddles, window and the Slaney table live in LDS — the per-weight global
// loads of the mel dot were a dependent-latency chain.  |X| of a frame aliases its FFT buffer.
constexpr int WAVES = CHUNK / FPG;     // 7
constexpr int MEL_LDS_CAP = 6144;      // floats of the [n_mels][max_width] table staged in LDS

template <bool MEL_LDS>
__global__ __launch_bounds__(64 * WAVES) void k_spec640(SpecArgs a, int n_chunks) {
    __shared__ float2 zbuf[WAVES * FPG * ZS];
    __shared__ float dbuf[80 * CHUNK];
    __shared__ float2 twl[640];
    __shared__ float2 winl[320];
    __shared__ float wmax[WAVES];
    extern __shared__ __attribute__((aligned(16))) float mel_sm[];   // [n_mels * mw] weights, start, width

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int chunk = blockIdx.x;
    const long long u = blockIdx.y;
    const int T = a.n_frames;
    const int t0 = chunk * CHUNK;
    const int nf = min(CHUNK, T - t0);
    const int g = FPG * wave;                       // this wave's first frame in the chunk
    const int ng = max(0, min(FPG, nf - g));
    const long long L = a.n_samples;
    const float* __restrict__ sig = a.sig + u * L;
    const int n_mels = a.n_mels, mw = a.mel_max_width;
    float* mel_w = mel_sm;
    int* mel_st = reinterpret_cast<int*>(mel_sm + (MEL_LDS ? n_mels * mw : 0));
    int* mel_wd = mel_st + n_mels;

    for (int i = tid; i < 640; i += 64 * WAVES) twl[i] = a.twiddle[i];
    for (int i = tid; i < 320; i += 64 * WAVES) winl[i] = reinterpret_cast<const float2*>(a.window)[i];
    if (MEL_LDS)
        for (int i = tid; i < n_mels * mw; i += 64 * WAVES) mel_w[i] = a.mel_weight[i];
    for (int i = tid; i < n_mels; i += 64 * WAVES) {
        mel_st[i] = a.mel_start[i];
        mel_wd[i] = a.mel_width[i];
    }
    // samples of step 1 (issued before the table barrier so their latency overlaps it)
    const int f1 = lane >> 4, n1 = lane & 15;
    float2 x[20];
    if (f1 < ng) {
        const long long s0 = (long long)(t0 + g + f1) * a.hop - 320;
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) x[n2] = sample_pair(sig, L, s0 + 2 * (n1 + 16 * n2), a.pad_mode);
    }
    __syncthreads();

    float2* zw = zbuf + wave * FPG * ZS;
    // ---- step 1: 20-point DFTs over n2, lane = (f, n1) ----
    if (f1 < ng) {
        float2 v[20];
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) {
            const float2 w = winl[n1 + 16 * n2];
            v[n2] = make_float2(x[n2].x * w.x, x[n2].y * w.y);
        }
        dft20(v, twl);
        // v[5c + d] = Y[c + 4d]; twiddle W320^{n1 k2} = W640^{2 n1 k2}
        float2* zf = zw + f1 * ZS;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const int k2 = c + 4 * d;
                float2 y = v[5 * c + d];
                if (k2) y = cmul(y, twl[(2 * n1 * k2) % 640]);
                zf[k2 * 17 + n1] = y;
            }
    }
    __syncthreads();
    // ---- step 2: 16-point DFTs over n1, lane = (f, k2) ----
    {
        const int f = lane / 20, k2 = lane - 20 * (lane / 20);
        const bool act = f < ng;
        float2 v[16];
        float2* zf = zw + min(f, FPG - 1) * ZS;
        if (act) {
#pragma unroll
            for (int n = 0; n < 16; ++n) v[n] = zf[k2 * 17 + n];
        }
        __syncthreads();
        if (act) {
            dft16(v, twl);
            // v[4c + d] = Z[k2 + 20 (c + 4d)]
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int d = 0; d < 4; ++d) zf[k2 + 20 * (c + 4 * d)] = v[4 * c + d];
        }
    }
    __syncthreads();
    // ---- step 3: real-FFT untangling + magnitude, item = (f, k), k in [0,160]; |X| overwrites Z ----
    constexpr int IT3 = (FPG * 161 + 63) / 64;
    float mk[IT3], mm[IT3];
#pragma unroll
    for (int j = 0; j < IT3; ++j) {
        const int it = lane + 64 * j;
        if (it >= ng * 161) break;
        const int f = it / 161, k = it - 161 * f;
        const float2* zf = zw + f * ZS;
        const float2 zk = zf[k];
        const float2 zm = zf[k == 0 ? 0 : 320 - k];
        // E = (Zk + conj Zm)/2 ; O = -i/2 (Zk - conj Zm)
        const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
        const float2 O = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
        const float2 WO = cmul(twl[k], O);
        const float2 X = cadd(E, WO);
        const float2 Xm = make_float2(E.x - WO.x, -(E.y - WO.y));   // X[320 - k] = conj(E - W^k O)
        mk[j] = sqrtf(X.x * X.x + X.y * X.y);
        mm[j] = sqrtf(Xm.x * Xm.x + Xm.y * Xm.y);
        if (a.stft_ri) {
            const long long t = t0 + g + f;
            float2* o = reinterpret_cast<float2*>(a.stft_ri);
            o[(u * 321 + k) * T + t] = X;
            if (k != 160) o[(u * 321 + (320 - k)) * T + t] = Xm;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT3; ++j) {
        const int it = lane + 64 * j;
        if (it >= ng * 161) break;
        const int f = it / 161, k = it - 161 * f;
        float* mf = reinterpret_cast<float*>(zw + f * ZS);
        mf[k] = mk[j];
        mf[320 - k] = mm[j];
    }
    __syncthreads();
    // ---- step 4: Slaney mel + dB, item = (f, m) ----
    float vmax = -INFINITY;
    for (int it = lane; it < ng * n_mels; it += 64) {
        const int f = it / n_mels, m = it - n_mels * f;
        const float* mf = reinterpret_cast<const float*>(zw + f * ZS) + mel_st[m];
        const float* wm = MEL_LDS ? mel_w + m * mw : a.mel_weight + m * mw;
        const int wdt = mel_wd[m];
        float acc = 0.f;
        for (int j = 0; j < wdt; ++j) acc = fmaf(mf[j], wm[j], acc);
        const float db = acc > a.amin ? 20.0f * log10f(acc) : a.db_floor;
        vmax = fmaxf(vmax, db);
        dbuf[m * CHUNK + g + f] = db;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    if (lane == 0) wmax[wave] = vmax;
    __syncthreads();
    vmax = wmax[0];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) vmax = fmaxf(vmax, wmax[w]);
    // ---- clamp / publish ----
    const bool single = (n_chunks == 1);
    const float floor_db = (single && a.top_db >= 0.f) ? vmax - a.top_db : -INFINITY;
    for (int it = tid; it < n_mels * nf; it += 64 * WAVES) {
        const int m = it / nf, tl = it - nf * m;
        const long long oi = out_index(a.spf, a.n_slices, n_mels, T, u, m, t0 + tl);
        if (oi >= 0) a.mel_db[oi] = fmaxf(dbuf[m * CHUNK + tl], floor_db);
    }
    if (!single && tid == 0) atomicMax(a.umax + u, f2ord(vmax));
}

// Direct DFT fallback for n_fft != 640: one 256-thread block per (frame, utterance).
__global__ __launch_bounds__(256) void k_spec_dft(SpecArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int N = a.n_fft, nb = N / 2 + 1;
    float* xb = sm;            // [N]
    float* mb = sm + N;        // [nb]
    const int t = blockIdx.x;
    const long long u = blockIdx.y;
    const long long L = a.n_samples;
    const float* sig = a.sig + u * L;
    const long long s0 = (long long)t * a.hop - N / 2;
    for (int n = threadIdx.x; n < N; n += 256) xb[n] = sample_at(sig, L, s0 + n, a.pad_mode) * a.window[n];
    __syncthreads();
    for (int k = threadIdx.x; k < nb; k += 256) {
        float re = 0.f, im = 0.f;
        int idx = 0;
        for (int n = 0; n < N; ++n) {
            const float2 w = a.twiddle[idx];
            re = fmaf(xb[n], w.x, re);
            im = fmaf(xb[n], w.y, im);
            idx += k;
            if (idx >= N) idx -= N;
        }
        mb[k] = sqrtf(re * re + im * im);
        if (a.stft_ri) reinterpret_cast<float2*>(a.stft_ri)[(u * nb + k) * a.n_frames + t] = make_float2(re, im);
    }
    __syncthreads();
    float vmax = -INFINITY;
    for (int m = threadIdx.x; m < a.n_mels; m += 256) {
        const float* mf = mb + a.mel_start[m];
        const float* wm = a.mel_weight + m * a.mel_max_width;
        float acc = 0.f;
        for (int j = 0; j < a.mel_width[m]; ++j) acc = fmaf(mf[j], wm[j], acc);
        const float db = acc > a.amin ? 20.0f * log10f(acc) : a.db_floor;
        vmax = fmaxf(vmax, db);
        const long long oi = out_index(a.spf, a.n_slices, a.n_mels, a.n_frames, u, m, t);
        if (oi >= 0) a.mel_db[oi] = db;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    if ((threadIdx.x & 63) == 0) atomicMax(a.umax + u, f2ord(vmax));
}

__global__ void k_spec_clamp(SpecArgs a) {
    const long long per_u = (a.spf > 0) ? (long long)a.n_slices * a.n_mels * a.spf : (long long)a.n_mels * a.n_frames;
    const long long total = per_u * a.n_utt;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const long long u = i / per_u;
        const float fl = ord2f(a.umax[u]) - a.top_db;
        a.mel_db[i] = fmaxf(a.mel_db[i], fl);
    }
}

}  // namespace

int launch_spectrogram(const SpecArgs& a, hipStream_t s) {
    if (a.n_utt <= 0) return 0;
    const bool need_clamp_pass = a.top_db >= 0.f;
    if (a.n_fft == 640) {
        const int n_chunks = (a.n_frames + CHUNK - 1) / CHUNK;
        if (n_chunks > 1) AVSE_HIP_CHECK(hipMemsetAsync(a.umax, 0, sizeof(unsigned) * a.n_utt, s));
        const bool mel_lds = a.n_mels * a.mel_max_width <= MEL_LDS_CAP;
        const size_t shm = sizeof(float) * ((mel_lds ? a.n_mels * a.mel_max_width : 0) + 2 * a.n_mels);
        if (mel_lds)
            hipLaunchKernelGGL(k_spec640<true>, dim3(n_chunks, (unsigned)a.n_utt), dim3(64 * WAVES), shm, s, a, n_chunks);
        else
            hipLaunchKernelGGL(k_spec640<false>, dim3(n_chunks, (unsigned)a.n_utt), dim3(64 * WAVES), shm, s, a, n_chunks);
        AVSE_HIP_CHECK(hipGetLastError());
        if (n_chunks > 1 && need_clamp_pass) {
            hipLaunchKernelGGL(k_spec_clamp, dim3(1024), dim3(256), 0, s, a);
            AVSE_HIP_CHECK(hipGetLastError());
        }
        return 0;
    }
    AVSE_HIP_CHECK(hipMemsetAsync(a.umax, 0, sizeof(unsigned) * a.n_utt, s));
    const size_t shm = sizeof(float) * (a.n_fft + a.n_fft / 2 + 1);
    hipLaunchKernelGGL(k_spec_dft, dim3(a.n_frames, (unsigned)a.n_utt), dim3(256), shm, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    if (need_clamp_pass) {
        hipLaunchKernelGGL(k_spec_clamp, dim3(1024), dim3(256), 0, s, a);
        AVSE_HIP_CHECK(hipGetLastError());
    }
    return 0;
}

}  // namespace avse
