// K6: mel-dB -> amplitude -> pinv(mel) -> x phase -> inverse real FFT -> Hann overlap-add ->
// window-sum-square normalisation -> centre trim, for gfx950.
//
// Replaces reconstruct_signal_from_spectrogram (/root/reference/data_processor.py:99-116):
//   librosa.db_to_amplitude (:101), np.dot(np.linalg.pinv(mel), .) (:112), librosa.istft (:114),
// fed by reconstruct_speech_signal (:60-74) with the mixture's complex STFT from K1 (the phase
// exp(i angle D) = D / |D| is taken in-kernel, so the mixture is not re-analysed).
//
// k_istft640 (n_fft 640): one 64-lane block per 3 frames of one utterance.  The 321-bin one-sided
// spectrum is folded into a 320-point complex sequence (E[k] + i O[k]) and inverted with the same
// in-register 20 x 16 DFTs as K1 through the conjugation identity IDFT(Z) = conj(DFT(conj Z)) / 320;
// each lane then writes two windowed output samples per frame.  k_istft_dft handles other sizes
// (n_fft = 2 (n_bins - 1), e.g. 532 at 29.97 fps) with a direct inverse DFT.  k_ola sums the <= 4
// overlapping frames of each output sample in increasing frame order (librosa's order), divides by
// the window sum-square where it exceeds float32 tiny, and drops n_fft/2 samples at both ends.
#include <algorithm>

#include "avse_common.h"
#include "fft_common.h"

#ifdef AVSE_NO_WPE   // A/B: no occupancy cap
#define AVSE_WPE4
#else
#define AVSE_WPE4 __attribute__((amdgpu_waves_per_eu(4)))
#endif

namespace avse {
namespace {

constexpr int FPG = 3;
constexpr int ZS = 340;

__device__ __forceinline__ float mel_at(const IstftArgs& a, long long u, int m, int t) {
    if (a.spf > 0) {
        const int sl = t / a.spf;
        return a.mel_db[((u * a.n_slices + sl) * a.n_mels + m) * (long long)a.spf + (t - sl * a.spf)];
    }
    return a.mel_db[(u * a.n_mels + m) * (long long)a.T + t];
}

// D / |D| (librosa.magphase; 1 where D == 0) as D * rsq(|D|^2): one v_rsq_f32 and two multiplies instead of a
// square root and two IEEE divisions (~10 instructions each; 16 per lane per chunk in k_istft_fused)
__device__ __forceinline__ float2 unit_phase(float2 d) {
    const float r2 = d.x * d.x + d.y * d.y;
    const float s = __builtin_amdgcn_rsqf(r2);
    return r2 > 0.f ? make_float2(d.x * s, d.y * s) : make_float2(1.f, 0.f);
}

// X[k] = (pinv(mel) @ 10^(dB/20))[k] * D[k]/|D[k]| for one frame, k in [0, nb)
__device__ __forceinline__ float2 spectrum_bin(const IstftArgs& a, const float* amp, long long u, int k, int t) {
    float acc = 0.f;
    for (int m = 0; m < a.n_mels; ++m) acc = fmaf(a.pinvT[m * a.nb + k], amp[m], acc);
    const float2 d = a.stft[(u * a.nb + k) * (long long)a.stft_frames + t];
    const float2 ph = unit_phase(d);
    return make_float2(acc * ph.x, acc * ph.y);
}

__global__ __launch_bounds__(64) void k_istft640(IstftArgs a) {
    __shared__ float amp[FPG][80];
    __shared__ float2 xb[FPG][324];
    __shared__ float2 zbuf[FPG * ZS];
    const int lane = threadIdx.x;
    const long long u = blockIdx.y;
    const int t0 = blockIdx.x * FPG;
    const int ng = min(FPG, a.T - t0);
    const float2* __restrict__ tw = a.twiddle;   // W640^k

    // db_to_amplitude: (10^(0.1 S))^0.5
    for (int it = lane; it < ng * a.n_mels; it += 64) {
        const int f = it / a.n_mels, m = it - f * a.n_mels;
        amp[f][m] = sqrtf(exp10f(0.1f * mel_at(a, u, m, t0 + f)));
    }
    __syncthreads();
    for (int it = lane; it < ng * 321; it += 64) {
        const int f = it / 321, k = it - f * 321;
        float2 x = spectrum_bin(a, amp[f], u, k, t0 + f);
        if (k == 0 || k == 320) x.y = 0.f;            // irfft ignores the DC / Nyquist imaginary parts
        xb[f][k] = x;
    }
    __syncthreads();
    // fold into Z'[k] = conj(E[k] + i O[k]), k in [0,320):
    //   E = (X[k] + conj X[320-k]) / 2,  O = (X[k] - conj X[320-k]) W640^{-k} / 2
    for (int it = lane; it < ng * 320; it += 64) {
        const int f = it / 320, k = it - f * 320;
        const float2 xk = xb[f][k], xm = cconj(xb[f][320 - k]);
        const float2 E = make_float2(0.5f * (xk.x + xm.x), 0.5f * (xk.y + xm.y));
        const float2 O = cmul(make_float2(0.5f * (xk.x - xm.x), 0.5f * (xk.y - xm.y)), cconj(tw[k]));
        const float2 Z = make_float2(E.x - O.y, E.y + O.x);   // E + i O
        zbuf[f * ZS + k] = cconj(Z);
    }
    __syncthreads();
    // forward 320-point DFT of Z' (step 1: 20-point over n2 of z[n1 + 16 n2], lane = (f, n1))
    {
        const int f = lane >> 4, n1 = lane & 15;
        float2 v[20];
        const bool act = f < ng;
        if (act) {
#pragma unroll
            for (int n2 = 0; n2 < 20; ++n2) v[n2] = zbuf[f * ZS + n1 + 16 * n2];
        }
        __syncthreads();
        if (act) {
            dft20(v, tw);
            float2* zf = zbuf + f * ZS;
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    const int k2 = c + 4 * d;
                    float2 y = v[5 * c + d];
                    if (k2) y = cmul(y, tw[(2 * n1 * k2) % 640]);
                    zf[k2 * 17 + n1] = y;
                }
        }
    }
    __syncthreads();
    // step 2: 16-point DFT over n1, lane = (f, k2); write the time samples
    {
        const int f = lane / 20, k2 = lane - 20 * (lane / 20);
        if (f < ng) {
            float2 v[16];
            const float2* zf = zbuf + f * ZS;
#pragma unroll
            for (int n1 = 0; n1 < 16; ++n1) v[n1] = zf[k2 * 17 + n1];
            dft16(v, tw);
            float* fr = a.frames + ((u * a.T) + t0 + f) * 640LL;
            const float s = 1.0f / 320.0f;
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int n = k2 + 20 * (c + 4 * d);       // z[n] = conj(out[n]) / 320
                    const float2 o = v[4 * c + d];
                    fr[2 * n] = o.x * s * a.window[2 * n];
                    fr[2 * n + 1] = -o.y * s * a.window[2 * n + 1];
                }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_istft_fused (n_fft 640, hop 160): one persistent 8-wave block per output chunk of OF = 21 hops
// (3,360 samples) of one utterance.  The chunk's samples are the overlap-add of frames
// [21 b - 1, 21 b + 22] (24 frames, 3 of them shared with each neighbour and recomputed), so the
// frames never leave LDS: the unfused path wrote 2,560 B per frame to a scratch buffer and re-read it in
// k_ola, and its per-bin 80-term dense pinv dot (25.7K global-load MACs per frame) was the dominant cost
// (2.4 ms for 10k clips).  Per chunk:
//   1. amp = 10^(dB/20) for the 24 frames -> LDS [24][80]
//   2. y = (M M^T)^{-1} amp by the Thomas recurrence (one lane per frame, coefficients from the host)
//   3. X[k] = M[j0][k] y[j0] + M[j0+1][k] y[j0+1] (pinv(M) amp = M^T y), times the mixture's unit phase,
//      read bin-major / frame-minor (24-frame runs of the [bin][frame] STFT); folded into the 320-point
//      complex sequence Z' of the real inverse FFT, both halves (k, 320 - k) by one lane
//   4. the in-register 20 x 16 DFTs of K1 (3 frames per wave) -> time samples in the frame's slot
//   5. window x overlap-add in increasing frame order / window sum-square -> the trimmed signal, coalesced
constexpr int OF = 21;                       // output hops per chunk
constexpr int FW = OF + 3;                   // frames per chunk (n_fft / hop - 1 = 3 extra)
constexpr int IWAVES = FW / FPG;             // 8

__device__ __forceinline__ void ibarrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(64 * IWAVES) void k_istft_fused(IstftArgs a, int n_chunks, int n_items) {
    __shared__ float2 zbuf[FW * ZS];            // frame f's slot: zbuf + f * ZS (Z', then 640 time samples)
    __shared__ float amp[FW][80];               // amplitudes, then y in place
    __shared__ float4 tri_l[80];
    __shared__ float win_l[640];
    __shared__ float2 tw[640];                  // W640^k
    __shared__ float4 bins_l[321];              // per bin: the two pinv weights and the first mel band
    const int T = a.T, n_mels = a.n_mels;
    const long long Lout = (long long)a.hop * (T - 1);

    // tables -> LDS once per (persistent) block: the DFT twiddles and bin weights were global-memory reads in
    // every item's dependency chain
    for (int i = threadIdx.x; i < n_mels; i += 64 * IWAVES) tri_l[i] = a.tri[i];
    for (int i = threadIdx.x; i < 640; i += 64 * IWAVES) {
        win_l[i] = a.window[i];
        tw[i] = a.twiddle[i];
    }
    for (int i = threadIdx.x; i < 321; i += 64 * IWAVES) bins_l[i] = a.bins[i];
    __syncthreads();

    for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));           // keep index math inside the loop (see k_spec640)
        const int lane = tid & 63, wave = tid >> 6;
        const int u = item / n_chunks, b = item - u * n_chunks;
        const int t_lo = max(0, b * OF - 1);
        const int t_hi = min(T - 1, b * OF + OF + 1);
        const int nfr = t_hi - t_lo + 1;

        // ---- 1. amplitudes (frame fastest: runs of consecutive frames of one band); all of a lane's loads
        //         (clamped in range) are issued before the first is used ----
        {
            constexpr int IT1 = (FW * 80 + 64 * IWAVES - 1) / (64 * IWAVES);   // 4 (n_mels <= 80, host-checked)
            float mv[IT1];
#pragma unroll
            for (int j = 0; j < IT1; ++j) {
                const int it = min(tid + 64 * IWAVES * j, FW * n_mels - 1);
                const int m = it / FW, f = it - FW * m;
                mv[j] = mel_at(a, u, m, t_lo + min(f, nfr - 1));
            }
#pragma unroll
            for (int j = 0; j < IT1; ++j) {
                const int it = tid + 64 * IWAVES * j;
                const int m = it / FW, f = it - FW * m;
                if (it < FW * n_mels && f < nfr) amp[f][m] = sqrtf(exp10f(0.1f * mv[j]));
            }
        }
        ibarrier();
        // ---- 2. Thomas solve, lanes 0..2 of every wave = frames wave + 8 lane; 8 bands per batch of loads ----
        if (lane < FPG) {
            const int f = wave + IWAVES * lane;
            if (f < nfr) {
                float* d = amp[f];
                float prev = 0.f;
                for (int i0 = 0; i0 < n_mels; i0 += 8) {
                    float dv[8];
                    float2 cv[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (i0 + q < n_mels) {
                            dv[q] = d[i0 + q];
                            cv[q] = make_float2(tri_l[i0 + q].x, tri_l[i0 + q].y);
                        }
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (i0 + q < n_mels) {
                            prev = (dv[q] - cv[q].x * prev) * cv[q].y;
                            d[i0 + q] = prev;
                        }
                }
                for (int i1 = n_mels - 2; i1 >= 0; i1 -= 8) {
                    float dv[8], cz[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (i1 - q >= 0) {
                            dv[q] = d[i1 - q];
                            cz[q] = tri_l[i1 - q].z;
                        }
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (i1 - q >= 0) {
                            prev = dv[q] - cz[q] * prev;
                            d[i1 - q] = prev;
                        }
                }
            }
        }
        ibarrier();
        // ---- 3. spectrum x unit phase, folded into Z' = conj(E + i O) (k) and E - i O (320 - k) ----
        // All of a lane's mixture-STFT loads are issued before any is used (one HBM latency per chunk).
        {
            constexpr int IT3 = (161 * FW + 64 * IWAVES - 1) / (64 * IWAVES);   // 8
            const float2* __restrict__ D = a.stft + (long long)u * a.nb * a.stft_frames + t_lo;
            float2 dk[IT3], dm[IT3];
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = tid + 64 * IWAVES * j;
                const int k = it / FW, f = it - FW * k;
                if (k <= 160 && f < nfr) {
                    dk[j] = D[(long long)k * a.stft_frames + f];
                    dm[j] = D[(long long)(k == 0 ? 320 : 320 - k) * a.stft_frames + f];
                }
            }
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = tid + 64 * IWAVES * j;
                const int k = it / FW, f = it - FW * k;
                asm volatile("" ::: "memory");           // one iteration's table loads at a time (register pressure)
                if (k > 160 || f >= nfr) continue;
                const int km = k == 0 ? 320 : 320 - k;
                const float4 bk = bins_l[k], bm = bins_l[km];
                const int jk = __float_as_int(bk.z), jm = __float_as_int(bm.z);
                const float* y = amp[f];
                const float ak = (jk >= 0 ? bk.x * y[jk] : 0.f) + (jk + 1 < n_mels && jk >= 0 ? bk.y * y[jk + 1] : 0.f);
                const float am = (jm >= 0 ? bm.x * y[jm] : 0.f) + (jm + 1 < n_mels && jm >= 0 ? bm.y * y[jm + 1] : 0.f);
                const float2 pk = unit_phase(dk[j]);
                const float2 pm = unit_phase(dm[j]);
                float2 xk = make_float2(ak * pk.x, ak * pk.y);
                float2 xm = make_float2(am * pm.x, am * pm.y);
                if (k == 0) { xk.y = 0.f; xm.y = 0.f; }           // irfft ignores the DC / Nyquist imaginary parts
                const float2 cxm = cconj(xm);
                const float2 E = make_float2(0.5f * (xk.x + cxm.x), 0.5f * (xk.y + cxm.y));
                const float2 O = cmul(make_float2(0.5f * (xk.x - cxm.x), 0.5f * (xk.y - cxm.y)), cconj(tw[k]));
                float2* zf = zbuf + f * ZS;
                zf[k] = make_float2(E.x - O.y, -(E.y + O.x));          // conj(E + i O)
                if (k != 0 && k != 160) zf[320 - k] = make_float2(E.x + O.y, E.y - O.x);   // E - i O
            }
        }
        ibarrier();
        // ---- 4. forward 320-point DFT of Z' per frame (wave = 3 frames) -> windowed samples ----
        {
            const int f = FPG * wave + (lane >> 4), n1 = lane & 15;
            const bool act = (lane >> 4) < FPG && f < nfr;
            float2 v[20];
            if (act) {
#pragma unroll
                for (int n2 = 0; n2 < 20; ++n2) v[n2] = zbuf[f * ZS + n1 + 16 * n2];
            }
            ibarrier();
            if (act) {
                dft20(v, tw);
                float2* zf = zbuf + f * ZS;
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 5; ++d) {
                        const int k2 = c + 4 * d;
                        float2 yv = v[5 * c + d];
                        if (k2) yv = cmul(yv, tw[(2 * n1 * k2) % 640]);
                        zf[k2 * 17 + n1] = yv;
                    }
            }
        }
        ibarrier();
        {
            const int f = FPG * wave + lane / 20, k2 = lane - 20 * (lane / 20);
            const bool act = lane < 20 * FPG && f < nfr;
            float2 v[16];
            float2* zf = zbuf + min(f, FW - 1) * ZS;
            if (act) {
#pragma unroll
                for (int n1 = 0; n1 < 16; ++n1) v[n1] = zf[k2 * 17 + n1];
            }
            ibarrier();
            if (act) {
                dft16(v, tw);
                float* fr = reinterpret_cast<float*>(zf);
                const float s = 1.0f / 320.0f;
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const int n = k2 + 20 * (c + 4 * d);       // z[n] = conj(out[n]) / 320
                        const float2 o = v[4 * c + d];
                        fr[2 * n] = o.x * s;                          // windowed in the overlap-add
                        fr[2 * n + 1] = -o.y * s;
                    }
            }
        }
        ibarrier();
        // ---- 5. overlap-add + window-sum-square + centre trim ----
        {
            const long long i0 = (long long)b * OF * 160;
            const int n_out = (int)min((long long)OF * 160, Lout - i0);
            float* __restrict__ out = a.sig + (long long)u * Lout + i0;
#pragma unroll 1
            for (int j = tid; j < n_out; j += 64 * IWAVES) {
                const int p = (int)(i0 + j) + 320;                 // position in the untrimmed signal
                const int tlo = max(0, (p - 640 + 160) / 160);     // first frame t with t*160 + 639 >= p
                const int thi = min(T - 1, p / 160);
                float yv = 0.f, wss = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {                      // <= 4 frames overlap, increasing t
                    const int t = thi - 3 + q;
                    if (t < tlo) continue;
                    const int o = p - 160 * t;
                    const float w = win_l[o];
                    yv += reinterpret_cast<const float*>(zbuf + (t - t_lo) * ZS)[o] * w;
                    wss += w * w;
                }
                if (wss > 1.17549435e-38f) yv /= wss;
                out[j] = yv;
            }
        }
        ibarrier();
    }
}

// direct inverse real DFT, one 256-thread block per (frame, utterance); N = 2 (nb - 1)
__global__ __launch_bounds__(256) void k_istft_dft(IstftArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* amp = sm;                                        // [n_mels]
    float2* xs = reinterpret_cast<float2*>(sm + 80);        // [nb]
    const int t = blockIdx.x;
    const long long u = blockIdx.y;
    const int N = a.N, nb = a.nb;
    for (int m = threadIdx.x; m < a.n_mels; m += 256) amp[m] = sqrtf(exp10f(0.1f * mel_at(a, u, m, t)));
    __syncthreads();
    for (int k = threadIdx.x; k < nb; k += 256) xs[k] = spectrum_bin(a, amp, u, k, t);
    __syncthreads();
    float* fr = a.frames + ((u * a.T) + t) * (long long)N;
    for (int n = threadIdx.x; n < N; n += 256) {
        // x[n] = (1/N) (Re X0 + (-1)^n Re X[N/2] + 2 sum_{k=1}^{N/2-1} Re(X_k e^{+2 pi i k n / N}))
        float acc = xs[0].x + ((n & 1) ? -xs[nb - 1].x : xs[nb - 1].x);
        float part = 0.f;
        int idx = n;
        for (int k = 1; k < nb - 1; ++k) {
            const float2 w = a.twiddle[idx];                // e^{-2 pi i idx / N}; conj for the inverse
            part = fmaf(xs[k].x, w.x, part);
            part = fmaf(xs[k].y, w.y, part);                // Re(X (cos + i sin)) = Xr cos - Xi sin, sin = -w.y
            idx += n;
            if (idx >= N) idx -= N;
        }
        fr[n] = (acc + 2.f * part) / (float)N * a.window[n];
    }
}

// overlap-add + window-sum-square normalisation + centre trim
__global__ void k_ola(IstftArgs a) {
    const long long L = (long long)a.hop * (a.T - 1);
    const long long total = L * a.n_utt;
    const int N = a.N;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const long long u = i / L;
        const long long p = i - u * L + N / 2;            // position in the untrimmed signal
        // frames t with t*hop <= p <= t*hop + N - 1
        const long long tlo = (p - N + 1 <= 0) ? 0 : (p - N + 1 + a.hop - 1) / a.hop;
        const long long thi = min((long long)a.T - 1, p / a.hop);
        float y = 0.f, wss = 0.f;
        for (long long t = tlo; t <= thi; ++t) {
            const int o = (int)(p - t * a.hop);
            y += a.frames[(u * a.T + t) * (long long)N + o];
            const float w = a.window[o];
            wss += w * w;
        }
        if (wss > 1.17549435e-38f) y /= wss;
        a.sig[i] = y;
    }
}

}  // namespace

int launch_istft(const IstftArgs& a, hipStream_t s) {
    if (a.n_utt <= 0 || a.T <= 0) return 0;
    if (a.N == 640 && a.hop == 160 && a.tri && a.bins) {
        if (a.T < 2) return 0;
        const int n_chunks = (a.T - 1 + OF - 1) / OF;
        const long long items = (long long)n_chunks * a.n_utt;
        if (items > INT32_MAX) {
            set_error("istft batch too large");
            return 3;   // AVSE_ERR_UNSUPPORTED
        }
        int dev = 0, cus = 256;
        AVSE_HIP_CHECK(hipGetDevice(&dev));
        AVSE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        const int grid = (int)std::min<long long>(items, 2LL * cus);
        hipLaunchKernelGGL(k_istft_fused, dim3(grid), dim3(64 * IWAVES), 0, s, a, n_chunks, (int)items);
        AVSE_HIP_CHECK(hipGetLastError());
        return 0;
    }
    if (a.N == 640) {
        hipLaunchKernelGGL(k_istft640, dim3((a.T + FPG - 1) / FPG, (unsigned)a.n_utt), dim3(64), 0, s, a);
    } else {
        const size_t shm = sizeof(float) * 80 + sizeof(float2) * a.nb;
        hipLaunchKernelGGL(k_istft_dft, dim3(a.T, (unsigned)a.n_utt), dim3(256), shm, s, a);
    }
    AVSE_HIP_CHECK(hipGetLastError());
    if (a.T > 1) {
        const long long total = (long long)a.hop * (a.T - 1) * a.n_utt;
        long long g = (total + 255) / 256;
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(k_ola, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, s, a);
        AVSE_HIP_CHECK(hipGetLastError());
    }
    return 0;
}

}  // namespace avse
