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
// each lane then writes two windowed output samples per frame.  k_istft532 (532 = 2 (267 - 1), the inverse at
// 29.97 / 30 fps) is a 28 x 19 prime-factor DFT; k_istft_dft handles other sizes with a direct inverse DFT.  k_ola sums the <= 4
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
AVSE_DEBUG_RECORD(debug_read_istft)
namespace {

constexpr int FPG = 3;
// frame slot stride in float2: >= 340 (the 20 x 17 layout of the DFT steps); 353 makes 2 ZS = 2 (mod 32) dwords, so
// the step-3 stores of 16 consecutive frames at one bin (ds_write_b64 lane groups) hit distinct bank pairs (340: 4-way)
constexpr int ZS = 353;

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

// a D / |D| (1 where D == 0) in packed form
__device__ __forceinline__ v2f pk_unit_phase(v2f d, float a) {
    const v2f d2 = d * d;
    const float r2 = d2.x + d2.y;
    const float s = a * __builtin_amdgcn_rsqf(r2);
    return r2 > 0.f ? d * v2f(s) : v2f{a, 0.f};
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
//   2. y = (M M^T)^{-1} amp for all 24 frames as one fp32 MFMA product with the host-inverted Gram matrix
//      (round 2: a Thomas recurrence, one lane per frame)
//   3. X[k] = M[j0][k] y[j0] + M[j0+1][k] y[j0+1] (pinv(M) amp = M^T y), times the mixture's unit phase,
//      read bin-major / frame-minor (24-frame runs of the [bin][frame] STFT); folded into the 320-point
//      complex sequence Z' of the real inverse FFT, both halves (k, 320 - k) by one lane
//   4. the in-register 20 x 16 DFTs of K1 (3 frames per wave) -> windowed time samples in the frame's slot
//   5. overlap-add in increasing frame order x 1 / window sum-square (a per-position table in the interior)
//      -> the trimmed signal, coalesced; first, the next chunk's global loads are issued (software pipeline)
#ifndef AVSE_ISTFT_OF                         // A/B builds (tools/stft_time.py variant libraries)
#define AVSE_ISTFT_OF 30
#endif
#ifndef AVSE_ISTFT_ATTR
#define AVSE_ISTFT_ATTR __attribute__((amdgpu_waves_per_eu(3)))   // 11 waves: 3 per SIMD, <= 168 VGPRs
#endif
#ifndef AVSE_ISTFT_BPC
#define AVSE_ISTFT_BPC 1
#endif
constexpr int OF = AVSE_ISTFT_OF;            // output hops per chunk
constexpr int FW = OF + 3;                   // frames per chunk (n_fft / hop - 1 = 3 extra)
static_assert(FW % FPG == 0, "whole waves of 3 frames");
constexpr int IWAVES = FW / FPG;             // 8
constexpr int NMEL = 80;                     // bands (host-checked: the fused kernel runs only for n_mels == 80)

__device__ __forceinline__ void ibarrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// AVSE_ISTFT_STAMP (diagnostic variant builds only, never the library): thread 0 of each block adds the s_memtime
// cycles of every phase of every item into g_ist_stamps[block][phase]; avse_istft_stamps() copies them out
#ifdef AVSE_ISTFT_STAMP
__device__ unsigned long long g_ist_stamps[1024][9];
#define IST_STAMP_INIT unsigned long long ist_t0 = __builtin_amdgcn_s_memtime();
#define IST_STAMP(i)                                                                 \
    if (threadIdx.x == 0) {                                                          \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                  \
        g_ist_stamps[blockIdx.x & 1023][i] += t1 - ist_t0;                           \
        ist_t0 = t1;                                                                 \
    }
#else
#define IST_STAMP_INIT
#define IST_STAMP(i)
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ist_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > 0x7fffff00 ? 0x7fffff00 : (int)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}

__global__ __launch_bounds__(64 * IWAVES) AVSE_ISTFT_ATTR void k_istft_fused(IstftArgs a, int n_chunks, int n_items) {
    __shared__ float2 zbuf[FW * ZS];            // frame f's slot: zbuf + f * ZS (Z', then 640 time samples)
    // amplitudes, then y in place; odd row pitch (81 floats): the MFMA fragment reads (16 consecutive frames at one
    // band) are conflict-free and step 3's frame-pair lanes 2-way (a pitch of 80 put them on 2 banks)
    __shared__ float amp[FW][81];
    __shared__ float yb[FW][81];                // y = (M M^T)^{-1} amp (step 2), read by step 3
    __shared__ float win_l[640];
    __shared__ float ws_l[640];                 // window / 320: applied as the DFT's samples are stored
    __shared__ float iwss_l[160];               // 1 / window sum-square of an interior sample, by position mod 160
    __shared__ float ginv_l[NMEL * NMEL];       // (M M^T)^{-1} for the MFMA solve of step 2
    __shared__ float2 tw[640];                  // W640^k
    __shared__ float4 bins_l[321];              // per bin: the two pinv weights and the first mel band
    const int T = a.T, n_mels = a.n_mels;
    const long long Lout = (long long)a.hop * (T - 1);

    // tables -> LDS once per (persistent) block: the DFT twiddles and bin weights were global-memory reads in
    // every item's dependency chain
    for (int i = threadIdx.x; i < 640; i += 64 * IWAVES) {
        win_l[i] = a.window[i];
        ws_l[i] = a.window[i] * (1.0f / 320.0f);
        tw[i] = a.twiddle[i];
    }
    for (int i = threadIdx.x; i < 321; i += 64 * IWAVES) bins_l[i] = a.bins[i];
    for (int i = threadIdx.x; i < NMEL * NMEL; i += 64 * IWAVES) ginv_l[i] = a.gram_inv[i];
    for (int i = threadIdx.x; i < 160; i += 64 * IWAVES) {   // the four overlapping frames, increasing t
        float wss = 0.f;
#pragma unroll
        for (int q = 3; q >= 0; --q) {
            const float w = a.window[i + 160 * q];
            wss += w * w;
        }
        iwss_l[i] = 1.0f / wss;
    }
    __syncthreads();

    // the global loads of an item (mel-dB for step 1, the mixture STFT for step 3) are issued by the previous item's
    // step 5, before its output stores: vmcnt retires in order, so loads issued at the top of an item waited for the
    // previous item's stores too (step 1 measured 12.4K cycles of a 47K-cycle item, tools/istft_stamps.py)
    constexpr int IT1 = (FW * 80 + 64 * IWAVES - 1) / (64 * IWAVES);   // 4 (n_mels == 80, host-checked)
    // step 3 works on (bin k, frame pair): the pair's two STFT values are one 16-B load (the [bin][frame] layout keeps
    // a bin's frames adjacent); 8-B loads of single frames issued ~4.4K cycles per item (tools/istft_stamps.py)
    constexpr int FP = (FW + 1) / 2;                                    // frame pairs per chunk (odd FW: the last
                                                                        // pair's second frame is skipped)
    constexpr int IT3 = (161 * FP + 64 * IWAVES - 1) / (64 * IWAVES);  // 4
    float mv[IT1];
    float4 dk[IT3], dm[IT3];
    // per-utterance buffer resources and 32-bit offsets (the 64-bit pointer math of 20 loads per lane was most of
    // the issuing step's VALU work)
    const float inv_spf = a.spf > 0 ? 1.0f / (float)a.spf : 0.f;
    // part < 0: the mel-dB loads; part j >= 0: the STFT frame pairs of iteration j (spread over step 4's sub-steps so
    // the texture unit streams them while the DFTs compute: issued as one burst they took ~3.2K cycles of issue)
    auto issue_loads = [&](int item, int part) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int u = item / n_chunks, b = item - u * n_chunks;
        const int t_lo = max(0, b * OF - 1);
        const int nfr = min(T - 1, b * OF + OF + 1) - t_lo + 1;
        if (part < 0) {
            const long long mel_u = a.spf > 0 ? (long long)a.n_slices * n_mels * a.spf : (long long)n_mels * T;
            const __amdgpu_buffer_rsrc_t rsM = ist_rsrc(a.mel_db + u * mel_u, mel_u * 4);
#pragma unroll
            for (int j = 0; j < IT1; ++j) {
                const int it = min(tid + 64 * IWAVES * j, FW * n_mels - 1);
                const int m = it / FW, f = it - FW * m;
                const int t = t_lo + min(f, nfr - 1);
                int e;
                if (a.spf > 0) {   // t / spf by a float reciprocal and one correction (t < 2^24)
                    int sl = (int)((float)t * inv_spf);
                    sl -= sl * a.spf > t;
                    sl += (sl + 1) * a.spf <= t;
                    e = (sl * n_mels + m) * a.spf + (t - sl * a.spf);
                } else {
                    e = m * T + t;
                }
                mv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsM, e * 4, 0, 0));
            }
            return;
        }
        const long long stft_u = (long long)a.nb * a.stft_frames;
        const __amdgpu_buffer_rsrc_t rsD = ist_rsrc(a.stft + u * stft_u, stft_u * 8);
#pragma unroll
        for (int j = 0; j < IT3; ++j) {
            if (j != part) continue;
            const int it = tid + 64 * IWAVES * j;
            const int k = it / FP, f = 2 * (it - FP * k);
            if (k <= 160 && f < nfr) {   // the pair's second frame may lie past the chunk / utterance: not used
                const int ok = (k * a.stft_frames + t_lo + f) * 8;
                const int om = ((k == 0 ? 320 : 320 - k) * a.stft_frames + t_lo + f) * 8;
                dk[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsD, ok, 0, 0));
                dm[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsD, om, 0, 0));
            }
        }
    };
    auto issue_all = [&](int item) {
        issue_loads(item, -1);
#pragma unroll
        for (int j = 0; j < IT3; ++j) issue_loads(item, j);
    };
    if (blockIdx.x < n_items) issue_all(blockIdx.x);

    for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
        IST_STAMP_INIT
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));           // keep index math inside the loop (see k_spec640)
        const int lane = tid & 63, wave = tid >> 6;
        const int u = item / n_chunks, b = item - u * n_chunks;
        const int t_lo = max(0, b * OF - 1);
        const int t_hi = min(T - 1, b * OF + OF + 1);
        const int nfr = t_hi - t_lo + 1;
        if (kDebugBuild && tid == 0) {   // checked build: the chunk's frame window fits the block's frame slots
            AVSE_CHECK_DEV(t_lo >= 0 && t_hi < T && nfr >= 1 && nfr <= FW, DK_ISTFT, 1, nfr, FW);
            AVSE_CHECK_DEV(u < a.n_utt, DK_ISTFT, 2, u, (int)a.n_utt);
        }

        // ---- 1. amplitudes (frame fastest: runs of consecutive frames of one band) ----
        {
#pragma unroll
            for (int j = 0; j < IT1; ++j) {
                const int it = tid + 64 * IWAVES * j;
                const int m = it / FW, f = it - FW * m;
                // db_to_amplitude: 10^(dB / 20) = 2^(dB log2(10) / 20) by the hardware v_exp_f32 (1 ulp; the
                // exp10f + sqrtf sequence was ~40 instructions): relative error ~|dB| 2^-24 log2(10) / 20 <= 1e-6
                if (it < FW * n_mels && f < nfr) amp[f][m] = __builtin_amdgcn_exp2f(0.16609640474436813f * mv[j]);
            }
        }
        ibarrier();
        IST_STAMP(0)
        // ---- 2. y = (M M^T)^{-1} amp for the chunk's frames ----
        // MFMA form: Y [48 frames (FW used) x 80] = A [48 x 80] x G [80 x 80], G = (M M^T)^{-1} (host, double ->
        // float): v_mfma_f32_16x16x4_f32 (exact fp32 products) over 3 x 5 output tiles of 16 frames x 16 bands, unit
        // u = wave + IWAVES i (band tile u % 5, frame tile u / 5).  y has its own rows (yb), so each K-step's A and B
        // fragments are read right before its MFMA (no pre-read into ~60 registers and no barrier between).  The
        // Thomas chain it replaces (one lane per frame, 159 dependent steps) took 8.5K of a 34K-cycle item.
        {
            constexpr int NFT = (FW + 15) / 16, NU = NFT * (NMEL / 16);
            const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
            for (int i = 0; i < (NU + IWAVES - 1) / IWAVES; ++i) {
                const int un = wave + IWAVES * i;
                if (un >= NU) break;
                const int bt = un % (NMEL / 16), ft = un / (NMEL / 16);
                if (16 * ft >= nfr) continue;
                const int f = 16 * ft + r16;
                const float* ap = amp[min(f, FW - 1)] + kq;
                const float* gp = ginv_l + kq * NMEL + 16 * bt + r16;
                const bool va = f < nfr;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int st = 0; st < NMEL / 4; ++st)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va ? ap[4 * st] : 0.f, gp[4 * st * NMEL], acc, 0, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int fo = 16 * ft + 4 * kq + e;
                    if (fo < nfr) yb[fo][16 * bt + r16] = acc[e];
                }
            }
        }
        ibarrier();
        IST_STAMP(1)
        // ---- 3. spectrum x unit phase, folded into Z' = conj(E + i O) (k) and E - i O (320 - k) ----
        // (the mixture-STFT loads dk / dm were issued at the start of the item)
        {
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = tid + 64 * IWAVES * j;
                const int k = it / FP, f0 = 2 * (it - FP * k);
                if (k > 160 || f0 >= nfr) continue;
                const int km = k == 0 ? 320 : 320 - k;
                const float4 bk = bins_l[k], bm = bins_l[km];
                const int jk = __float_as_int(bk.z), jm = __float_as_int(bm.z);
                // packed fp32 (fft_common.h): cw = conj(W640^k) / 2, so O = (xk - conj xm) cw and E = (xk + conj xm) / 2
                const float2 twk = tw[k];
                const v2f cw = v2f{0.5f * twk.x, -0.5f * twk.y};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int f = f0 + h;
                    if (h == 1 && f >= nfr) break;
                    const float* y = yb[f];
                    const float ak = (jk >= 0 ? bk.x * y[jk] : 0.f) + (jk + 1 < n_mels && jk >= 0 ? bk.y * y[jk + 1] : 0.f);
                    const float am = (jm >= 0 ? bm.x * y[jm] : 0.f) + (jm + 1 < n_mels && jm >= 0 ? bm.y * y[jm + 1] : 0.f);
                    const v2f dkh = h ? v2f{dk[j].z, dk[j].w} : v2f{dk[j].x, dk[j].y};
                    const v2f dmh = h ? v2f{dm[j].z, dm[j].w} : v2f{dm[j].x, dm[j].y};
                    v2f xk = pk_unit_phase(dkh, ak), xm = pk_unit_phase(dmh, am);
                    if (k == 0) { xk.y = 0.f; xm.y = 0.f; }       // irfft ignores the DC / Nyquist imaginary parts
                    const v2f E = v2f(0.5f) * pk_add_conj(xk, xm);
                    const v2f O = pk_cmul_t(pk_sub_conj(xk, xm), cw);
                    v2f* zf = reinterpret_cast<v2f*>(zbuf + f * ZS);
                    const v2f Zp = pk_sub_mi(E, O);                            // E + i O
                    zf[k] = v2f{Zp.x, -Zp.y};                                  // conj(E + i O)
                    if (k != 0 && k != 160) zf[320 - k] = pk_add_mi(E, O);     // E - i O
                }
            }
        }
        ibarrier();
        IST_STAMP(2)
        const bool more = item + (int)gridDim.x < n_items;   // the next item's loads, spread over step 4
        if (more) { issue_loads(item + gridDim.x, -1); issue_loads(item + gridDim.x, 0); }
        asm volatile("" ::: "memory");
        // ---- 4. forward 320-point DFT of Z' per frame (wave = 3 frames) -> windowed samples ----
        {
            const int f = FPG * wave + (lane >> 4), n1 = lane & 15;
            const bool act = (lane >> 4) < FPG && f < nfr;
            v2f v[20];   // packed-fp32 DFT (fft_common.h pk_*)
            if (act) {
                const v2f* zv = reinterpret_cast<const v2f*>(zbuf) + f * ZS + n1;
#pragma unroll
                for (int n2 = 0; n2 < 20; ++n2) v[n2] = zv[16 * n2];
            }
            ibarrier();
            IST_STAMP(3)
            if (more) issue_loads(item + gridDim.x, 1);
            if (act) {
                pk_dft20(v);
                v2f* zf = reinterpret_cast<v2f*>(zbuf) + f * ZS;
                const v2f* twv = reinterpret_cast<const v2f*>(tw);
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 5; ++d) {
                        const int k2 = c + 4 * d;
                        v2f yv = v[5 * c + d];
                        if (k2) yv = pk_cmul_t(yv, twv[2 * n1 * k2]);   // W320^{n1 k2}, 2 n1 k2 <= 570
                        zf[k2 * 17 + n1] = yv;
                    }
            }
        }
        ibarrier();
        IST_STAMP(4)
        if (more) issue_loads(item + gridDim.x, 2);
        {
            const int f = FPG * wave + lane / 20, k2 = lane - 20 * (lane / 20);
            const bool act = lane < 20 * FPG && f < nfr;
            v2f v[16];
            float2* zf = zbuf + min(f, FW - 1) * ZS;
            if (act) {
                const v2f* zv = reinterpret_cast<const v2f*>(zf) + k2 * 17;
#pragma unroll
                for (int n1 = 0; n1 < 16; ++n1) v[n1] = zv[n1];
            }
            ibarrier();
            IST_STAMP(5)
            if (more) issue_loads(item + gridDim.x, 3);
            if (act) {
                pk_dft16(v);
                float* fr = reinterpret_cast<float*>(zf);
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const int n = k2 + 20 * (c + 4 * d);       // z[n] = conj(out[n]) / 320, then windowed
                        const v2f o = v[4 * c + d];
                        const v2f w = *reinterpret_cast<const v2f*>(ws_l + 2 * n);
                        *reinterpret_cast<v2f*>(fr + 2 * n) = o * v2f{w.x, -w.y};
                    }
            }
        }
        ibarrier();
        IST_STAMP(6)
        // ---- 5. overlap-add + window-sum-square + centre trim (first: the next item's loads) ----
        {
            const long long i0 = (long long)b * OF * 160;
            const int n_out = (int)min((long long)OF * 160, Lout - i0);
            float* __restrict__ out = a.sig + (long long)u * Lout + i0;
#pragma unroll 1
            for (int j = tid; j < n_out; j += 64 * IWAVES) {
                const int p = (int)(i0 + j) + 320;                 // position in the untrimmed signal
                const int hq = p / 160, o0 = p - 160 * hq;
                float yv = 0.f;
                if (hq >= 3 && hq <= T - 1) {                      // interior: four frames, constant sum-square
#pragma unroll
                    for (int q = 0; q < 4; ++q) {                  // increasing t = hq - 3 + q
                        AVSE_CHECK_DEV(hq - 3 + q - t_lo >= 0 && hq - 3 + q - t_lo < nfr, DK_ISTFT, 3,
                                       hq - 3 + q - t_lo, nfr);
                        yv += reinterpret_cast<const float*>(zbuf + (hq - 3 + q - t_lo) * ZS)[o0 + 160 * (3 - q)];
                    }
                    yv *= iwss_l[o0];
                } else {                                           // the utterance's first / last hops
                    const int tlo = max(0, (p - 640 + 160) / 160); // first frame t with t*160 + 639 >= p
                    const int thi = min(T - 1, hq);
                    float wss = 0.f;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int t = thi - 3 + q;
                        if (t < tlo) continue;
                        const int o = p - 160 * t;
                        const float w = win_l[o];
                        yv += reinterpret_cast<const float*>(zbuf + (t - t_lo) * ZS)[o];
                        wss += w * w;
                    }
                    if (wss > 1.17549435e-38f) yv /= wss;
                }
                out[j] = yv;
            }
        }
        ibarrier();
        IST_STAMP(7)
    }
}

// ------------------------------------------------------------------------------------------------------------
// k_istft532: the inverse for n_fft 533's 267 bins (N = 2 (267 - 1) = 532 = 28 x 19, librosa.istft's n_fft at 29.97 /
// 30 fps) by the Good-Thomas prime-factor algorithm over the Hermitian-complete spectrum Xf:
//   input map  k = (19 k1 + 28 k2) mod 532,  output map  n = (57 n1 + 476 n2) mod 532
//   (57 = 19 (19^-1 mod 28), 476 = 28 (28^-1 mod 19)), so that e^{+2 pi i k n / 532} = V28^{k1 n1} V19^{k2 n2}:
//   stage A: item (frame, k1 in 0..14): Z[k1][n2] = sum_k2 Xf V19^{k2 n2}, folded over k2 <-> 19 - k2, n2 <-> 19 - n2
//            (Z[28 - k1][n2] = conj Z[k1][n2] by Hermitian symmetry, so k1 = 15..27 are not computed);
//   stage B: item (frame, n2): x[n1, n2] = Re sum_k1 Z[k1][n2] V28^{k1 n1}, folded over k1 <-> 28 - k1 and
//            n1 <-> 28 - n1; x / 532 times the window goes to the frame scratch for k_ola (as k_istft_dft's output).
// Before the stages: amplitudes from the mel dB, the pinv(mel) projection to 267 bins for a chunk of frames per
// thread (the pinv rows read once per block, coalesced) and the mixture's unit phase.  One 256-thread block per
// (utterance, chunk of 16 frames); ~20K pinv + ~11K DFT multiply-adds per frame against the direct inverse's ~300K.
constexpr int I532_CH = 16;
constexpr int I532_THREADS = 256;
constexpr int I532_XS = 272;                           // float2 bin row pitch
constexpr int I532_LDS = 4 * I532_CH * 80 + 8 * I532_CH * I532_XS + 8 * I532_CH * 15 * 19;

__device__ constexpr float kCos19[19] = {
    1.000000000e+00f, 9.458172321e-01f, 7.891405225e-01f, 5.469481349e-01f, 2.454854846e-01f, -8.257934451e-02f,
    -4.016954303e-01f, -6.772815585e-01f, -8.794737458e-01f, -9.863613248e-01f, -9.863613248e-01f, -8.794737458e-01f,
    -6.772815585e-01f, -4.016954303e-01f, -8.257934451e-02f, 2.454854846e-01f, 5.469481349e-01f, 7.891405225e-01f,
    9.458172321e-01f};
__device__ constexpr float kSin19[19] = {
    0.000000000e+00f, 3.246994615e-01f, 6.142126918e-01f, 8.371664882e-01f, 9.694002867e-01f, 9.965844750e-01f,
    9.157733321e-01f, 7.357239127e-01f, 4.759473801e-01f, 1.645945907e-01f, -1.645945907e-01f, -4.759473801e-01f,
    -7.357239127e-01f, -9.157733321e-01f, -9.965844750e-01f, -9.694002867e-01f, -8.371664882e-01f, -6.142126918e-01f,
    -3.246994615e-01f};
__device__ constexpr float kCos28[28] = {
    1.000000000e+00f, 9.749279022e-01f, 9.009688497e-01f, 7.818315029e-01f, 6.234897971e-01f, 4.338837266e-01f,
    2.225209326e-01f, 0.0f, -2.225209326e-01f, -4.338837266e-01f, -6.234897971e-01f, -7.818315029e-01f,
    -9.009688497e-01f, -9.749279022e-01f, -1.000000000e+00f, -9.749279022e-01f, -9.009688497e-01f, -7.818315029e-01f,
    -6.234897971e-01f, -4.338837266e-01f, -2.225209326e-01f, 0.0f, 2.225209326e-01f, 4.338837266e-01f,
    6.234897971e-01f, 7.818315029e-01f, 9.009688497e-01f, 9.749279022e-01f};
__device__ constexpr float kSin28[28] = {
    0.000000000e+00f, 2.225209326e-01f, 4.338837266e-01f, 6.234897971e-01f, 7.818315029e-01f, 9.009688497e-01f,
    9.749279022e-01f, 1.000000000e+00f, 9.749279022e-01f, 9.009688497e-01f, 7.818315029e-01f, 6.234897971e-01f,
    4.338837266e-01f, 2.225209326e-01f, 0.0f, -2.225209326e-01f, -4.338837266e-01f, -6.234897971e-01f,
    -7.818315029e-01f, -9.009688497e-01f, -9.749279022e-01f, -1.000000000e+00f, -9.749279022e-01f, -9.009688497e-01f,
    -7.818315029e-01f, -6.234897971e-01f, -4.338837266e-01f, -2.225209326e-01f};

__global__ __launch_bounds__(I532_THREADS) void k_istft532(IstftArgs a, int n_chunks) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const amp = sm;                                                         // [CH][80]
    float2* const Xs = reinterpret_cast<float2*>(sm + I532_CH * 80);                // [CH][XS] bins 0..266
    float2* const Z = Xs + I532_CH * I532_XS;                                       // [CH][15][19]
    float* const fo = reinterpret_cast<float*>(Xs);                                 // [CH][532] (stage B: aliases Xs)
    const int tid = threadIdx.x;
    const long long u = blockIdx.x / n_chunks;
    const int t0 = (int)(blockIdx.x - u * n_chunks) * I532_CH;
    const int nt = min(I532_CH, a.T - t0);

    for (int it = tid; it < nt * a.n_mels; it += I532_THREADS) {
        const int f = it / a.n_mels, m = it - f * a.n_mels;
        amp[f * 80 + m] = sqrtf(exp10f(0.1f * mel_at(a, u, m, t0 + f)));
    }
    __syncthreads();
    // bins: thread k, all frames of the chunk (pinv row element read once per block)
    for (int k = tid; k < 267; k += I532_THREADS) {
        float acc[I532_CH];
#pragma unroll
        for (int f = 0; f < I532_CH; ++f) acc[f] = 0.f;
        for (int m = 0; m < a.n_mels; ++m) {
            const float p = a.pinvT[m * 267 + k];
#pragma unroll
            for (int f = 0; f < I532_CH; ++f) acc[f] = fmaf(p, amp[f * 80 + m], acc[f]);
        }
        const float2* d = a.stft + (u * 267 + k) * (long long)a.stft_frames + t0;
#pragma unroll
        for (int f = 0; f < I532_CH; ++f) {
            if (f >= nt) break;
            const float2 ph = unit_phase(d[f]);
            float2 x = make_float2(acc[f] * ph.x, acc[f] * ph.y);
            if (k == 0 || k == 266) x.y = 0.f;   // irfft ignores the DC / Nyquist imaginary parts
            Xs[f * I532_XS + k] = x;
        }
    }
    __syncthreads();
    // stage A: item (f, k1 in 0..14)
    if (tid < nt * 15) {
        const int f = tid / 15, k1 = tid - 15 * f;
        const float2* xr = Xs + f * I532_XS;
        float2 y[19];
#pragma unroll
        for (int k2 = 0; k2 < 19; ++k2) {
            int k = 19 * k1 + 28 * k2;
            k = k >= 532 ? k - 532 : k;
            k = k >= 532 ? k - 532 : k;
            const float2 v = xr[k <= 266 ? k : 532 - k];
            y[k2] = k <= 266 ? v : make_float2(v.x, -v.y);
        }
        float pr[10], pi[10], mr[10], mi[10];
        float z0r = y[0].x, z0i = y[0].y;
#pragma unroll
        for (int k2 = 1; k2 <= 9; ++k2) {
            pr[k2] = y[k2].x + y[19 - k2].x;
            pi[k2] = y[k2].y + y[19 - k2].y;
            mr[k2] = y[k2].x - y[19 - k2].x;
            mi[k2] = y[k2].y - y[19 - k2].y;
            z0r += pr[k2];
            z0i += pi[k2];
        }
        float2* zo = Z + (f * 15 + k1) * 19;
        zo[0] = make_float2(z0r, z0i);
#pragma unroll
        for (int n2 = 1; n2 <= 9; ++n2) {
            // V = c + i s: Y V + Y' conj V = (Pr c - Mi s) + i (Pi c + Mr s); n2 -> 19 - n2 flips s
            float A = y[0].x, B = 0.f, C = y[0].y, D = 0.f;
#pragma unroll
            for (int k2 = 1; k2 <= 9; ++k2) {
                const float c = kCos19[(k2 * n2) % 19], s = kSin19[(k2 * n2) % 19];
                A = fmaf(pr[k2], c, A);
                B = fmaf(mi[k2], s, B);
                C = fmaf(pi[k2], c, C);
                D = fmaf(mr[k2], s, D);
            }
            zo[n2] = make_float2(A - B, C + D);
            zo[19 - n2] = make_float2(A + B, C - D);
        }
    }
    __syncthreads();
    // stage B: item (f, n2); Z[28 - k1][n2] = conj Z[k1][n2] (Hermitian Xf), so the pair k1, 28 - k1 adds
    // 2 Re(Z[k1][n2] V28^{k1 n1}); k1 = 0 and 14 are their own partners (real: V28^{14 n1} = (-1)^n1)
    const float scale = 1.f / 532.f;
    for (int it = tid; it < nt * 19; it += I532_THREADS) {
        const int f = it / 19, n2 = it - 19 * f;
        const float2* zf = Z + f * 15 * 19;
        float sr[15], si[15];
        const float z0 = zf[n2].x;
        const float2 z14 = zf[14 * 19 + n2];
#pragma unroll
        for (int k1 = 1; k1 <= 13; ++k1) {
            const float2 p = zf[k1 * 19 + n2];
            sr[k1] = 2.f * p.x;
            si[k1] = 2.f * p.y;
        }
        float xo[28];
#pragma unroll
        for (int n1 = 0; n1 <= 14; ++n1) {
            float E = z0 + ((n1 & 1) ? -z14.x : z14.x), O = 0.f;
#pragma unroll
            for (int k1 = 1; k1 <= 13; ++k1) {
                E = fmaf(sr[k1], kCos28[(k1 * n1) % 28], E);
                O = fmaf(si[k1], kSin28[(k1 * n1) % 28], O);
            }
            xo[n1] = E - O;
            if (n1 >= 1 && n1 <= 13) xo[28 - n1] = E + O;
        }
        float* fr = fo + f * 532;
#pragma unroll
        for (int n1 = 0; n1 < 28; ++n1) {
            int n = 57 * n1 + 476 * n2;
            n %= 532;
            fr[n] = xo[n1] * scale;
        }
    }
    __syncthreads();
    // windowed frames to the scratch for k_ola
    for (int it = tid; it < nt * 532; it += I532_THREADS) {
        const int f = it / 532, n = it - 532 * f;
        a.frames[((u * a.T) + t0 + f) * 532LL + n] = fo[f * 532 + n] * a.window[n];
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

#ifdef AVSE_ISTFT_STAMP
extern "C" int avse_istft_stamps(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ist_stamps), sizeof(unsigned long long) * 1024 * 9) != hipSuccess) return 2;
    if (reset) {
        static unsigned long long zero[1024 * 9];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ist_stamps), zero, sizeof(zero)) != hipSuccess) return 2;
    }
    return 0;
}
#endif

int launch_istft(const IstftArgs& a, hipStream_t s) {
    if (a.n_utt <= 0 || a.T <= 0) return 0;
    // fused path: 32-bit offsets into one utterance's STFT (nb x frames x 8 B < 2 GiB: ~2 hours at 16 kHz)
    if (a.N == 640 && a.hop == 160 && a.n_mels == NMEL && a.gram_inv && a.bins &&
        (long long)a.nb * a.stft_frames * 8 < 0x7fffff00LL) {
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
        const int grid = (int)std::min<long long>(items, (long long)AVSE_ISTFT_BPC * cus);
        hipLaunchKernelGGL(k_istft_fused, dim3(grid), dim3(64 * IWAVES), 0, s, a, n_chunks, (int)items);
        AVSE_HIP_CHECK(hipGetLastError());
        return 0;
    }
    if (a.N == 640) {
        hipLaunchKernelGGL(k_istft640, dim3((a.T + FPG - 1) / FPG, (unsigned)a.n_utt), dim3(64), 0, s, a);
    } else if (a.N == 532 && a.nb == 267 && a.n_mels <= 80) {
        const int n_chunks = (a.T + I532_CH - 1) / I532_CH;
        const long long items = (long long)n_chunks * a.n_utt;
        if (items > INT32_MAX) {
            set_error("istft batch too large");
            return 3;   // AVSE_ERR_UNSUPPORTED
        }
        if (int rc = ensure_lds_attr((const void*)k_istft532, I532_LDS)) return rc;
        hipLaunchKernelGGL(k_istft532, dim3((unsigned)items), dim3(I532_THREADS), I532_LDS, s, a, n_chunks);
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
