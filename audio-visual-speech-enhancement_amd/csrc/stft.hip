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
// A 448-lane block handles a chunk of up to 21 frames of one utterance, 3 frames per
// wave (48 / 60 active lanes in steps 1 / 2).  When the chunk covers the whole utterance (the
// 200-ms segment case: 3200 samples -> 21 frames) the top_db clamp (max over the WHOLE
// [80, T] array, including the frame the slicing later drops) happens in-kernel; otherwise each
// chunk publishes its max with an ordered-uint atomicMax and a clamp kernel follows.
//
// n_fft = 533 (29.97 / 30 fps) runs k_spec533 (a Good-Thomas 13 x 41 prime-factor DFT); other n_fft use k_spec_dft,
// a direct DFT, one block per frame.
#include <algorithm>

#include "avse_common.h"
#include "fft_common.h"

#ifdef AVSE_NO_WPE   // A/B: no occupancy cap
#define AVSE_WPE4
#else
#define AVSE_WPE4 __attribute__((amdgpu_waves_per_eu(4)))
#endif

namespace avse {
AVSE_DEBUG_RECORD(debug_read_stft)

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

// One block of 7 waves per work item (utterance, chunk of CHUNK frames); wave w owns frames [3w, 3w + 3).
// Round-1 version: 0.198 ms for 4096 segments (5 % of the HBM roofline).  Changes (0.173 ms):
//  - capped at 128 VGPRs (amdgpu_waves_per_eu(4)) so two ~80-KB blocks share a CU (137 VGPRs allowed one);
//  - interior frames (the whole 640-sample window inside the signal) load 8-B sample pairs without the
//    reflect / zero-pad index arithmetic, which stays on the edge frames only (branch-free);
//  - the mel dot runs over a compile-time 24-bin band (host rows zero-padded, 16-B weight reads);
//  - step 3 maps items bin-major / frame-minor over the whole chunk, so the complex-STFT store (librosa's
//    [bin][frame] layout) writes 21-frame runs instead of 8-B scatters (configs[4] STFT 0.65 -> 0.50 ms).
//  - without the complex-STFT output (the segment / configs[1] case) steps 1-4 touch only the wave's own frames:
//    wave-synchronous LDS hand-offs, one block barrier per item (0.172 -> 0.154 ms), dB via v_log_f32 (0.151 ms).
// Tried: a persistent grid with the next item's samples prefetched into registers during steps 2-4 — the
// loop-invariant address math the compiler hoisted out of the item loop needed 207-256 VGPRs (one block
// per CU): 0.224 ms.  PMC (r02, B = 4096): 1,907 VALU instructions per wave (636 per frame), 48 % of wave
// cycles parked on waitcnt / barrier, 21 % issue-stalled.
constexpr int WAVES = CHUNK / FPG;     // 7
constexpr int MW = 24;                 // padded Slaney band width of the LDS table (host-checked)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// wave-synchronous LDS hand-off: a wave's LDS operations complete in issue order, so draining lgkmcnt (and keeping the
// compiler from moving memory operations across) is enough when every lane that wrote belongs to the reading wave
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// index of sample i after centre padding: reflect (librosa's 2017 default) or zero (then `keep` is false)
__device__ __forceinline__ int padded_index(int i, int L, int pad_mode, bool& keep) {
    keep = pad_mode == 0 || (i >= 0 && i < L);
    if (pad_mode == 0) {
        const int j = abs(i);
        return min(j, 2 * (L - 1) - j);
    }
    return min(max(i, 0), L - 1);
}

// |X| by the hardware v_sqrt_f32 (1 ulp; sqrtf's correctly rounded sequence is ~12 instructions, 16 per lane per
// chunk, and the magnitudes only feed the mel sums, dB tolerance 1e-3) of the packed square
__device__ __forceinline__ float pk_abs(v2f x) {
    const v2f x2 = x * x;
    return __builtin_amdgcn_sqrtf(x2.x + x2.y);
}

// Slaney band dot of NQ weight quads against the band's magnitudes (k_spec_seg step 4, k_spec640): loads first,
// then the FMAs (same summation order as the quad loop it replaced)
template <int NQ>
__device__ __forceinline__ float band_dot(const float4* wm, const v2f* mf) {
    float4 w[NQ];
    v2f x[2 * NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        w[q] = wm[q];
        x[2 * q] = mf[2 * q];
        x[2 * q + 1] = mf[2 * q + 1];
    }
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        acc = fmaf(x[2 * q].x, w[q].x, acc);
        acc = fmaf(x[2 * q].y, w[q].y, acc);
        acc = fmaf(x[2 * q + 1].x, w[q].z, acc);
        acc = fmaf(x[2 * q + 1].y, w[q].w, acc);
    }
    return acc;
}
// the same over 16-B magnitude quads from a 4-aligned band start (k_spec_seg): ds_read_b128 for weights and magnitudes
template <int NQ>
__device__ __forceinline__ float band_dot4(const float4* wm, const float4* mf) {
    float4 w[NQ], x[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        w[q] = wm[q];
        x[q] = mf[q];
    }
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        acc = fmaf(x[q].x, w[q].x, acc);
        acc = fmaf(x[q].y, w[q].y, acc);
        acc = fmaf(x[q].z, w[q].z, acc);
        acc = fmaf(x[q].w, w[q].w, acc);
    }
    return acc;
}

// real-FFT untangling of the packed 320-point transform Z of one frame (z[n] = x[2n] + i x[2n+1]):
// packed form: X = X[k], Y = conj X[320 - k] from Z[k], Z[320 - k]; U = -i W640^k / 2 (a float2 table):
// E = (Zk + conj Zm) / 2, W^k O = U (Zk - conj Zm), X = E + W^k O, Y = E - W^k O
__device__ __forceinline__ void pk_untangle(const v2f* __restrict__ zf, int k, const v2f* __restrict__ ut, v2f& X, v2f& Y) {
    const v2f zk = zf[k], zm = zf[k == 0 ? 0 : 320 - k];
    const v2f S = pk_add_conj(zk, zm);
    const v2f WO = pk_cmul_t(pk_sub_conj(zk, zm), ut[k]);
    X = __builtin_elementwise_fma(v2f(0.5f), S, WO);
    Y = __builtin_elementwise_fma(v2f(0.5f), S, -WO);
}

// lane (f1, n1) of step 1 loads z[n1 + 16 n2] = (x[s0 + 2(n1 + 16 n2)], x[s0 + 2(n1 + 16 n2) + 1]), n2 < 20
__device__ __forceinline__ void load_frame(float2 (&x)[20], const float* __restrict__ s, int L, int s0, int n1,
                                           int pad_mode) {
    if (s0 >= 0 && s0 + 640 <= L) {
        const float2* p = reinterpret_cast<const float2*>(s + s0) + n1;
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) x[n2] = p[16 * n2];
    } else {   // edge frame: branch-free per-sample index arithmetic
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) {
            const int i = s0 + 2 * (n1 + 16 * n2);
            bool k0, k1;
            const int j0 = padded_index(i, L, pad_mode, k0), j1 = padded_index(i + 1, L, pad_mode, k1);
            const float v0 = s[j0], v1 = s[j1];
            x[n2] = make_float2(k0 ? v0 : 0.f, k1 ? v1 : 0.f);
        }
    }
}

// RI: the complex STFT is stored too (bin-major over the whole chunk: block barriers between the steps).  Without it
// every step until the top_db maximum touches only the wave's own three frames, so the waves hand off through LDS
// wave-synchronously and one block barrier remains per item.
// AVSE_STFT_STAMP (diagnostic variant builds only, never the library): thread 0 of every block adds the s_memtime
// cycles of each step to its block's slot of g_spec_stamps; avse_spec_stamps() copies them out (tools/stft_stamps.py)
#ifdef AVSE_STFT_STAMP
__device__ unsigned long long g_spec_stamps[4096][8];   // per block slot (blockIdx % 4096): no atomics
#define SPEC_STAMP_INIT unsigned long long spec_t0 = __builtin_amdgcn_s_memtime();
#define SPEC_STAMP(i)                                                                \
    if (threadIdx.x == 0) {                                                          \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                  \
        g_spec_stamps[blockIdx.x & 4095][i] += t1 - spec_t0;                         \
        spec_t0 = t1;                                                                \
    }
#else
#define SPEC_STAMP_INIT
#define SPEC_STAMP(i)
#endif

template <bool FAST_MEL, bool RI>
__global__ __launch_bounds__(64 * WAVES) AVSE_WPE4 void k_spec640(SpecArgs a, int n_chunks) {
    SPEC_STAMP_INIT
    __shared__ float2 zbuf[WAVES * FPG * ZS];
    __shared__ float dbuf[80 * CHUNK];
    __shared__ float2 twl[640];
    __shared__ v2f ut2[161];       // U = -i W640^k / 2 (untangling)
    __shared__ float2 winl[320];
    __shared__ float4 melw4[FAST_MEL ? 80 * MW / 4 : 1];
    __shared__ int mel_st[80], mel_wd[80];
    __shared__ float wmax[1][WAVES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.n_frames;
    const int L = (int)a.n_samples;
    const int n_mels = a.n_mels, mw = a.mel_max_width;
    const int g = FPG * wave;                       // this wave's first frame in the chunk

    for (int i = tid; i < 640; i += 64 * WAVES) twl[i] = a.twiddle[i];
    for (int k = tid; k < 161; k += 64 * WAVES) {
        const float2 w = a.twiddle[k];
        ut2[k] = v2f{0.5f * w.y, -0.5f * w.x};
    }
    for (int i = tid; i < 320; i += 64 * WAVES) winl[i] = reinterpret_cast<const float2*>(a.window)[i];
    if (FAST_MEL)   // host rows are zero-padded to MW
        for (int i = tid; i < n_mels * MW / 4; i += 64 * WAVES) melw4[i] = reinterpret_cast<const float4*>(a.mel_weight)[i];
    for (int i = tid; i < n_mels; i += 64 * WAVES) {
        mel_st[i] = a.mel_start[i];
        mel_wd[i] = a.mel_width[i];
    }

    const int f1 = lane >> 4, n1 = lane & 15;
    const int item = blockIdx.x;
    const int u = item / n_chunks, chunk = item - u * n_chunks;
    float2 x[20];
    {
        const int nf = min(CHUNK, T - chunk * CHUNK);
        if (f1 < min(FPG, nf - g))
            load_frame(x, a.sig + (long long)u * L, L, (chunk * CHUNK + g + f1) * a.hop - 320, n1, a.pad_mode);
    }
    __syncthreads();
    SPEC_STAMP(0)
    {
        const int parity = 0;   // (wmax slot of the item)
        const int t0 = chunk * CHUNK;
        const int nf = min(CHUNK, T - t0);
        const int ng = max(0, min(FPG, nf - g));
        float2* zw = zbuf + wave * FPG * ZS;

        // ---- step 1: 20-point DFTs over n2, lane = (f, n1) (packed fp32, fft_common.h pk_*) ----
        v2f v[20];
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) {
            const float2 w = winl[n1 + 16 * n2];
            v[n2] = v2f{x[n2].x, x[n2].y} * v2f{w.x, w.y};
        }
        if (f1 < ng) {
            pk_dft20(v);
            // v[5c + d] = Y[c + 4d]; twiddle W320^{n1 k2} = W640^{2 n1 k2} (2 n1 k2 <= 570)
            v2f* zf = reinterpret_cast<v2f*>(zw + f1 * ZS);
            const v2f* twv = reinterpret_cast<const v2f*>(twl);
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    const int k2 = c + 4 * d;
                    v2f y = v[5 * c + d];
                    if (k2) y = pk_cmul_t(y, twv[2 * n1 * k2]);
                    zf[k2 * 17 + n1] = y;
                }
        }
        if constexpr (RI) lds_barrier(); else wave_lds_sync();
        SPEC_STAMP(1)
        // ---- step 2: 16-point DFTs over n1, lane = (f, k2) ----
        {
            const int f = lane / 20, k2 = lane - 20 * (lane / 20);
            const bool act = f < ng;
            v2f w[16];
            v2f* zf = reinterpret_cast<v2f*>(zw + min(f, FPG - 1) * ZS);
            if (act) {
#pragma unroll
                for (int n = 0; n < 16; ++n) w[n] = zf[k2 * 17 + n];
            }
            if constexpr (RI) lds_barrier(); else wave_lds_sync();
            SPEC_STAMP(2)
            if (act) {
                pk_dft16(w);
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 4; ++d) zf[k2 + 20 * (c + 4 * d)] = w[4 * c + d];
            }
        }
        SPEC_STAMP(3)
        if constexpr (RI) {
            lds_barrier();
            // ---- step 3: real-FFT untangling + magnitude over the chunk, item = (k, f), f fastest ----
            constexpr int IT3 = (161 * CHUNK + 64 * WAVES - 1) / (64 * WAVES);   // 8
            float mk[IT3], mm[IT3];
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = tid + 64 * WAVES * j;
                const int k = it / CHUNK, f = it - CHUNK * k;
                if (k > 160 || f >= nf) continue;
                const v2f* zf = reinterpret_cast<const v2f*>(zbuf + f * ZS);
                v2f X, Y;
                pk_untangle(zf, k, ut2, X, Y);
                mk[j] = pk_abs(X);
                mm[j] = pk_abs(Y);
                float2* o = reinterpret_cast<float2*>(a.stft_ri) + (long long)u * 321 * T + t0 + f;
                o[(long long)k * T] = make_float2(X.x, X.y);
                if (k != 160) o[(long long)(320 - k) * T] = make_float2(Y.x, -Y.y);   // X[320 - k] = conj(Y)
            }
            lds_barrier();
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = tid + 64 * WAVES * j;
                const int k = it / CHUNK, f = it - CHUNK * k;
                if (k > 160 || f >= nf) continue;
                float* mf = reinterpret_cast<float*>(zbuf + f * ZS);
                mf[k] = mk[j];
                mf[320 - k] = mm[j];
            }
            if (FAST_MEL) {   // bins [321, 321 + MW) are read by the padded band dots: make them zero
                for (int it = tid; it < CHUNK * MW; it += 64 * WAVES) {
                    const int f = it / MW, j = it - MW * f;
                    reinterpret_cast<float*>(zbuf + f * ZS)[321 + j] = 0.f;
                }
            }
            lds_barrier();
        } else {
            wave_lds_sync();
            // ---- step 3: untangling + magnitude of the wave's own frames, item = (f, k) ----
            constexpr int IT3 = (FPG * 161 + 63) / 64;   // 8
            float mk[IT3], mm[IT3];
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = lane + 64 * j;
                if (it >= ng * 161) break;
                const int f = it / 161, k = it - 161 * f;
                v2f X, Y;
                pk_untangle(reinterpret_cast<const v2f*>(zw + f * ZS), k, ut2, X, Y);
                mk[j] = pk_abs(X);
                mm[j] = pk_abs(Y);
            }
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = lane + 64 * j;
                if (it >= ng * 161) break;
                const int f = it / 161, k = it - 161 * f;
                float* mf = reinterpret_cast<float*>(zw + f * ZS);
                mf[k] = mk[j];
                mf[320 - k] = mm[j];
            }
            if (FAST_MEL)
                for (int it = lane; it < FPG * MW; it += 64) {
                    const int f = it / MW, j = it - MW * f;
                    reinterpret_cast<float*>(zw + f * ZS)[321 + j] = 0.f;
                }
            wave_lds_sync();
        }
        SPEC_STAMP(4)
        // ---- step 4: Slaney mel + dB, item = (m, f), f fastest: the three lanes of a band read its weights at one LDS
        // address (broadcast; 0.0983 -> 0.094 ms with the float2 twiddle tables) ----
        float vmax = -INFINITY;
        // items (m, f) band-major, f fastest (as k_spec_seg): pass j covers bands 64 j / 3 .. and reads only the 4-bin
        // weight quads those bands use (MelTable::seg_nq); the frames past a partial last chunk (f >= ng) idle
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int it = lane + 64 * jj;
            if (it >= FPG * n_mels) break;
            const int m = __umul24(it, 43691) >> 17, f = it - 3 * m;   // m = it / 3 (it < 240)
            if (f >= ng) continue;
            const float* mf = reinterpret_cast<const float*>(zw + f * ZS) + mel_st[m];
            float acc = 0.f;
            if (FAST_MEL) {
                const float4* wm = melw4 + m * (MW / 4);
                const v2f* mf2 = reinterpret_cast<const v2f*>(mf);   // even band starts (host)
                switch (a.mel_seg_nq[jj]) {   // straight-line loads per quad count (k_spec_seg step 4)
                    case 1: acc = band_dot<1>(wm, mf2); break;
                    case 2: acc = band_dot<2>(wm, mf2); break;
                    case 3: acc = band_dot<3>(wm, mf2); break;
                    case 4: acc = band_dot<4>(wm, mf2); break;
                    case 5: acc = band_dot<5>(wm, mf2); break;
                    default: acc = band_dot<MW / 4>(wm, mf2); break;
                }
            } else {
                const float* wm = a.mel_weight + m * mw;
                const int wdt = mel_wd[m];
                for (int j = 0; j < wdt; ++j) acc = fmaf(mf[j], wm[j], acc);
            }
            const float db = acc > a.amin ? 6.0205999132796239f * __log2f(acc) : a.db_floor;
            vmax = fmaxf(vmax, db);
            dbuf[m * CHUNK + g + f] = db;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
        if (lane == 0) wmax[parity][wave] = vmax;
        lds_barrier();
        SPEC_STAMP(5)
        vmax = wmax[parity][0];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) vmax = fmaxf(vmax, wmax[parity][w]);
        // ---- clamp / publish ----
        const bool single = (n_chunks == 1);
        const float floor_db = (single && a.top_db >= 0.f) ? vmax - a.top_db : -INFINITY;
        for (int it = tid; it < n_mels * nf; it += 64 * WAVES) {
            const int m = it / nf, tl = it - nf * m;
            const long long oi = out_index(a.spf, a.n_slices, n_mels, T, u, m, t0 + tl);
            AVSE_CHECK_DEV(t0 + tl < T && oi < (a.spf > 0 ? (long long)a.n_utt * a.n_slices * n_mels * a.spf
                                                          : (long long)a.n_utt * n_mels * T),
                           DK_SPEC, 2, t0 + tl, T);
            if (oi >= 0) a.mel_db[oi] = fmaxf(dbuf[m * CHUNK + tl], floor_db);
        }
        if (!single && tid == 0) atomicMax(a.umax + u, f2ord(vmax));
        SPEC_STAMP(6)
    }
}

// The 200-ms segment case (configs[1]: every utterance is exactly one 3200-sample / 21-frame chunk, no complex output,
// padded Slaney rows): a persistent kernel, 2 blocks per CU looping over utterances.
//  - the tables are staged once per block instead of once per utterance (stamps, r03: about a third of k_spec640's
//    block time was that prologue plus the sample-load latency);
//  - a wave's 3 frames span 960 padded samples: the next utterance's span goes straight into the wave's own zbuf region
//    by LDS-DMA (buffer loads with the LDS flag, no VGPRs; reflect padding resolved by the two edge waves) as soon as
//    step 4 has read it, so the load runs under the store pass and the other block's work;
//  - packed-fp32 FFT (fft_common.h pk_*): complex adds are one v_pk_add, products v_pk_mul + v_pk_fma with the
//    quarter turns and the (re, im) swap in the op_sel / neg modifiers, so twiddle tables stay float2 (1,524 -> ~800
//    VALU per wave and utterance, PMC);
//  - one block barrier per utterance (the top_db maximum): every wave keeps its frames' dB values in registers and
//    stores them itself once the maximum is known (no dB buffer, no store pass over the block; a variant that staged
//    them in LDS for float4 stores needed a second barrier per utterance and measured 3 % slower).
// Tried (r03): the mel product on the matrix cores ([21 frames x bins] x [bins x 16-band tiles], v_mfma_f32_16x16x4f32,
// B fragments evaluated from the triangle coefficients, one tile job per wave, a third barrier): 0.0941 vs 0.0928 ms.
// f32 MFMA runs at the f32 VALU rate and the dense tiles carry ~2x the sparse band FMAs; the gain in LDS gathers
// was eaten by the job imbalance (39-42 dependent MFMAs on the longest waves) at the extra barrier.
#ifndef AVSE_SEG_BPC
#define AVSE_SEG_BPC 2
#endif
constexpr int SEG_L = 3200;
// step 4 layout (LDS bank model of MI355X_MICROARCH.md §LDS, one wave's mel reads per utterance): magnitudes of frame f
// at f * SEG_FS floats, bands from a 4-aligned start with weight rows of SEG_MW floats, both read as 16-B quads
// (ds_read_b128): 160 LDS cycles per wave and utterance against 418 for 8-B pairs at 680-float frames / 24-float rows
constexpr int SEG_FS = 360, SEG_MW = MW + 4;
static_assert(2 * SEG_FS + 321 + SEG_MW <= FPG * 2 * ZS && SEG_FS % 4 == 0, "magnitude frames inside the wave region");

__device__ __forceinline__ void seg_dma(float* sb, const float* __restrict__ sg, int wave, int lane, int pad_mode) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sg), (short)0, SEG_L * 4, 0x00020000);
    const int base = FPG * wave * 160 - 320;   // sample index of buffer slot 0
    typedef __attribute__((address_space(3))) void* lds_ptr;
    if (wave != 0 && wave != WAVES - 1) {      // (wave-uniform) interior: base .. base + 1023 inside the utterance
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(sb + 256 * j), 16, (base + 4 * lane) * 4, 1024 * j, 0, 0);
    } else {
        // edge waves: 640 samples inside the utterance as 16-B pieces (3 instructions, the last half used) and the 320
        // padded ones one dword per lane with a reversed index (reflect) or an offset past the range (reads 0)
        const bool first = wave == 0;
        const int cslot = first ? 320 : 0, csmp = first ? 0 : SEG_L - 640;   // contiguous run: slots / samples
        const int rslot = first ? 0 : 640, rbase = first ? 320 : 2 * (SEG_L - 1) - base;   // reflected run
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (j < 2 || lane < 32)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(sb + cslot + 256 * j), 16, (csmp + 4 * lane) * 4,
                                                         1024 * j, 0, 0);
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int sl = rslot + 64 * j + lane;     // slot; reflected sample rbase - slot (reflect padding)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(sb + rslot + 64 * j), 4,
                                                     pad_mode == 0 ? (rbase - sl) * 4 : 0x40000000, 0, 0, 0);
        }
    }
}

__global__ __launch_bounds__(64 * WAVES) AVSE_WPE4 void k_spec_seg(SpecArgs a) {
    SPEC_STAMP_INIT
    __shared__ __attribute__((aligned(16))) v2f zbuf[WAVES * FPG * ZS];
    __shared__ v2f twp[19 * 16];   // W320^(n1 k2) at (k2 - 1) * 16 + n1 (step 1: conflict-free rows per k2)
    __shared__ v2f ut2[161];       // U = -i W640^k / 2 (untangling)
    __shared__ v2f winl[320];
    __shared__ float4 melw4[80 * SEG_MW / 4];
    __shared__ int mel_st[80];     // 4-aligned band starts
    __shared__ float wmax[2][WAVES];   // by utterance parity: a wave at most one utterance ahead writes the other row
    static_assert(FPG * ZS * 2 >= 1024, "the sample buffer lives in the wave's zbuf region");

    int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n_mels = a.n_mels;
    // the first utterance's samples are requested before the tables, so both latencies overlap
    v2f* zw = zbuf + wave * FPG * ZS;
    float* zwf = reinterpret_cast<float*>(zw);
    const long long n_utt = a.n_utt;
    long long u = blockIdx.x;
    if (u < n_utt) seg_dma(zwf, a.sig + u * SEG_L, wave, tid & 63, a.pad_mode);
    for (int i = tid; i < 320; i += 64 * WAVES) {
        if (i < 19 * 16) {
            const float2 w = a.twiddle[2 * (i & 15) * ((i >> 4) + 1)];
            twp[i] = v2f{w.x, w.y};
        }
        winl[i] = reinterpret_cast<const v2f*>(a.window)[i];
    }
    for (int k = tid; k < 161; k += 64 * WAVES) {
        const float2 w = a.twiddle[k];
        ut2[k] = v2f{0.5f * w.y, -0.5f * w.x};
    }
    // weight rows re-based to the 4-aligned start: 0 or 2 leading zeros (host starts are even), zero tail
    for (int i = tid; i < n_mels * SEG_MW; i += 64 * WAVES) {
        const int m = i / SEG_MW, src = i - SEG_MW * m - (a.mel_start[m] & 3);
        reinterpret_cast<float*>(melw4)[i] = src >= 0 && src < MW ? a.mel_weight[m * MW + src] : 0.f;
    }
    for (int i = tid; i < n_mels; i += 64 * WAVES) mel_st[i] = a.mel_start[i] & ~3;

    lds_barrier();   // the tables are complete before any wave's step 1 (the first utterance's samples stay in flight)
    int parity = 0;
    for (; u < n_utt; u += gridDim.x, parity ^= 1) {
        // the per-lane index math stays inside the loop: hoisted out of it, the loop-invariant addresses held more
        // registers than the 128 of two blocks per CU (k_spec640's note)
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63;
        const int f1 = lane >> 4, n1 = lane & 15;
        const long long nx = u + gridDim.x;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's samples have landed (wave-local buffer)
        if (kDebugBuild && lane == 0) {   // checked build: the staged span is this utterance's (slot 320 + 7 wave)
            [[maybe_unused]] const int sidx = 320 + 7 * wave, src = FPG * wave * 160 - 320 + sidx;   // in the utterance
            [[maybe_unused]] const float* zv = reinterpret_cast<const float*>(zw);
            AVSE_CHECK_DEV(zv[sidx] == a.sig[u * SEG_L + src], DK_SPEC, 1, (int)u, src);
        }
        SPEC_STAMP(0)
        // ---- step 1: windowed 20-point DFTs over n2, lane = (f, n1) ----
        v2f v[20];
        {
            const v2f* xs = zw + f1 * 80 + n1;   // padded samples 160 f1 + 2 (n1 + 16 n2) + {0, 1}
#pragma unroll
            for (int n2 = 0; n2 < 20; ++n2) v[n2] = xs[16 * n2];
        }
        wave_lds_sync();   // every lane's samples are read before the wave overwrites the buffer
#pragma unroll
        for (int n2 = 0; n2 < 20; ++n2) v[n2] *= winl[n1 + 16 * n2];
        if (f1 < FPG) {
            pk_dft20(v);
            // v[5c + d] = Y[c + 4d]; twiddle W320^{n1 k2}
            v2f* zf = zw + f1 * ZS;
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    const int k2 = c + 4 * d;
                    v2f y = v[5 * c + d];
                    if (k2) y = pk_cmul_t(y, twp[(k2 - 1) * 16 + n1]);
                    zf[k2 * 17 + n1] = y;
                }
        }
        wave_lds_sync();
        SPEC_STAMP(1)
        // ---- step 2: 16-point DFTs over n1, lane = (f, k2) -> Z[k2 + 20 k1] ----
        {
            const int f = lane / 20, k2 = lane - 20 * (lane / 20);
            const bool act = f < FPG;
            v2f w[16];
            v2f* zf = zw + min(f, FPG - 1) * ZS;
            if (act) {
#pragma unroll
                for (int n = 0; n < 16; ++n) w[n] = zf[k2 * 17 + n];
            }
            wave_lds_sync();
            if (act) {
                pk_dft16(w);
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int d = 0; d < 4; ++d) zf[k2 + 20 * (c + 4 * d)] = w[4 * c + d];
            }
        }
        wave_lds_sync();
        SPEC_STAMP(2)
        // ---- step 3: real-FFT untangling + magnitudes, item = (f, k): |X[k]|, |X[320 - k]| ----
        {
            constexpr int IT3 = (FPG * 161 + 63) / 64;   // 8
            float mk[IT3], mm[IT3];
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = lane + 64 * j;
                if (it >= FPG * 161) break;
                const int f = it / 161, k = it - 161 * f;
                v2f X, Y;
                pk_untangle(zw + f * ZS, k, ut2, X, Y);
                mk[j] = pk_abs(X);
                mm[j] = pk_abs(Y);
            }
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < IT3; ++j) {
                const int it = lane + 64 * j;
                if (it >= FPG * 161) break;
                const int f = it / 161, k = it - 161 * f;
                float* mf = zwf + f * SEG_FS;
                mf[k] = mk[j];
                mf[320 - k] = mm[j];
            }
            for (int it = lane; it < FPG * SEG_MW; it += 64) {   // bins [321, 321 + SEG_MW) read by the padded band dots
                const int f = it / SEG_MW, j = it - SEG_MW * f;
                zwf[f * SEG_FS + 321 + j] = 0.f;
            }
            wave_lds_sync();
        }
        SPEC_STAMP(3)
        // ---- step 4: Slaney mel + dB, item = (m, f), f fastest: the three lanes of a band read its weights at one LDS
        // address (broadcast; 0.0983 -> 0.094 ms with the float2 twiddle tables) ----
        float vmax = -INFINITY;
        float db[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int it = lane + 64 * j;
            db[j] = -INFINITY;
            if (it >= FPG * n_mels) continue;
            const int m = __umul24(it, 43691) >> 17, f = it - 3 * m;   // m = it / 3 (it < 240)
            const float4* mf = reinterpret_cast<const float4*>(zwf + f * SEG_FS + mel_st[m]);
            const float4* wm = melw4 + m * (SEG_MW / 4);
            // (uniform) quads the pass's bands use: 1-7 of 7 (Slaney widths 5-24 from a 4-aligned start); one
            // straight-line body per count so that all of a band's LDS reads issue back to back (a loop with a break
            // waited for each quad in turn).  The extra leading / trailing terms are x * 0 added to an exact 0 or to
            // the sum: the same value as the sum over the band's own bins.
            float acc;
            switch (a.mel_seg_nq4[j]) {
                case 1: acc = band_dot4<1>(wm, mf); break;
                case 2: acc = band_dot4<2>(wm, mf); break;
                case 3: acc = band_dot4<3>(wm, mf); break;
                case 4: acc = band_dot4<4>(wm, mf); break;
                case 5: acc = band_dot4<5>(wm, mf); break;
                case 6: acc = band_dot4<6>(wm, mf); break;
                default: acc = band_dot4<SEG_MW / 4>(wm, mf); break;
            }
            db[j] = acc > a.amin ? 6.0205999132796239f * __log2f(acc) : a.db_floor;
            vmax = fmaxf(vmax, db[j]);
        }
        // one block barrier per utterance (the dB maximum): each wave keeps its frames' dB values in registers and
        // stores them itself once the maximum is known, so no wave reads another wave's region and the next
        // utterance's step 1 needs no barrier; the maxima alternate between two rows by utterance parity
        wave_lds_sync();   // the magnitude reads are done: the region takes the next samples
        if (nx < n_utt) seg_dma(zwf, a.sig + nx * SEG_L, wave, lane, a.pad_mode);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
        if (lane == 0) wmax[parity][wave] = vmax;
        lds_barrier();
        SPEC_STAMP(4)
        vmax = wmax[parity][0];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) vmax = fmaxf(vmax, wmax[parity][w]);
        const float floor_db = a.top_db >= 0.f ? vmax - a.top_db : -INFINITY;
        const int ts = a.spf == 20 ? 20 : CHUNK;   // frames stored per band (the 20-frame slice drops frame 20)
        float* o = a.mel_db + u * (long long)n_mels * ts;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int it = lane + 64 * j;
            const int m = __umul24(it, 43691) >> 17, t = FPG * wave + it - 3 * m;   // item (m, f): frame 3 w + f
            if (it < FPG * n_mels && t < ts) o[m * ts + t] = fmaxf(db[j], floor_db);
        }
        SPEC_STAMP(5)
    }
}

// ------------------------------------------------------------------------------------------------------------
// k_spec533: n_fft = 533 (int(16000 / 29.97) and int(16000 / 30), data_processor.py:44) by the Good-Thomas prime
// factor algorithm, 533 = 13 x 41 (coprime: no twiddle factors between the stages):
//   input map  n = (41 n1 + 13 n2) mod 533,  output map  k = (287 k1 + 247 k2) mod 533
//   (287 = 41 (41^-1 mod 13), 247 = 13 (13^-1 mod 41)), so that W533^{nk} = W13^{n1 k1} W41^{n2 k2}:
//   stage 1: item (frame t, n1): the real 41-point DFT of x[(41 n1 + 13 n2) mod 533] (windowed), k2 = 0..20 only
//            (real input: k2 and 41 - k2 are conjugate), folded over n2 <-> 41 - n2 (20 cos + 20 sin FMAs per k2);
//   stage 2: item (t, k2 in 0..20): the complex 13-point DFT over n1, folded over n1 <-> 13 - n1 and k1 <-> 13 - k1.
// The 13 x 21 outputs of a frame are its 267 bins once each: (k1, k2) with k2 >= 1 gives bin k or, when k > 266, bin
// 533 - k as conj(X) (the (-k1, -k2) partner has k2 >= 21 and is not computed); k2 = 0 pairs k1 with 13 - k1, of
// which the one with k <= 266 is kept.  14.5K FMAs per frame against the direct DFT's 285K; the cos / sin of both
// DFT lengths are compile-time constants (float32 of the exact values), so no table is read in the stages.
// One 384-thread block per (utterance, chunk of up to 25 frames: the 200-ms segment's 25 frames in one block, whose
// top_db clamp then happens in-kernel as k_spec640's); the padded sample span and the window are staged in LDS.
constexpr int P533_CH = 25;                           // frames per block
constexpr int P533_THREADS = 384;
constexpr int P533_HOPMAX = 160;
constexpr int P533_SPAN = (P533_CH - 1) * P533_HOPMAX + 533;
constexpr int P533_MAGP = 300;                        // magnitude row pitch (267 bins + band-read overrun, zeroed)
constexpr int P533_MW = 32;                           // mel row width staged in LDS (host rows are padded to >= 24)
constexpr int P533_UNION = (P533_SPAN + 536) > P533_CH * P533_MAGP ? (P533_SPAN + 536) : P533_CH * P533_MAGP;
constexpr int P533_LDS = 4 * P533_UNION + 8 * P533_CH * 13 * 21 + 4 * 80 * P533_MW + 8 * 80 + 4 * 8;

__device__ constexpr float kCos41[41] = {
    1.000000000e+00f, 9.882804155e-01f, 9.533963799e-01f, 8.961655498e-01f, 8.179293871e-01f, 7.205215693e-01f,
    6.062254310e-01f, 4.777198136e-01f, 3.380168676e-01f, 1.903911084e-01f, 3.830273449e-02f, -1.146834269e-01f,
    -2.649815083e-01f, -4.090686440e-01f, -5.435675383e-01f, -6.653257012e-01f, -7.714892030e-01f, -8.595696092e-01f,
    -9.275024533e-01f, -9.736953974e-01f, -9.970657825e-01f, -9.970657825e-01f, -9.736953974e-01f, -9.275024533e-01f,
    -8.595696092e-01f, -7.714892030e-01f, -6.653257012e-01f, -5.435675383e-01f, -4.090686440e-01f, -2.649815083e-01f,
    -1.146834269e-01f, 3.830273449e-02f, 1.903911084e-01f, 3.380168676e-01f, 4.777198136e-01f, 6.062254310e-01f,
    7.205215693e-01f, 8.179293871e-01f, 8.961655498e-01f, 9.533963799e-01f, 9.882804155e-01f};
__device__ constexpr float kSin41[41] = {
    0.000000000e+00f, 1.526492834e-01f, 3.017205894e-01f, 4.437198341e-01f, 5.753186345e-01f, 6.934325099e-01f,
    7.952928543e-01f, 8.785122633e-01f, 9.411400557e-01f, 9.817083478e-01f, 9.992662072e-01f, 9.934020638e-01f,
    9.642534852e-01f, 9.125036001e-01f, 8.393654227e-01f, 7.465532422e-01f, 6.362424493e-01f, 5.110186934e-01f,
    3.738170862e-01f, 2.278535068e-01f, 7.654925436e-02f, -7.654925436e-02f, -2.278535068e-01f, -3.738170862e-01f,
    -5.110186934e-01f, -6.362424493e-01f, -7.465532422e-01f, -8.393654227e-01f, -9.125036001e-01f, -9.642534852e-01f,
    -9.934020638e-01f, -9.992662072e-01f, -9.817083478e-01f, -9.411400557e-01f, -8.785122633e-01f, -7.952928543e-01f,
    -6.934325099e-01f, -5.753186345e-01f, -4.437198341e-01f, -3.017205894e-01f, -1.526492834e-01f};
__device__ constexpr float kCos13[13] = {1.000000000e+00f, 8.854560256e-01f, 5.680647492e-01f, 1.205366775e-01f,
                                         -3.546048999e-01f, -7.485107780e-01f, -9.709418416e-01f, -9.709418416e-01f,
                                         -7.485107780e-01f, -3.546048999e-01f, 1.205366775e-01f, 5.680647492e-01f,
                                         8.854560256e-01f};
__device__ constexpr float kSin13[13] = {0.000000000e+00f, 4.647231698e-01f, 8.229838610e-01f, 9.927088618e-01f,
                                         9.350162148e-01f, 6.631226540e-01f, 2.393156588e-01f, -2.393156588e-01f,
                                         -6.631226540e-01f, -9.350162148e-01f, -9.927088618e-01f, -8.229838610e-01f,
                                         -4.647231698e-01f};

__global__ __launch_bounds__(P533_THREADS) void k_spec533(SpecArgs a, int n_chunks) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const seg = sm;                                  // [P533_SPAN] padded samples of the chunk's frames
    float* const win = sm + P533_SPAN;                      // [533] window   (seg / win: stages 0-1)
    float* const mag = sm;                                  // [CH][MAGP]     (stage 2 on: aliases seg / win)
    float2* const Y = reinterpret_cast<float2*>(sm + P533_UNION);                 // [CH][13][21]
    float* const melw = sm + P533_UNION + 2 * P533_CH * 13 * 21;                  // [n_mels][P533_MW]
    int* const mst = reinterpret_cast<int*>(melw + 80 * P533_MW);                 // [n_mels] band starts
    int* const mwd = mst + 80;                                                    // [n_mels] band widths
    float* const red = reinterpret_cast<float*>(mwd + 80);                        // [6] block max
    const int tid = threadIdx.x;
    const long long u = blockIdx.x / n_chunks;
    const int t0 = (int)(blockIdx.x - u * n_chunks) * P533_CH;
    const int nt = min(P533_CH, a.n_frames - t0);
    const long long L = a.n_samples;
    const float* sig = a.sig + u * L;
    const int hop = a.hop;

    // stage 0: the chunk's padded samples (reflect / zero centre padding), the window, the Slaney rows
    const long long s0 = (long long)t0 * hop - 266;
    const int span = (nt - 1) * hop + 533;
    for (int j = tid; j < span; j += P533_THREADS) seg[j] = sample_at(sig, L, s0 + j, a.pad_mode);
    for (int j = tid; j < 533; j += P533_THREADS) win[j] = a.window[j];
    for (int j = tid; j < a.n_mels * P533_MW; j += P533_THREADS) {
        const int m = j / P533_MW, i = j - m * P533_MW;
        melw[j] = i < a.mel_max_width ? a.mel_weight[m * a.mel_max_width + i] : 0.f;
    }
    for (int m = tid; m < a.n_mels; m += P533_THREADS) {
        mst[m] = a.mel_start[m];
        mwd[m] = a.mel_width[m];
    }
    __syncthreads();

    // stage 1: item (t, n1) -> Y[t][n1][k2], k2 = 0..20
    if (tid < nt * 13) {
        const int t = tid / 13, n1 = tid - 13 * t;
        const float* xs = seg + t * hop;
        float x[41];
#pragma unroll
        for (int n2 = 0; n2 < 41; ++n2) {
            int n = 41 * n1 + 13 * n2;
            n = n >= 533 ? n - 533 : n;
            x[n2] = xs[n] * win[n];
        }
        float ps[21], ms[21];   // x[n2] + x[41 - n2], x[n2] - x[41 - n2]
#pragma unroll
        for (int n2 = 1; n2 <= 20; ++n2) {
            ps[n2] = x[n2] + x[41 - n2];
            ms[n2] = x[n2] - x[41 - n2];
        }
        float2* yo = Y + (t * 13 + n1) * 21;
        float r0 = x[0];
#pragma unroll
        for (int n2 = 1; n2 <= 20; ++n2) r0 += ps[n2];
        yo[0] = make_float2(r0, 0.f);
#pragma unroll
        for (int k2 = 1; k2 <= 20; ++k2) {
            float re = x[0], im = 0.f;
#pragma unroll
            for (int n2 = 1; n2 <= 20; ++n2) {
                re = fmaf(ps[n2], kCos41[(n2 * k2) % 41], re);
                im = fmaf(ms[n2], -kSin41[(n2 * k2) % 41], im);
            }
            yo[k2] = make_float2(re, im);
        }
    }
    __syncthreads();

    // stage 2: item (t, k2) -> X(k1, k2), k1 = 0..12 -> |X| rows (and the complex STFT)
    const int nb = 267;
    for (int it = tid; it < nt * 21; it += P533_THREADS) {
        const int t = it / 21, k2 = it - 21 * t;
        const float2* yi = Y + t * 13 * 21 + k2;
        float2 y[13];
#pragma unroll
        for (int n1 = 0; n1 < 13; ++n1) y[n1] = yi[n1 * 21];
        float pr[7], pi[7], mr[7], mi[7];
        float x0r = y[0].x, x0i = y[0].y;
#pragma unroll
        for (int n1 = 1; n1 <= 6; ++n1) {
            pr[n1] = y[n1].x + y[13 - n1].x;
            pi[n1] = y[n1].y + y[13 - n1].y;
            mr[n1] = y[n1].x - y[13 - n1].x;
            mi[n1] = y[n1].y - y[13 - n1].y;
            x0r += pr[n1];
            x0i += pi[n1];
        }
        float2 X[13];
        X[0] = make_float2(x0r, x0i);
#pragma unroll
        for (int k1 = 1; k1 <= 6; ++k1) {
            float A = y[0].x, B = 0.f, C = y[0].y, D = 0.f;
#pragma unroll
            for (int n1 = 1; n1 <= 6; ++n1) {
                const float c = kCos13[(n1 * k1) % 13], s = kSin13[(n1 * k1) % 13];
                A = fmaf(pr[n1], c, A);
                B = fmaf(mi[n1], s, B);
                C = fmaf(pi[n1], c, C);
                D = fmaf(mr[n1], s, D);
            }
            X[k1] = make_float2(A + B, C - D);
            X[13 - k1] = make_float2(A - B, C + D);
        }
        float* mrow = mag + t * P533_MAGP;
#pragma unroll
        for (int k1 = 0; k1 < 13; ++k1) {
            int k = (287 * k1 + 247 * k2) % 533;
            float2 v = X[k1];
            if (k > 266) {
                if (k2 == 0) continue;   // the k1 <-> 13 - k1 partner holds this bin
                k = 533 - k;
                v.y = -v.y;
            }
            mrow[k] = __builtin_amdgcn_sqrtf(v.x * v.x + v.y * v.y);
            if (a.stft_ri) reinterpret_cast<float2*>(a.stft_ri)[(u * nb + k) * a.n_frames + t0 + t] = v;
        }
    }
    // the rows' tails past bin 266 (read by the padded band dots) are zero
    for (int j = tid; j < nt * (P533_MAGP - 267); j += P533_THREADS) {
        const int t = j / (P533_MAGP - 267);
        mag[t * P533_MAGP + 267 + (j - t * (P533_MAGP - 267))] = 0.f;
    }
    __syncthreads();

    // stage 3: Slaney mel + dB, item (m, t); top_db in-kernel when the block holds the whole utterance
    const bool whole = n_chunks == 1;
    float vmax = -INFINITY;
    constexpr int NIT = (80 * P533_CH + P533_THREADS - 1) / P533_THREADS;
    float dbv[NIT];
#pragma unroll
    for (int r = 0; r < NIT; ++r) {
        const int it = tid + r * P533_THREADS;
        dbv[r] = -INFINITY;
        if (it >= a.n_mels * nt) continue;
        const int m = it / nt, t = it - m * nt;
        const float* mf = mag + t * P533_MAGP + mst[m];
        const float* wm = melw + m * P533_MW;
        float acc = 0.f;
        for (int j = 0; j < mwd[m]; ++j) acc = fmaf(mf[j], wm[j], acc);
        const float db = acc > a.amin ? 20.0f * log10f(acc) : a.db_floor;
        dbv[r] = db;
        vmax = fmaxf(vmax, db);
        if (!whole) {
            const long long oi = out_index(a.spf, a.n_slices, a.n_mels, a.n_frames, u, m, t0 + t);
            if (oi >= 0) a.mel_db[oi] = db;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
    if (!whole) {
        if ((tid & 63) == 0) atomicMax(a.umax + u, f2ord(vmax));
        return;
    }
    if ((tid & 63) == 0) red[tid >> 6] = vmax;
    __syncthreads();
    vmax = red[0];
#pragma unroll
    for (int w = 1; w < P533_THREADS / 64; ++w) vmax = fmaxf(vmax, red[w]);
    const float floor_db = a.top_db >= 0.f ? vmax - a.top_db : -INFINITY;
#pragma unroll
    for (int r = 0; r < NIT; ++r) {
        const int it = tid + r * P533_THREADS;
        if (it >= a.n_mels * nt) continue;
        const int m = it / nt, t = it - m * nt;
        const long long oi = out_index(a.spf, a.n_slices, a.n_mels, a.n_frames, u, m, t0 + t);
        if (oi >= 0) a.mel_db[oi] = fmaxf(dbv[r], floor_db);
    }
}

// Direct DFT fallback for n_fft != 640 / 533: one 256-thread block per (frame, utterance).
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

#ifdef AVSE_STFT_STAMP
extern "C" int avse_spec_stamps(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_spec_stamps), sizeof(unsigned long long) * 4096 * 8) != hipSuccess) return 2;
    if (reset) {
        static unsigned long long zero[4096 * 8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_spec_stamps), zero, sizeof(zero)) != hipSuccess) return 2;
    }
    return 0;
}
#endif

int launch_spectrogram(const SpecArgs& a, hipStream_t s) {
    if (a.n_utt <= 0) return 0;
    const bool need_clamp_pass = a.top_db >= 0.f;
    if (a.n_fft == 640) {
        const int n_chunks = (a.n_frames + CHUNK - 1) / CHUNK;
        const long long items = (long long)n_chunks * a.n_utt;
        if (items > INT32_MAX || a.n_samples > INT32_MAX) {
            set_error("spectrogram batch too large (n_utt * chunks and n_samples must fit in int32)");
            return 3;   // AVSE_ERR_UNSUPPORTED
        }
        if (n_chunks > 1) AVSE_HIP_CHECK(hipMemsetAsync(a.umax, 0, sizeof(unsigned) * a.n_utt, s));
        const bool fast = a.n_mels <= 80 && a.mel_max_width == MW, ri = a.stft_ri != nullptr;
        const dim3 grid((unsigned)items), block(64 * WAVES);
#ifndef AVSE_NO_SEG
        if (fast && !ri && a.n_samples == SEG_L && a.n_frames == CHUNK && a.hop == 160 &&
            ((reinterpret_cast<uintptr_t>(a.sig) | reinterpret_cast<uintptr_t>(a.mel_db)) & 15) == 0 &&
            (a.spf == 0 || (a.spf == 20 && a.n_slices == 1))) {
            int dev = 0, cus = 256;
            AVSE_HIP_CHECK(hipGetDevice(&dev));
            AVSE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const unsigned g = (unsigned)std::min<long long>(a.n_utt, (long long)AVSE_SEG_BPC * cus);
            hipLaunchKernelGGL(k_spec_seg, dim3(g), block, 0, s, a);
            AVSE_HIP_CHECK(hipGetLastError());
            return 0;
        }
#endif
        if (fast && ri) hipLaunchKernelGGL((k_spec640<true, true>), grid, block, 0, s, a, n_chunks);
        else if (fast) hipLaunchKernelGGL((k_spec640<true, false>), grid, block, 0, s, a, n_chunks);
        else if (ri) hipLaunchKernelGGL((k_spec640<false, true>), grid, block, 0, s, a, n_chunks);
        else hipLaunchKernelGGL((k_spec640<false, false>), grid, block, 0, s, a, n_chunks);
        AVSE_HIP_CHECK(hipGetLastError());
        if (n_chunks > 1 && need_clamp_pass) {
            hipLaunchKernelGGL(k_spec_clamp, dim3(1024), dim3(256), 0, s, a);
            AVSE_HIP_CHECK(hipGetLastError());
        }
        return 0;
    }
    if (a.n_fft == 533 && a.hop <= P533_HOPMAX && a.n_mels <= 80 && a.mel_max_width <= P533_MW) {
        const int n_chunks = (a.n_frames + P533_CH - 1) / P533_CH;
        const long long items = (long long)n_chunks * a.n_utt;
        if (items > INT32_MAX) {
            set_error("spectrogram batch too large (n_utt * chunks must fit in int32)");
            return 3;   // AVSE_ERR_UNSUPPORTED
        }
        if (int rc = ensure_lds_attr((const void*)k_spec533, P533_LDS)) return rc;
        if (n_chunks > 1) AVSE_HIP_CHECK(hipMemsetAsync(a.umax, 0, sizeof(unsigned) * a.n_utt, s));
        hipLaunchKernelGGL(k_spec533, dim3((unsigned)items), dim3(P533_THREADS), P533_LDS, s, a, n_chunks);
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
