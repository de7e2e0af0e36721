// Persistent, warp-specialised implicit-GEMM for the bf16 layers outside the video trunk's big convs:
// audio encoder a_conv2..5 (network.py:92-109), v_conv6 (:169), the three Dense layers (:56, :69,
// :75-78) and the deconvolution decoder d_deconv1..5 (:112-133).  Same layer semantics and argument
// block (ConvArgs) as the generic k_conv in conv.hip — TF 'SAME' zero padding, deconvolution as
// sub-pixel phases with per-phase tap tables, folded bias/BN scale-shift, LeakyReLU(0.3), fused 2x2 max
// pool with the pool-window M order, strided NHWC stores into concat slices, split-K with fp32
// partials — re-organised the way conv_stream.hip is (see its header for the measurements):
//   * 512 threads: 4 compute waves (one per SIMD, tile 64 x BN each, v_mfma_f32_32x32x16_bf16,
//     issue priority) + 4 loader waves (all address arithmetic, im2col gathers, LDS stores);
//   * persistent over work items (phase, K-split, M-tile of 256 rows, N-tile of BN), numbered so each
//     XCD walks a contiguous block (its L2 keeps the shared im2col window); one barrier per
//     64-deep K step, which the compute waves run as two 32-deep halves (fragments of the next half
//     are read while the current half's MFMAs run);
//   * a loader lane owns 64 contiguous bytes (32 channels of one tap, Ci % 32 == 0) of two A rows per
//     step: one bounds/address computation feeds four 16-byte loads (the 32-deep first version spent
//     its loader issue on per-chunk address arithmetic and was slower than k_conv);
//   * loads run LAT + 2 steps ahead of their step into a ring of LAT register sets; the set loaded LAT
//     steps earlier is stored into a 3-slot LDS ring (vmcnt retires in order; the ring gives the
//     gathers LAT - 1 whole steps of latency budget).
// LDS images (conflict-free for the 32x32x16 operand reads): A row r / B row n is 128 B, 16-B chunk j
// at position j ^ ((row >> 1) & 7).
#include <type_traits>

#include "avse_common.h"

namespace avse {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;
constexpr int BM = 256;         // rows per work item (4 compute waves x 64)
constexpr int BK = 64;          // K elements per step
constexpr int LAT = 4;          // load -> LDS store distance in steps
constexpr int NS = 3;           // LDS slots
constexpr int MAXTAPS = 128;    // tap table entries staged in LDS

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ i32x4 ld16(__amdgpu_buffer_rsrc_t rs, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
}

// work-item geometry (identical in both roles)
struct Item {
    int ph, ks, m0, n0;
    int k0;       // first K element of this split
    int kend;     // one past its last K element
    int steps;    // max(ceil((kend - k0) / BK), 1)
};

template <int BN>
struct Geo {
    static constexpr int NB = BN / 32;                    // 32-wide N blocks per compute wave
    static constexpr int ASLOT = BM * 128, BSLOT = BN * 128;
    static constexpr int SLOT = ASLOT + BSLOT;
    static constexpr int BLD = BN == 128 ? 4 : 2;         // B loads per loader lane per step
    static constexpr int NLD = 8 + BLD;                   // loads per loader lane per step
    static constexpr int LDS = NS * SLOT + MAXTAPS * 8;
};

template <int BN>
__global__ __launch_bounds__(512, 1) void k_igemm(ConvArgs a, int mtiles, int ntiles, int nitems) {
    using G = Geo<BN>;
    constexpr int NB = G::NB, ASLOT = G::ASLOT, SLOT = G::SLOT, BLD = G::BLD, NLD = G::NLD;

    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const ring = lds;                                        // [NS][ASLOT + BSLOT]
    int2* const tapl = reinterpret_cast<int2*>(lds + NS * SLOT);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;
    // XCD-aware numbering: workgroups are dealt round-robin to the 8 XCDs (b % 8); renumber so each XCD
    // walks a contiguous block of work items and its 4 MB L2 holds the im2col window they share
    const int gx = (int)gridDim.x, b = (int)blockIdx.x;
    const int vb = gx % 8 == 0 ? (b % 8) * (gx / 8) + b / 8 : b;
    const int nmine = (nitems - vb + gx - 1) / gx;
    if (nmine <= 0) return;
    const int M = a.N * a.Hq * a.Wq;

    auto item = [&](int k) {
        Item it;
        const int id = vb + k * gx;
        const int nt = id % ntiles, r1 = id / ntiles;
        const int mt = r1 % mtiles, r2 = r1 / mtiles;
        it.ks = r2 % a.ksplit;
        it.ph = r2 / a.ksplit;
        it.m0 = mt * BM;
        it.n0 = nt * BN;
        const int K = a.ph[it.ph].kpad;
        const int nst = (K + BK - 1) / BK;
        const int sps = (nst + a.ksplit - 1) / a.ksplit;
        it.k0 = min(K, it.ks * sps * BK);
        it.kend = min(K, it.k0 + sps * BK);
        it.steps = max((it.kend - it.k0 + BK - 1) / BK, 1);
        return it;
    };
    // total steps of this workgroup, padded to a multiple of LAT (extra steps: barriers only)
    int total = 0;
    for (int k = 0; k < nmine; ++k) total += item(k).steps;
    const int total_pad = (total + LAT - 1) / LAT * LAT;

    if (wave >= 4) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;
        {
            int ntap = 0;
            for (int p = 0; p < a.nphase; ++p) ntap = max(ntap, a.ph[p].tap_off + a.ph[p].ntaps);
            for (int i = L; i < ntap && i < MAXTAPS; i += 256) tapl[i] = a.taps[i];
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        barrier_raw();

        const __amdgpu_buffer_rsrc_t rsA = make_rsrc(a.in, (long long)a.N * a.in_clip_stride * 2);
        const __amdgpu_buffer_rsrc_t rsB = make_rsrc(a.w, 0x7fffffffLL);
        const int h = L & 1;                // A: which 64-byte half of the 128-byte row
        const int ci = a.Ci;
        // B lanes: BN = 128: row L >> 1, 64 B at (L & 1) * 64; BN = 64: row L >> 2, 32 B at (L & 3) * 32
        const int brow = BN == 128 ? (L >> 1) : (L >> 2);
        const int bbyte = BN == 128 ? (L & 1) * 64 : (L & 3) * 32;
        // cursor: the step being loaded
        int ck = 0, cs = 0;
        Item cit = item(0);
        int rcb[2], riy[2], rix[2];          // A rows r = L/2 + 128u: clip byte base (< 0: past M), iy0, ix0
        int kj = 0, kc = 0;                 // tap / channel of this lane's 32 elements in the step
        int ke = 0;                         // their K index (>= kend: zeros)
        auto set_rows = [&]() {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int m = cit.m0 + (L >> 1) + 128 * u;
                const int mm = m < M ? m : 0;
                int clip, yq, xq;
                if (a.pool) {
                    const int p = mm >> 2, q = mm & 3, pw = a.Wq >> 1, phh = a.Hq >> 1;
                    clip = p / (phh * pw);
                    const int r = p - clip * phh * pw;
                    yq = 2 * (r / pw) + (q >> 1);
                    xq = 2 * (r % pw) + (q & 1);
                } else {
                    clip = mm / (a.Hq * a.Wq);
                    const int r = mm - clip * a.Hq * a.Wq;
                    yq = r / a.Wq;
                    xq = r - (r / a.Wq) * a.Wq;
                }
                rcb[u] = m < M ? clip * (int)a.in_clip_stride * 2 : -1;
                riy[u] = yq * a.sy;
                rix[u] = xq * a.sx;
            }
            ke = cit.k0 + 32 * h;
            kj = ke / ci;
            kc = ke - kj * ci;
        };
        set_rows();
        auto advance = [&]() {
            ke += BK;
            kc += BK;
            while (kc >= ci) { kc -= ci; ++kj; }
            if (++cs == cit.steps) {
                cs = 0;
                if (++ck < nmine) {
                    cit = item(ck);
                    set_rows();
                }
            }
        };
        auto load = [&](i32x4 (&ra)[8], i32x4 (&rb)[BLD]) {
            const int live = (int)(ck < nmine);
            const ConvPhase& ph = a.ph[live ? cit.ph : 0];
            const int2 t = tapl[ph.tap_off + min(kj, ph.ntaps - 1)];
            const int kok = live & (int)(ke < cit.kend) & (int)(kj < ph.ntaps);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int iy = riy[u] + t.x, ix = rix[u] + t.y;
                const int ok = kok & (int)(rcb[u] >= 0) & (int)((unsigned)iy < (unsigned)a.Hi) &
                               (int)((unsigned)ix < (unsigned)a.Wi);
                const int off = rcb[u] + ((iy * a.Wi + ix) * ci + kc) * 2, mask = -ok;
                const int o = (off & mask) | (kOOB & ~mask);
#pragma unroll
                for (int j = 0; j < 4; ++j) ra[4 * u + j] = ld16(rsA, o + 16 * j);
            }
            // B: this step's K window [k0 + cs*BK, +BK) of rows n0 + brow (zeros past Co / past kend)
            const int kb = cit.k0 + cs * BK + bbyte / 2;
            const int n = cit.n0 + brow;
            const int okb = live & (int)(n < a.Co) & (int)(kb < cit.kend), maskb = -okb;
            const int offb = ((((int)ph.w_off + n * ph.kpad + kb) * 2) & maskb) | (kOOB & ~maskb);
#pragma unroll
            for (int j = 0; j < BLD; ++j) rb[j] = ld16(rsB, offb + 16 * j);
        };
        auto store = [&](int slot, const i32x4 (&ra)[8], const i32x4 (&rb)[BLD]) {
            char* as = ring + slot * SLOT;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int row = (L >> 1) + 128 * u;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    *reinterpret_cast<i32x4*>(as + row * 128 + (((4 * h + j) ^ swz(row)) << 4)) = ra[4 * u + j];
            }
#pragma unroll
            for (int j = 0; j < BLD; ++j)
                *reinterpret_cast<i32x4*>(as + ASLOT + brow * 128 + (((bbyte / 16 + j) ^ swz(brow)) << 4)) = rb[j];
        };
        // prologue: steps 0, 1 straight to LDS slots 0, 1; steps 2 .. LAT+1 into the register ring
        i32x4 ra[LAT][8], rb[LAT][BLD];
        {
            i32x4 ta[8], tb[BLD];
            load(ta, tb);
            advance();
            wait_vm_lgkm0<0>();
            store(0, ta, tb);
            load(ta, tb);
            advance();
            wait_vm_lgkm0<0>();
            store(1, ta, tb);
        }
        [&]<int... S>(std::integer_sequence<int, S...>) { ((load(ra[S], rb[S]), advance()), ...); }(
            std::make_integer_sequence<int, LAT>{});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();
        // step t: store the set loaded LAT steps ago (step t+2) into slot (t+2) % 3 — its previous
        // contents (step t-1) were read before the last barrier — and load step t+LAT+2 into that set
        int sl = 2;
        for (int t = 0; t < total_pad; t += LAT)
            [&]<int... S>(std::integer_sequence<int, S...>) {
                ((store(sl, ra[S], rb[S]), load(ra[S], rb[S]), advance(), wait_vm_lgkm0<(LAT - 1) * NLD>(),
                  barrier_raw(), sl = sl == NS - 1 ? 0 : sl + 1),
                 ...);
            }(std::make_integer_sequence<int, LAT>{});
        wait_vm_lgkm0<0>();
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    barrier_raw();   // tap tables
    barrier_raw();   // prologue steps
    const int r32 = lane & 31, hi = lane >> 5;
    const int asw = swz(r32);
    // fragments of half hf (K 32 hf .. 32 hf + 31) of the step in slot `slot`
    auto frags = [&](int slot, int hf, i32x4 (&fa)[4], i32x4 (&fb)[2 * NB]) {
        const char* as = ring + slot * SLOT;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int pos = ((4 * hf + 2 * m + hi) ^ asw) << 4;
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[2 * i + m] = *reinterpret_cast<const i32x4*>(as + (64 * w + 32 * i + r32) * 128 + pos);
#pragma unroll
            for (int jb = 0; jb < NB; ++jb) fb[2 * jb + m] = *reinterpret_cast<const i32x4*>(as + ASLOT + (32 * jb + r32) * 128 + pos);
        }
    };
    f32x16 acc[2][NB];
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(a.out, 0x7fffffffLL);
    const __amdgpu_buffer_rsrc_t prs = make_rsrc(a.partial, 0x7fffffffLL);
    // accumulator register 4g + e of block i, column block jb: row 64w + 32i + 8g + 4hi + e, column 32jb + r32
    auto epilogue = [&](const Item& it) {
        const ConvPhase& ph = a.ph[it.ph];
#pragma unroll
        for (int jb = 0; jb < NB; ++jb) {
            const int n = it.n0 + 32 * jb + r32;
            const bool nok = n < a.Co;
            const float sc = nok ? a.scale[n] : 0.f, sh = nok ? a.shift[n] : 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int mb = it.m0 + 64 * w + 32 * i + 8 * g + 4 * hi;
                    if (a.ksplit > 1) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int ok = (int)nok & (int)(mb + e < M), mask = -ok;
                            const int off = ((it.ks * M + mb + e) * a.Co + n) * 4;
                            // (the element is copied first: __builtin_bit_cast on an ext-vector element
                            // lvalue reads element 0 — measured wrong partial sums)
                            const float v = acc[i][jb][4 * g + e];
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), prs, (off & mask) | (kOOB & ~mask), 0, 0);
                        }
                    } else if (a.pool) {
                        float x = -INFINITY;
#pragma unroll
                        for (int e = 0; e < 4; ++e) x = fmaxf(x, fmaf(acc[i][jb][4 * g + e], sc, sh));
                        if (a.act) x = fmaxf(x, LRELU * x);
                        const int p = mb >> 2, pw = a.Wq >> 1, phh = a.Hq >> 1;
                        const int clip = p / (phh * pw), r = p - clip * phh * pw;
                        const int ok = (int)nok & (int)(mb < M), mask = -ok;
                        const int off = ((int)(clip * a.out_clip_stride) + r * a.out_pix_stride + a.out_c_off + n) * 2;
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)x), ors,
                                                              (off & mask) | (kOOB & ~mask), 0, 0);
                    } else {
                        // (clip, yq, xq) of row mb once per 4-row group, then carried across the 4 rows
                        const int mm = mb < M ? mb : 0;
                        int clip = mm / (a.Hq * a.Wq);
                        const int rr = mm - clip * a.Hq * a.Wq;
                        int yq = rr / a.Wq, xq = rr - (rr / a.Wq) * a.Wq;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float x = fmaf(acc[i][jb][4 * g + e], sc, sh);
                            if (a.act) x = fmaxf(x, LRELU * x);
                            const int oy = yq * a.oys + ph.py, ox = xq * a.oxs + ph.px;
                            const int ok = (int)nok & (int)(mb + e < M), mask = -ok;
                            const int off = ((int)(clip * a.out_clip_stride) + (oy * a.Wo + ox) * a.out_pix_stride + a.out_c_off + n) * 2;
                            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)x), ors,
                                                                  (off & mask) | (kOOB & ~mask), 0, 0);
                            if (++xq == a.Wq) {
                                xq = 0;
                                if (++yq == a.Hq) {
                                    yq = 0;
                                    ++clip;
                                }
                            }
                        }
                    }
                }
        }
    };
    auto mfma_half = [&](auto first, const i32x4 (&ca)[4], const i32x4 (&cb)[2 * NB]) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jb = 0; jb < NB; ++jb)
                    acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, ca[2 * i + m]), __builtin_bit_cast(bf16x8, cb[2 * jb + m]),
                        (decltype(first)::value && m == 0) ? (f32x16){} : acc[i][jb], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 2 + 2 * NB; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // X: first half of the current step (read during the previous step), Y: its second half
    i32x4 xa[4], xb[2 * NB], ya[4], yb[2 * NB];
    int slot = 0;
    frags(0, 0, xa, xb);
    int t = 0;
    auto cstep = [&](auto first) {
        const int nslot = slot == NS - 1 ? 0 : slot + 1;
        frags(slot, 1, ya, yb);
        mfma_half(first, xa, xb);
        frags(nslot, 0, xa, xb);
        mfma_half(std::false_type{}, ya, yb);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();
        slot = nslot;
        ++t;
    };
    for (int k = 0; k < nmine; ++k) {
        const Item it = item(k);
        cstep(std::true_type{});
        for (int s = 1; s < it.steps; ++s) cstep(std::false_type{});
        epilogue(it);
    }
    for (; t < total_pad; ++t) barrier_raw();   // the loaders' padding steps
}

}  // namespace

int choose_ksplit_ws(long long M, int Co, int kpad) {
    const int BN = Co <= 64 ? 64 : 128;
    const long long items = ((M + BM - 1) / BM) * ((Co + BN - 1) / BN);
    const int nstep = (kpad + BK - 1) / BK;
    int ks = 1;
    while (items * ks < 256 && nstep / (ks * 2) >= 4) ks *= 2;
    return ks;
}

int launch_igemm(const ConvArgs& a, hipStream_t s) {
    const int M = a.N * a.Hq * a.Wq;
    const int BN = (a.Co <= 64) ? 64 : 128;
    if (a.ksplit < 1 || (a.ksplit > 1 && (a.nphase != 1 || !a.partial))) {
        set_error("bad split-K configuration");
        return 1;
    }
    if (a.Ci % 32) {
        set_error("igemm: Ci must be a multiple of 32");
        return 3;
    }
    for (int p = 0; p < a.nphase; ++p)
        if (a.ph[p].tap_off + a.ph[p].ntaps > MAXTAPS || a.ph[p].kpad % 32) {
            set_error("igemm: tap table too large or K not slab-aligned");
            return 3;
        }
    if ((long long)a.N * a.in_clip_stride * 2 >= kOOB || (long long)a.N * a.out_clip_stride * 2 >= kOOB ||
        (a.ksplit > 1 && (long long)a.ksplit * M * a.Co * 4 >= kOOB)) {
        set_error("igemm: tensor exceeds 32-bit buffer offsets");
        return 3;
    }
    const int mtiles = (M + BM - 1) / BM, ntiles = (a.Co + BN - 1) / BN;
    const int nitems = a.nphase * a.ksplit * mtiles * ntiles;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int gx = nitems < ncu ? nitems : ncu;
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_igemm<64>, hipFuncAttributeMaxDynamicSharedMemorySize, Geo<64>::LDS));
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_igemm<128>, hipFuncAttributeMaxDynamicSharedMemorySize, Geo<128>::LDS));
        attr = true;
    }
    // both sizes exceed 80 KB: one workgroup per CU
    static_assert(Geo<64>::LDS > 80 * 1024 && Geo<128>::LDS <= 160 * 1024, "igemm LDS budget");
    if (BN == 64) hipLaunchKernelGGL(k_igemm<64>, dim3(gx), dim3(512), Geo<64>::LDS, s, a, mtiles, ntiles, nitems);
    else hipLaunchKernelGGL(k_igemm<128>, dim3(gx), dim3(512), Geo<128>::LDS, s, a, mtiles, ntiles, nitems);
    AVSE_HIP_CHECK(hipGetLastError());
    if (a.ksplit > 1) return launch_splitk_reduce(a, 1, s);
    return 0;
}

}  // namespace avse
