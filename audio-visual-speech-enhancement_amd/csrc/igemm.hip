// Persistent, warp-specialised implicit-GEMM for the bf16 layers outside the video trunk's big convs:
// audio encoder a_conv1..5 (network.py:88-109), v_conv6 (:169), the three Dense layers (:56, :69,
// :75-78) and the deconvolution decoder d_deconv1..5 (:112-133).  Same layer semantics and argument
// block (ConvArgs) as the generic k_conv in conv.hip — TF 'SAME' zero padding, deconvolution as
// sub-pixel phases with per-phase tap tables, folded bias/BN scale-shift, LeakyReLU(0.3), fused 2x2 max
// pool with the pool-window M order, strided NHWC stores into concat slices, split-K with fp32
// partials — re-organised the way conv_stream.hip is (see its header for the measurements):
//   * 512 threads: 4 compute waves (one per SIMD, tile 64 x BN each, v_mfma_f32_32x32x16_bf16,
//     issue priority) + 4 loader waves (all address arithmetic, im2col gathers, LDS stores);
//   * persistent over work items (phase, K-split, M-tile of 256 rows, N-tile of BN); each item's K loop
//     runs in 32-element slabs, one slab and one barrier per step, padded to an even step count;
//   * loaders issue every load LAT + 2 steps ahead of its slab into a ring of LAT register sets and
//     store the set loaded LAT steps earlier into a 2-slot LDS ring (vmcnt retires in order; the
//     ring gives the im2col gathers LAT-1 whole steps of latency budget).
// LDS images (conflict-free for the 32x32x16 operand reads): A row r / B row n is 64 B, 16-B chunk j
// at position j ^ ((row >> 2) & 3).
#include <type_traits>

#include "avse_common.h"

namespace avse {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;
constexpr int BM = 256;         // rows per work item (4 compute waves x 64)
constexpr int LAT = 4;          // load -> LDS store distance in steps
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
__device__ __forceinline__ int swz(int row) { return (row >> 2) & 3; }

// work-item geometry (identical in both roles)
struct Item {
    int ph, ks, m0, n0;
    int sb;       // first slab of this K-split
    int nreal;    // slabs with data
    int steps;    // max(nreal, 1) rounded up to even
};

template <int BN>
__global__ __launch_bounds__(512, 1) void k_igemm(ConvArgs a, int mtiles, int ntiles, int nitems) {
    constexpr int NB = BN / 32;                       // 32-wide N blocks per compute wave
    constexpr int ASLOT = BM * 64, BSLOT = BN * 64;   // one slab of A / B
    constexpr int NBL = BN * 4 / 256;                 // B loads per loader lane per step
    constexpr int NLD = 4 + NBL;                      // loads per loader lane per step

    extern __shared__ __attribute__((aligned(1024))) char lds[];   // launch: > 80 KB, one workgroup per CU
    char* const ring = lds;                                        // [2][ASLOT + BSLOT]
    int2* const tapl = reinterpret_cast<int2*>(lds + 2 * (ASLOT + BSLOT));

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;
    const int nmine = (nitems - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    if (nmine <= 0) return;
    const int M = a.N * a.Hq * a.Wq;

    auto item = [&](int k) {
        Item it;
        const int id = (int)blockIdx.x + k * (int)gridDim.x;
        const int nt = id % ntiles, r1 = id / ntiles;
        const int mt = r1 % mtiles, r2 = r1 / mtiles;
        it.ks = r2 % a.ksplit;
        it.ph = r2 / a.ksplit;
        it.m0 = mt * BM;
        it.n0 = nt * BN;
        const int nslab = a.ph[it.ph].kpad / 32;
        const int sps = (nslab + a.ksplit - 1) / a.ksplit;
        it.sb = it.ks * sps;
        const int se = min(nslab, it.sb + sps);
        it.nreal = max(se - it.sb, 0);
        it.steps = (max(it.nreal, 1) + 1) & ~1;
        return it;
    };
    // total steps of this workgroup, padded to a multiple of LAT (extra steps: barriers only)
    int total = 0;
    for (int k = 0; k < nmine; ++k) total += item(k).steps;
    const int total_pad = (total + LAT - 1) / LAT * LAT;

    if (wave >= 4) {
        // =============================== loader waves ===============================
        const int L = w * 64 + lane;
        // stage every phase's tap table
        {
            int ntap = 0;
            for (int p = 0; p < a.nphase; ++p) ntap = max(ntap, a.ph[p].tap_off + a.ph[p].ntaps);
            for (int i = L; i < ntap && i < MAXTAPS; i += 256) tapl[i] = a.taps[i];
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        barrier_raw();

        const __amdgpu_buffer_rsrc_t rsA = make_rsrc(a.in, (long long)a.N * a.in_clip_stride * 2);
        const __amdgpu_buffer_rsrc_t rsB = make_rsrc(a.w, 0x7fffffffLL);
        const int g = L & 3;               // this lane's 16-B chunk column (A)
        const int ci = a.Ci;
        // cursor: the slab being loaded (WD steps ahead of the computing step)
        int ck = 0, cs = 0;                 // local item, step within item
        Item cit = item(0);
        int rcb[4], riy[4], rix[4];          // A rows r = L/4 + 64u: clip byte base, iy0, ix0 (row < M: rcb >= 0)
        int kj = 0, kc = 0;                 // tap / channel of this lane's chunk in the current slab
        auto set_rows = [&]() {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = cit.m0 + (L >> 2) + 64 * u;
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
            const int e = cit.sb * 32 + g * 8;
            kj = e / ci;
            kc = e - kj * ci;
        };
        set_rows();
        auto advance = [&]() {
            kc += 32;
            while (kc >= ci) { kc -= ci; ++kj; }
            if (++cs == cit.steps) {
                cs = 0;
                if (++ck < nmine) {
                    cit = item(ck);
                    set_rows();
                }
            }
        };
        // loads of the cursor's slab into a register set (zeros past the item's data / the last item)
        auto load = [&](i32x4 (&ra)[4], i32x4 (&rb)[NBL]) {
            const bool live = ck < nmine && cs < cit.nreal;
            const ConvPhase& ph = a.ph[live ? cit.ph : 0];
            const int2 t = tapl[ph.tap_off + min(kj, ph.ntaps - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int iy = riy[u] + t.x, ix = rix[u] + t.y;
                const int ok = (int)live & (int)(rcb[u] >= 0) & (int)(kj < ph.ntaps) & (int)((unsigned)iy < (unsigned)a.Hi) &
                               (int)((unsigned)ix < (unsigned)a.Wi);
                const int off = rcb[u] + ((iy * a.Wi + ix) * ci + kc) * 2;
                const int mask = -ok;
                ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rsA, (off & mask) | (kOOB & ~mask), 0, 0);
            }
            const int slab = cit.sb + cs;
#pragma unroll
            for (int v = 0; v < NBL; ++v) {
                const int idx = L + 256 * v, row = idx >> 2, gg = idx & 3;
                const int n = cit.n0 + row;
                const int ok = (int)live & (int)(n < a.Co);
                const int off = ((int)ph.w_off + n * ph.kpad + slab * 32 + gg * 8) * 2;
                const int mask = -ok;
                rb[v] = __builtin_amdgcn_raw_buffer_load_b128(rsB, (off & mask) | (kOOB & ~mask), 0, 0);
            }
        };
        auto store = [&](int slot, const i32x4 (&ra)[4], const i32x4 (&rb)[NBL]) {
            char* as = ring + slot * (ASLOT + BSLOT);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int row = (L >> 2) + 64 * u;
                *reinterpret_cast<i32x4*>(as + row * 64 + ((g ^ swz(row)) << 4)) = ra[u];
            }
#pragma unroll
            for (int v = 0; v < NBL; ++v) {
                const int idx = L + 256 * v, row = idx >> 2, gg = idx & 3;
                *reinterpret_cast<i32x4*>(as + ASLOT + row * 64 + ((gg ^ swz(row)) << 4)) = rb[v];
            }
        };
        // prologue: slabs of steps 0, 1 straight to LDS; steps 2 .. LAT+1 into the register ring
        i32x4 ra[LAT][4], rb[LAT][NBL];
        {
            i32x4 ta[4], tb[NBL];
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
        barrier_raw();   // the compute waves have read slab 0 (slot 0 is overwritten at step 0)
        // step t: store the set loaded LAT steps ago (slab of step t+2) into ring slot t&1, load the
        // slab of step t+WD into the same set
        for (int t = 0; t < total_pad; t += LAT)
            [&]<int... S>(std::integer_sequence<int, S...>) {
                ((store(S & 1, ra[S], rb[S]), load(ra[S], rb[S]), advance(), wait_vm_lgkm0<(LAT - 1) * NLD>(),
                  barrier_raw()),
                 ...);
            }(std::make_integer_sequence<int, LAT>{});   // LAT even: slot (t + S) & 1 == S & 1
        wait_vm_lgkm0<0>();
        return;
    }

    // =============================== compute waves ===============================
    __builtin_amdgcn_s_setprio(2);
    barrier_raw();   // tap tables
    barrier_raw();   // prologue slabs
    const int r32 = lane & 31, hi = lane >> 5;
    const int asw = swz(r32);
    auto frags = [&](int slot, i32x4 (&fa)[4], i32x4 (&fb)[2 * NB]) {
        const char* as = ring + slot * (ASLOT + BSLOT);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int pos = ((2 * m + hi) ^ asw) << 4;
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[2 * i + m] = *reinterpret_cast<const i32x4*>(as + (64 * w + 32 * i + r32) * 64 + pos);
#pragma unroll
            for (int jb = 0; jb < NB; ++jb) fb[2 * jb + m] = *reinterpret_cast<const i32x4*>(as + ASLOT + (32 * jb + r32) * 64 + pos);
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
    i32x4 fa[4], fb[2 * NB], na[4], nb[2 * NB];
    frags(0, fa, fb);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();   // slab 0 read: the loaders may now overwrite slot 0
    int t = 0;
    auto cstep = [&](auto first, i32x4 (&ca)[4], i32x4 (&cb)[2 * NB], i32x4 (&xa)[4], i32x4 (&xb)[2 * NB]) {
        frags((t + 1) & 1, xa, xb);
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();
        ++t;
    };
    for (int k = 0; k < nmine; ++k) {
        const Item it = item(k);
        cstep(std::true_type{}, fa, fb, na, nb);
        cstep(std::false_type{}, na, nb, fa, fb);
        for (int s = 2; s < it.steps; s += 2) {
            cstep(std::false_type{}, fa, fb, na, nb);
            cstep(std::false_type{}, na, nb, fa, fb);
        }
        epilogue(it);
    }
    for (; t < total_pad; ++t) barrier_raw();   // the loaders' padding steps
}

}  // namespace

int choose_ksplit_ws(long long M, int Co, int kpad) {
    const int BN = Co <= 64 ? 64 : 128;
    const long long items = ((M + BM - 1) / BM) * ((Co + BN - 1) / BN);
    const int nslab = kpad / 32;
    int ks = 1;
    while (items * ks < 256 && nslab / (ks * 2) >= 8) ks *= 2;
    return ks;
}

int launch_igemm(const ConvArgs& a, hipStream_t s) {
    const int M = a.N * a.Hq * a.Wq;
    const int BN = (a.Co <= 64) ? 64 : 128;
    if (a.ksplit < 1 || (a.ksplit > 1 && (a.nphase != 1 || !a.partial))) {
        set_error("bad split-K configuration");
        return 1;
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
    // 2 x (A + B) slab ring + tap table = 49 KB used; 84 KB requested so a CU never holds two workgroups
    constexpr int kLds = 84 * 1024;
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_igemm<64>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_igemm<128>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
        attr = true;
    }
    if (BN == 64) hipLaunchKernelGGL(k_igemm<64>, dim3(gx), dim3(512), kLds, s, a, mtiles, ntiles, nitems);
    else hipLaunchKernelGGL(k_igemm<128>, dim3(gx), dim3(512), kLds, s, a, mtiles, ntiles, nitems);
    AVSE_HIP_CHECK(hipGetLastError());
    if (a.ksplit > 1) return launch_splitk_reduce(a, 1, s);
    return 0;
}

}  // namespace avse
