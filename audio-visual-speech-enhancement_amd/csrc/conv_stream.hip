// Persistent, warp-specialised MFMA convolution for the bf16 video encoder layers v_conv2..v_conv5
// (network.py:145-167: Conv2D 'same' -> BatchNorm -> LeakyReLU(0.3) -> MaxPooling2D(2x2)), gfx950.
//
// Design (every choice measured with tools/halo_ablate.hip / tools/stream_ablate.hip at the v_conv2
// bench shape; MFMA work alone runs at ~90% of the bf16 peak, so everything else must hide under it):
//   * 512 threads = 4 compute waves + 4 loader waves, one of each per SIMD (244 VGPRs: two waves fit).
//     Compute waves only read fragments from LDS, issue the MFMAs and run the epilogue; they hold issue
//     priority.  Loader waves do all address arithmetic, global loads and LDS stores.  With one wave per
//     SIMD doing both, that work (~120 instructions per step) did not fit in the MFMA shadow and cost +60%;
//   * each compute wave owns 64 conv pixels x 128 output channels and keeps its 128 accumulators in place
//     for the whole tile: per 32-channel K-slice it reads 4 A + 8 B fragments (12 KB), 25% fewer LDS bytes
//     per FLOP than 8 waves of 64 x 64.  Default (M16): 32 v_mfma_f32_16x16x32_bf16 per slice over 4x4-pixel
//     blocks (the chip holds a higher clock under this shape on random data); option mfma32: 16
//     v_mfma_f32_32x32x16_bf16 over 2 x 4 blocks of 32 x 32 (measured slower);
//   * the workgroup is persistent over tiles; one K-slice per step, one barrier per step;
//   * per step each loader lane issues two 16-byte weight loads (the slice LAT+2 steps ahead) and, on
//     the first HPW taps of a chunk, one 1-KB piece of the input window of the chunk after next, into a
//     ring of LAT register sets, and stores the set loaded LAT steps earlier.  vmcnt retires in issue
//     order, so the input window's HBM latency would stall the weights behind it with a short ring (LAT 4:
//     +14%); register staging costs a few issue cycles where an LDS-DMA (buffer_load ... lds) costs its
//     wave 100-200;
//   * the loader is unrolled over a chunk pair (2 x KS^2 steps), so tap, ring set, weight slot and piece
//     index are compile-time: a wave issues at most one instruction per 4 cycles, and the first loader
//     (runtime tap: piece address, chunk and tile bookkeeping every step, ~185 instructions per step)
//     took ~730 cycles per step against ~600 for the compute wave's 16 MFMAs (s_memtime split, ABL 128);
//   * the input window streams per 32-channel chunk through 3 LDS slots of 64-byte pixel rows: chunk g+2
//     arrives while chunk g computes, across tile boundaries too.
//
// K order per tile: slice = chunk * KS^2 + tap, chunk = 32 input channels (host packing in capi.hip,
// [slice][Cout][32] bf16).  M order: a 32-row MFMA block is 4 x 8 conv pixels; rows 4q..4q+3 are 2x2
// pool window q, and a lane's accumulator registers 4g..4g+3 are four such rows, so BN scale/shift,
// max pool and LeakyReLU happen in registers.
//
// LDS images (bank-conflict free for every tap and all three tile geometries, found and checked by
// exhaustive search over the ds_read_b128 lane groups):
//   halo chunk: pixel (cl, y, x) at row (cl*HH + y)*HW + x, 64 B per row, 16-B slot s holds channels
//               8*(s ^ (y & 3)) .. +8 of the chunk;
//   weights:    row co (0..127) 64 B, slot s holds k 8*(s ^ ((co >> 2) & 3)) .. +8.
// Stores are lane-linear (lane l of a wave writes bytes 16 l of a 1-KB row block), so both swizzles are
// applied on the global SOURCE address.
#include <cstdlib>
#include <type_traits>

#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
constexpr int kOOB = 0x7fffff00;   // buffer offset that reads as zero (past every resource we build)

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16-B slot swizzles of the LDS images (found by exhaustive search over the ds_read_b128 lane groups of
// the v_mfma_f32_32x32x16_bf16 operand layout, every tap offset and all three tile geometries)
// M16 = the v_mfma_f32_16x16x32_bf16 operand layout (lane l: row l & 15, 16-B k-group l >> 4), 4x4-pixel
// fragment blocks: found by the same search (tools/lds_swizzle_search.py)
template <bool M16> __device__ __forceinline__ int wswz(int row) { return M16 ? 2 * ((row >> 2) & 1) : (row >> 2) & 3; }
template <bool M16> __device__ __forceinline__ int hsw(int y) { return M16 ? 2 * (y & 1) : y & 3; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}

// cache-policy bits of the loaders' global loads (gfx950 buffer aux: 1 = sc0, 2 = nt, 16 = sc1), A/B switches
#ifndef AVSE_HALO_AUX
#define AVSE_HALO_AUX 0
#endif
#ifndef AVSE_WGT_AUX
#define AVSE_WGT_AUX 0
#endif
__device__ __forceinline__ i32x4 ld16(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {   // input window pieces
    return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AVSE_HALO_AUX);
}
__device__ __forceinline__ i32x4 ld16w(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {  // weight slices
    return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AVSE_WGT_AUX);
}
__device__ __forceinline__ void st16(char* p, i32x4 v) { *reinterpret_cast<i32x4*>(p) = v; }

// s_waitcnt vmcnt(N) lgkmcnt(0) and a bare s_barrier, as asm with a memory clobber: the compiler may
// not move LDS accesses across them, and adds no vmcnt(0) drain of the loads meant to stay in flight
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }

// LAT (load -> LDS store distance, steps): 10 for 5x5, 6 for 3x3; it divides the unrolled chunk pair
// (2 KS^2 steps).  Measured on v_conv2 (runtime-tap loader): LAT 4 / 5 / 10 / 20 = 1.14 / 1.04-1.13 / 1.00 /
// 1.27 ms (20 spills).
template <int KS, int TH, int TW, int NCLIP, int LAT_ = (KS == 5 ? 10 : 6), int BP_ = 1, bool S16_ = false>
struct StreamGeom {
    static constexpr int HH = TH + KS - 1, HW = TW + KS - 1;
    static constexpr int HPIX = NCLIP * HH * HW;              // halo pixels per chunk
    static constexpr int HPIECES = (HPIX * 64 + 1023) / 1024;  // 1-KB pieces per chunk
    static constexpr int HPW = (HPIECES + 3) / 4;              // pieces per wave per chunk
    static constexpr int NTAP = KS * KS;
    static constexpr int CSLOT = HPIECES * 1024;               // bytes per halo chunk slot
    static constexpr int WSLOT = 8192;                         // one K-slice of 128 co x 32 ci
    // LAT: steps between a load and its LDS write; BP: steps per barrier.  The loader stores slice j + BP + 1
    // during step j (loaded WD = LAT + BP + 1 steps ahead) into a ring of NWS = 2 BP weight slots: the slot
    // it overwrites held slice j + 1 - BP, whose fragments the compute waves read during step j - BP, before
    // the previous barrier; 3 halo chunk slots
    // S16 (split-f16 operands): BP / 2 slice pairs per barrier; during period p the compute waves read the weights of
    // slices BP p .. BP p + BP (one past the period: the next pair's first slice) while the loader stores the BP
    // slices after those: a ring of 2 BP + 1 slots
    // PAIR: loader steps per unrolled iteration (2 chunks; 4 when a period of 4 steps would not divide 2 chunks)
    static constexpr int LAT = LAT_, BP = BP_, NWS = S16_ ? 2 * BP + 1 : 2 * BP, WD = LAT + BP + 1, NHS = 3,
                         PAIR = ((2 * NTAP) % BP ? 4 : 2) * NTAP, CPI = PAIR / NTAP;
    static_assert(PAIR % BP == 0, "barrier periods align with the unrolled loader iteration");
    static_assert(BP == 1 || BP == 2 || (S16_ && BP == 4), "barrier period");
    static_assert(!S16_ || BP % 2 == 0, "split-f16 operands: whole slice pairs per barrier");
    static constexpr int LDS = NHS * CSLOT + NWS * WSLOT;
    static_assert(LDS + 1024 <= 160 * 1024, "LDS");   // one workgroup per CU: ~250 VGPRs x 8 waves fill the register file
    static_assert(NCLIP * TH * TW == 256, "tile = 256 conv pixels (4 waves x 4 fragments)");
    static_assert(PAIR % LAT == 0 && LAT < NTAP, "the ring set of a step is compile-time");
    // chunk g+2's pieces are loaded at taps 0..HPW-1 of chunk g and written LAT steps later, before
    // the first fragment read of chunk g+2 at step NTAP-1 of chunk g+1
    // (a store is visible after the barrier closing its BP-step group: at most BP - 1 steps later)
    // (S16 reads A fragments up to the slice after its period: chunk g+2's first slice is read BP + 1 steps before it)
    static_assert(HPW <= NTAP && HPW - 1 + LAT + BP - 1 <= 2 * NTAP - (S16_ ? BP + 1 : 2), "halo pieces must land in time");
    // loads issued by step j (tap j % NTAP): two weight chunks + one piece on the first HPW taps
    static constexpr int loads(int j, int abl) {
        const int tap = ((j % NTAP) + NTAP) % NTAP;
        return ((abl & 2) ? 0 : 2) + ((!(abl & 1) && tap < HPW) ? 1 : 0);
    }
    // vmcnt bound at the end of step j: the loads of steps j-LAT+2 .. j may stay in flight (the set of
    // step j-LAT+1 is stored by step j+1)
    static constexpr int vm_wait(int j, int abl) {
        int n = 0;
        for (int i = j - LAT + 2; i <= j; ++i) n += loads(i, abl);
        return n;
    }
};

// ABL: ablation mask for tools/stream_ablate.hip only (0 in the library): 1 = no halo pieces in the
// loop, 2 = no weight streaming in the loop, 4 = no barrier/wait, 8 = no fragment reads, 16 = no MFMAs,
// 64 = every tile reads clip 0's window (L2-resident input), 128 = s_memtime per step: cycles working /
// waiting (vmcnt, lgkmcnt) / in the barrier, per wave, into a.prof[(block * 8 + wave) * 4 + {0,1,2, 3=steps}]
//
// S16: fp32-accurate split-f16 operands (DESIGN.md §3 "split-f16").  Every fp32 value x is carried as the f16 pair
// (h, l) = (f16(x), f16(x - h)); the input activation holds, per pixel and per 16 channels, 32 f16 = [h(16) | l(16)]
// (a "chunk" of 32 halves is then 16 real channels), the weight row of output channel co per slice 32 f16 =
// [Bh(16) | Bl(16)] of the same 16 channels (scaled by a per-channel power of two folded into the BN scale).  The
// compute waves take two slices t, t+1 per barrier in three groups of 32 v_mfma_f32_16x16x32_f16 (each MFMA rounds
// its 32 exact products once into the fp32 accumulator):
//   1. A(t) = [Ah | Al] x the Bh half read for every lane (k-group kg & 1)        -> Ah Bh + Al Bh of slice t
//   2. the same for slice t+1
//   3. A' = [Ah(t) | Ah(t+1)] (v_permlane32_swap of the two A fragments: lanes 32..63 take the other slice's Ah) x
//      B' = [Bl(t) | Bl(t+1)] (lanes of k-groups 0, 1 read slice t's Bl half, 2, 3 slice t+1's) -> Ah Bl of both
// i.e. three of the four products of (Ah + Al)(Bh + Bl) — Al Bl (2^-22 of |a b|, below the pieces' representation
// error) is dropped — on 3/4 of the MFMAs of the four-product form.
template <int KS, int TH, int TW, int NCLIP, bool M16 = true, int LAT_ = StreamGeom<KS, TH, TW, NCLIP>::LAT, int ABL = 0,
          int BP_ = 1, bool S16 = false>
__global__ __launch_bounds__(512, 1) void k_conv_stream(HaloArgs a) {
    static_assert(!S16 || M16, "split-f16 operands: 16x16x32 compute waves only");
    using G = StreamGeom<KS, TH, TW, NCLIP, LAT_, BP_, S16>;
    constexpr int HH = G::HH, HW = G::HW, HPIX = G::HPIX, HPW = G::HPW, NTAP = G::NTAP;
    constexpr int CSLOT = G::CSLOT, WSLOT = G::WSLOT, LAT = G::LAT, WD = G::WD, PAIR = G::PAIR;
    constexpr int BP = G::BP, NWS = G::NWS;
    constexpr int BPR = TW / 8, BPC = (TH / 4) * BPR;     // 4x8-pixel blocks (32 MFMA rows) per row / clip
    static_assert(TW % 8 == 0 && TH % 4 == 0 && BPC % 2 == 0, "a wave's two blocks share their y origin mod 4");
    constexpr int PAD = (KS - 1) / 2;

    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const halo = lds;                    // [NHS][CSLOT]
    char* const wring = lds + G::NHS * CSLOT;  // [NWS][WSLOT]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;                    // index within the role

    const int nch = a.Ci / 32;                 // 32-channel chunks per tile (even: host check)
    const int spt = nch * NTAP;                // K-slices per tile (a multiple of 4: 4 | nch)
    const int tiles_x = a.Wc / TW, tiles_y = a.Hc / TH;
    const int tiles_per_clip = tiles_x * tiles_y;
    const int ntiles = ((a.N + NCLIP - 1) / NCLIP) * tiles_per_clip;
    // XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (XCD = linear id % 8), so
    // slot bx % 8 * (gx / 8) + bx / 8 gives each XCD a contiguous run of tiles per round (whole clips): the
    // halo rows neighbouring tiles share are then fetched into that XCD's L2 once
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    const int nchunks = nmine * nch;
    const int co0 = blockIdx.y * 128;
    const long long clip_bytes = (long long)a.Hc * a.Wc * a.Ci * 2;

    auto tile_origin = [&](int k, int& clip0, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip0 = (ABL & 64) ? 0 : (t / tiles_per_clip) * NCLIP;
        const int tt = t % tiles_per_clip;
        oy0 = (tt / tiles_x) * TH;
        ox0 = (tt % tiles_x) * TW;
    };

    if (wave >= 4) {
        // =============================== loader waves ===============================
        // weights: loader w stores bytes [2048 w, 2048 w + 2048) of a slot: rows 32w + 16u + lane/4
        const __amdgpu_buffer_rsrc_t wrs = make_rsrc(reinterpret_cast<const char*>(a.w) + (size_t)co0 * 64,
                                                     (long long)spt * a.Co * 64 - (long long)co0 * 64);
        const int wslice = a.Co * 64, wend = spt * wslice;
        int wvoff[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = 32 * w + 16 * u + (lane >> 2), sl = lane & 3;
            wvoff[u] = row * 64 + ((sl ^ wswz<M16>(row)) << 4);
        }
        char* const wdst = wring + 2048 * w + lane * 16;   // + slot * WSLOT + 1024 u
        auto tile_rsrc = [&](int clip0) {
            return make_rsrc(reinterpret_cast<const char*>(a.in) + (long long)clip0 * clip_bytes,
                             (long long)(a.N - clip0) * clip_bytes);
        };
        // piece pc of this loader is P = w + 4 pc (1-KB rows P*1024 .. of a halo slot; lane: 16 B of pixel
        // P*16 + lane/4).  Its source offset in the tile at (oy0, ox0) for chunk 0, or kOOB (reads zero)
        // outside the image / past the window — computed once per tile
        const int ci2 = a.Ci * 2, hc = a.Hc, wc = a.Wc;
        auto tile_voffs = [&](int oy0, int ox0, int (&vo)[HPW]) {
#pragma unroll
            for (int pc = 0; pc < HPW; ++pc) {
                const int P = w + 4 * pc;
                const int p = P * 16 + (lane >> 2), sl = lane & 3;
                const int cl = p / (HH * HW), rr = p - cl * (HH * HW);
                const int y = rr / HW, x = rr - y * HW;
                const int iy = oy0 + y - PAD, ix = ox0 + x - PAD;
                const int off = ((cl * hc + iy) * wc + ix) * ci2 + ((sl ^ hsw<M16>(y)) << 4);
                const bool ok = (P < G::HPIECES) & (p < HPIX) & ((unsigned)iy < (unsigned)hc) & ((unsigned)ix < (unsigned)wc);
                vo[pc] = ok ? off : kOOB;
            }
        };
        // a piece row past the chunk (P >= HPIECES: only for the last pc of some waves) is not stored
        auto piece_store = [&](auto pcc, char* base, i32x4 v) {
            constexpr int pc = decltype(pcc)::value;
            if constexpr (4 * pc + 3 < G::HPIECES) st16(base + pc * 4096, v);
            else if (w + 4 * pc < G::HPIECES) st16(base + pc * 4096, v);
        };

        // tiles: k (chunks being computed), k + 1 (chunk g+2 may belong to it)
        int cur_clip0, cur_oy0, cur_ox0, nxt_clip0, nxt_oy0, nxt_ox0;
        tile_origin(0, cur_clip0, cur_oy0, cur_ox0);
        tile_origin(1, nxt_clip0, nxt_oy0, nxt_ox0);
        __amdgpu_buffer_rsrc_t cur_rs = tile_rsrc(cur_clip0), nxt_rs = tile_rsrc(nxt_clip0);
        int vo_cur[HPW], vo_nxt[HPW];
        tile_voffs(cur_oy0, cur_ox0, vo_cur);
        tile_voffs(nxt_oy0, nxt_ox0, vo_nxt);
        char* const pbase0 = halo + w * 1024 + lane * 16;   // + slot * CSLOT + pc * 4096

        // prologue: chunk 0 and the pieces of chunk 1 that no virtual step -LAT..-1 loads, weight slices
        // 0, 1 straight to LDS; the sets of the virtual steps (weights of slices 2 .. LAT+1, pieces of chunk
        // 1 on taps NTAP-LAT ..) into the register ring — steps 0 .. LAT-1 store them
        [&]<int... PC>(std::integer_sequence<int, PC...>) {
            (piece_store(std::integral_constant<int, PC>{}, pbase0, ld16(cur_rs, vo_cur[PC], 0)), ...);
            ((PC < NTAP - LAT ? piece_store(std::integral_constant<int, PC>{}, pbase0 + CSLOT, ld16(cur_rs, vo_cur[PC], 64))
                              : (void)0), ...);
        }(std::make_integer_sequence<int, HPW>{});
#pragma unroll
        for (int s = 0; s <= BP; ++s)
#pragma unroll
            for (int u = 0; u < 2; ++u) st16(wdst + s * WSLOT + 1024 * u, ld16w(wrs, wvoff[u], (s % spt) * wslice));
        i32x4 rw[LAT][2], rp[LAT];
        [&]<int... S>(std::integer_sequence<int, S...>) {
            ([&] {
                 rw[S][0] = ld16w(wrs, wvoff[0], ((S + BP + 1) % spt) * wslice);
                 rw[S][1] = ld16w(wrs, wvoff[1], ((S + BP + 1) % spt) * wslice);
                 constexpr int vt = NTAP - LAT + S;   // tap of virtual step S - LAT
                 if constexpr (vt < HPW && !(ABL & 1)) rp[S] = ld16(cur_rs, vo_cur[vt < HPW ? vt : 0], 64);
             }(), ...);
        }(std::make_integer_sequence<int, LAT>{});
        wait_vm_lgkm0<0>();
        barrier_raw();
        barrier_raw();   // the compute waves have read slice 0 (weight slot 0 is overwritten at step 0)

        // per-chunk state of chunk g = k * nch + c: its pieces load chunk g+2 from (prs, vsel[], psoff) and
        // land at pd_cur; pd_prev = where the pieces loaded during chunk g-1 land
        int k = 0, c = 0, g = 0, hs2 = 2;           // hs2 = halo slot of chunk g+2
        int woff = (WD % spt) * wslice;             // weights loaded by the next step: slice step + WD
        // (first step of this chunk pair) % NWS: constant 0 unless the pair length is not a multiple of the ring
        constexpr bool kRot = PAIR % NWS != 0;
        int wrot = 0;
        int vsel[HPW];
        __amdgpu_buffer_rsrc_t prs = cur_rs;
        int psoff = 0;
        char* pd_cur = pbase0 + CSLOT;              // virtual steps' pieces: chunk 1
        char* pd_prev = pd_cur;
        unsigned long long ptp = (ABL & 128) ? __builtin_amdgcn_s_memtime() : 0, pt0 = 0, pt1 = 0, p_work = 0,
                           p_wait = 0, p_bar = 0;
        auto chunk_begin = [&]() {
            const bool nx = c + 2 >= nch;
            const bool real = g + 2 < nchunks;
#pragma unroll
            for (int pc = 0; pc < HPW; ++pc) vsel[pc] = !real ? kOOB : nx ? vo_nxt[pc] : vo_cur[pc];
            prs = nx ? nxt_rs : cur_rs;
            psoff = (nx ? c + 2 - nch : c + 2) * 64;
            pd_prev = pd_cur;
            pd_cur = pbase0 + hs2 * CSLOT;
        };
        auto chunk_end = [&]() {
            ++g;
            hs2 = hs2 == 2 ? 0 : hs2 + 1;
            if (++c == nch) {
                c = 0;
                ++k;
                cur_oy0 = nxt_oy0;
                cur_ox0 = nxt_ox0;
                cur_rs = nxt_rs;
#pragma unroll
                for (int pc = 0; pc < HPW; ++pc) vo_cur[pc] = vo_nxt[pc];
                tile_origin(k + 1, nxt_clip0, nxt_oy0, nxt_ox0);
                nxt_rs = tile_rsrc(nxt_clip0);
                tile_voffs(nxt_oy0, nxt_ox0, vo_nxt);
            }
        };
        // step j of a chunk pair (compile-time): tap j % NTAP, ring set j % LAT, weight slot j & 1
        auto lstep = [&](auto jidx) {
            constexpr int j = decltype(jidx)::value;
            constexpr int tap = j % NTAP, S = j % LAT;
            constexpr int jl = j - LAT;                                 // the step that loaded set S
            constexpr int tl = ((jl % NTAP) + NTAP) % NTAP;
            constexpr bool lprev = (jl < 0) || (jl / NTAP != j / NTAP);  // ... during the previous chunk
            if constexpr (tap == 0) chunk_begin();
            // 1. LDS stores of set S: weights of slice j+BP+1 (slot (j+BP+1) % NWS) and the piece loaded
            //    with them
            if constexpr (!(ABL & 2)) {
                int wsl = (j + BP + 1) % NWS + (kRot ? wrot : 0);
                if (wsl >= NWS) wsl -= NWS;
                char* const wd = wdst + wsl * WSLOT;
                st16(wd, rw[S][0]);
                st16(wd + 1024, rw[S][1]);
            }
            if constexpr (tl < HPW && !(ABL & 1))
                piece_store(std::integral_constant<int, (tl < HPW ? tl : 0)>{}, lprev ? pd_prev : pd_cur, rp[S]);
            // 2. this step's loads
            if constexpr (!(ABL & 2)) {
                rw[S][0] = ld16w(wrs, wvoff[0], woff);
                rw[S][1] = ld16w(wrs, wvoff[1], woff);
            }
            if constexpr (tap < HPW && !(ABL & 1)) rp[S] = ld16(prs, vsel[tap < HPW ? tap : 0], psoff);
            woff += wslice;
            if (woff == wend) woff = 0;
            // 3. at the end of a BP-step group: the set of step j-LAT+1 has landed (stored by step j+1);
            //    the group's stores are visible after the barrier
            if constexpr (!(ABL & 4) && j % BP == BP - 1) {
                if constexpr ((ABL & 128) != 0) pt0 = __builtin_amdgcn_s_memtime();
                wait_vm_lgkm0<G::vm_wait(j, ABL)>();
                if constexpr ((ABL & 128) != 0) pt1 = __builtin_amdgcn_s_memtime();
                barrier_raw();
                if constexpr ((ABL & 128) != 0) {
                    const unsigned long long pt2 = __builtin_amdgcn_s_memtime();
                    p_work += pt0 - ptp;
                    p_wait += pt1 - pt0;
                    p_bar += pt2 - pt1;
                    ptp = pt2;
                }
            }
            if constexpr (tap == NTAP - 1) chunk_end();
        };
        for (int pr = 0; pr < nchunks; pr += G::CPI) {   // nchunks % CPI == 0 (launch_stream)
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (lstep(std::integral_constant<int, J>{}), ...);
            }(std::make_integer_sequence<int, PAIR>{});
            if constexpr (kRot) wrot = (wrot + PAIR) % NWS;
        }
        wait_vm_lgkm0<0>();   // loads still in flight target registers and rows nobody reads
        if constexpr ((ABL & 128) != 0)
            if (lane == 0) {
                unsigned long long* pr = a.prof + ((size_t)blockIdx.x * 8 + wave) * 4;
                pr[0] = p_work; pr[1] = p_wait; pr[2] = p_bar; pr[3] = (unsigned long long)nchunks * NTAP;
            }
        return;
    }

    // =============================== compute waves ===============================
    // the MFMA stream gets issue priority over the co-resident loader wave of its SIMD (-2% time)
    __builtin_amdgcn_s_setprio(2);
    if constexpr (M16) {
        // v_mfma_f32_16x16x32_bf16 (lane l: row / column l & 15, channels 8 (l >> 4) .. +8 of the slice): on
        // random data the chip holds a higher clock under this shape than under 32x32x16 at equal cycles per
        // FLOP (MI355X_MICROARCH.md, DVFS item 7).  Wave w owns 4 fragment blocks of 4x4 conv pixels (blocks
        // 4w .. 4w+3 of the tile, row-major per clip) x 128 output channels (8 blocks of 16): per K-slice
        // 4 A + 8 B fragment reads (12 KB, as before) for 32 MFMAs.  Block row r = 4 q + 2 dy + dx is pixel
        // (2 (q >> 1) + dy, 2 (q & 1) + dx): a lane's 4 accumulator rows 4 (l >> 4) .. +3 are pool window l >> 4.
        constexpr int SBX = TW / 4, SB = (TH / 4) * SBX;   // 4x4 blocks per row / clip
        static_assert(TH % 4 == 0 && TW % 4 == 0 && (SBX % 4 == 0 || SBX == 2) && SB % 4 == 0, "block geometry");
        const int r16 = lane & 15, kg = lane >> 4;
        const int q = r16 >> 2, dy = (r16 >> 1) & 1, dx = r16 & 1;
        const int b0 = 4 * w, cl0 = b0 / SB, bb0 = b0 % SB;
        const int by0 = bb0 / SBX, bx0 = bb0 % SBX;
        const int ab = ((cl0 * HH + 4 * by0 + 2 * (q >> 1) + dy) * HW + 4 * bx0 + 2 * (q & 1) + dx) * 64;
        // block i of the wave relative to block 0 (bx0 % SBX == 0 or SBX == 2 with bx0 == 0)
        auto boff_of = [](int i) { return ((i / SBX) * 4 * HW + (i % SBX) * 4) * 64; };
        // + 1024 j for column block j.  S16: bo16 reads the Bh half of the row for every lane (k-group kg & 1), bo16l
        // the Bl half (2 + (kg & 1)); the per-16-lane address pattern is the bf16 one (same conflict-free image)
        const int bo16 = r16 * 64 + (((S16 ? (kg & 1) : kg) ^ wswz<true>(r16)) << 4);
        const int bo16l = r16 * 64 + (((2 + (kg & 1)) ^ wswz<true>(r16)) << 4);
        // ABL & 256 (harness only): B fragments of column blocks 4..7 reuse blocks 0..3 (the LDS fragment reads per MFMA of
        // a 128 x 128 wave tile; results meaningless)
        auto frags_lo = [&](int ws, i32x4 (&fb)[8]) {
            const char* wp = wring + ws * WSLOT + bo16l;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                fb[j] = ((ABL & 256) && j >= 4) ? fb[j - 4] : *reinterpret_cast<const i32x4*>(wp + 1024 * j);
        };
        auto frags = [&](int hs, int tap, int ws, i32x4 (&fa)[4], i32x4 (&fb)[8]) {
            const int ky = tap / KS, kx = tap % KS;
            const int pos = (kg ^ hsw<true>(dy + ky)) << 4;
            const char* hp = halo + hs * CSLOT + ab + (ky * HW + kx) * 64 + pos;
            const char* wp = wring + ws * WSLOT + bo16;
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const i32x4*>(hp + boff_of(i));
#pragma unroll
            for (int j = 0; j < 8; ++j)
                fb[j] = ((ABL & 256) && j >= 4) ? fb[j - 4] : *reinterpret_cast<const i32x4*>(wp + 1024 * j);
        };
        // BN scale / shift of this column block in LDS (past the rings), read in the epilogue: 16 VGPRs held
        // for the whole tile would spill the 256-register budget (128 accumulators + 2 x 12 fragments)
        float* const ssh = reinterpret_cast<float*>(lds + G::LDS);
        if (w == 0) {
            ssh[lane] = a.scale[co0 + lane];
            ssh[lane + 64] = a.scale[co0 + 64 + lane];
            ssh[128 + lane] = a.shift[co0 + lane];
            ssh[192 + lane] = a.shift[co0 + 64 + lane];
        }
        barrier_raw();   // the loaders' prologue (and ssh: the compute waves' LDS stores are drained by the
                         // lgkmcnt(0) wait before the next barrier, which precedes any epilogue)

        f32x4 acc[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){};
        const int Wp = a.Wc / 2;
        // output element (pooled pixel p, channel co): OUT_BF16 / OUT_F32 at p * out_pix_stride + out_c_off + co;
        // OUT_S16 (the next stream layer's split input, out_pix_stride = 2 Co) h at p * out_pix_stride + out_c_off +
        // 32 (co / 16) + co % 16 and l 16 halves further
        bool range_bad = false;   // OUT_S16: range guard over all tiles (avse_common.h pair_out_of_range), reported once
        auto epilogue_m = [&](auto modec, int clip0, int oy0, int ox0) {
            constexpr int OM = decltype(modec)::value;
            constexpr int ES = OM == OUT_F32 ? 4 : 2;
            const long long cbytes = a.out_clip_stride * ES;
            const __amdgpu_buffer_rsrc_t ors = make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip0 * cbytes,
                                                         (long long)(a.N - clip0) * cbytes);
            const int cbase = cl0 * (int)a.out_clip_stride + a.out_c_off + (OM == OUT_S16 ? 2 * co0 : co0) + r16;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int py = (oy0 + 4 * (by0 + i / SBX)) / 2 + (kg >> 1);
                const int px = (ox0 + 4 * (bx0 + i % SBX)) / 2 + (kg & 1);
                const int pbase = cbase + (py * Wp + px) * a.out_pix_stride;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float mx = fmaxf(fmaxf(acc[i][j][0], acc[i][j][1]), fmaxf(acc[i][j][2], acc[i][j][3]));
                    float x = fmaf(mx, ssh[16 * j + r16], ssh[128 + 16 * j + r16]);
                    x = fmaxf(x, LRELU * x);
                    if constexpr (OM == OUT_BF16) {
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)x), ors,
                                                              (pbase + 16 * j) * 2, 0, 0);
                    } else if constexpr (OM == OUT_S16) {
                        const _Float16 h = (_Float16)x;
                        const _Float16 l = (_Float16)(x - (float)h);
                        range_bad |= pair_out_of_range(x);
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ors,
                                                              (pbase + 32 * j) * 2, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, l), ors,
                                                              (pbase + 32 * j + 16) * 2, 0, 0);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, x), ors, (pbase + 16 * j) * 4, 0, 0);
                    }
                    // restart the chain in place: x * 0 (not a constant, which the register allocator would
                    // materialise elsewhere and then shuffle — that spilled the 256-register budget)
                    acc[i][j] *= 0.f;
                }
            }
        };
        auto epilogue = [&](int clip0, int oy0, int ox0) {
            if constexpr (!S16) {
                epilogue_m(std::integral_constant<int, OUT_BF16>{}, clip0, oy0, ox0);
            } else if (a.out_mode == OUT_S16) {
                epilogue_m(std::integral_constant<int, OUT_S16>{}, clip0, oy0, ox0);
            } else {
                epilogue_m(std::integral_constant<int, OUT_F32>{}, clip0, oy0, ox0);
            }
        };

        unsigned long long ptp = (ABL & 128) ? __builtin_amdgcn_s_memtime() : 0, pt0 = 0, pt1 = 0, p_work = 0,
                           p_wait = 0, p_bar = 0;
        int tap1 = 1, hs1 = 0;
        i32x4 fa[4], fb[8], na[4], nb[8];
        frags(0, 0, 0, fa, fb);
        if constexpr ((ABL & 8) != 0) frags(0, 0, 0, na, nb);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // slice 0 read: the loaders may now overwrite weight slot 0

        // bar: the step closes a BP-step group (t % BP == BP - 1; t is even on the first call of each pair)
        auto cstep = [&](auto bar, int t, i32x4 (&ca)[4], i32x4 (&cb)[8], i32x4 (&xa)[4], i32x4 (&xb)[8]) {
            if constexpr (!S16) {   // (split-f16 operands run pstep below)
                if constexpr (!(ABL & 8)) frags(hs1, tap1, (t + 1) & (NWS - 1), xa, xb);
                if constexpr (!(ABL & 16))
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8, ca[i]), __builtin_bit_cast(bf16x8, cb[j]), acc[i][j], 0, 0, 0);
            }
            // the next slice's 12 fragment reads one per MFMA from the start of the step (measured against two
            // MFMAs per read over 24 MFMAs, 3:2, 1:2 and all reads first: -1 to -2 % on v_conv2 / v_conv4, the
            // bunched forms +2 to +17 %).  A 3-slot weight ring that lets the compute waves skip the lgkmcnt(0)
            // drain before each barrier was slower (+2-4 %): the drain overlaps the barrier wait, the deferred
            // wait stalls the next step's first MFMAs
            if constexpr (!S16) {
#pragma unroll
                for (int r = 0; r < 12; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 20, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (!(ABL & 4) && decltype(bar)::value) {
                if constexpr ((ABL & 128) != 0) pt0 = __builtin_amdgcn_s_memtime();
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if constexpr ((ABL & 128) != 0) pt1 = __builtin_amdgcn_s_memtime();
                barrier_raw();
                if constexpr ((ABL & 128) != 0) {
                    const unsigned long long pt2 = __builtin_amdgcn_s_memtime();
                    p_work += pt0 - ptp;
                    p_wait += pt1 - pt0;
                    p_bar += pt2 - pt1;
                    ptp = pt2;
                }
            }
            if (++tap1 == NTAP) {
                tap1 = 0;
                hs1 = hs1 == 2 ? 0 : hs1 + 1;
            }
        };
        int t = 0;
        int cur_clip0, cur_oy0, cur_ox0;
        if constexpr (S16) {
            auto advance = [&]() {
                if (++tap1 == NTAP) {
                    tap1 = 0;
                    hs1 = hs1 == 2 ? 0 : hs1 + 1;
                }
            };
            auto mfma_group = [&](const i32x4 (&ca)[4], const i32x4 (&cb)[8]) {
                if constexpr (!(ABL & 16))
#pragma unroll
                    for (int j = 0; j < 8; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                __builtin_bit_cast(f16x8, ca[i]), __builtin_bit_cast(f16x8, cb[j]), acc[i][j], 0, 0, 0);
            };
            auto sched = [](auto nds, auto per) {
                constexpr int ND = decltype(nds)::value, PER = decltype(per)::value;
#pragma unroll
                for (int r = 0; r < ND; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // DS read
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 32 - ND * PER, 0);
                __builtin_amdgcn_sched_barrier(0);
            };
            const bool hi_half = kg >= 2;   // group 3's B': lanes of k-groups 2, 3 read slice t+1's Bl half
            // slices t, t+1 with (a0, b0) = A(t), Bh(t) in registers; reads A(t+2), Bh(t+2) into (na, nb); bar: the
            // pair closes a BP-slice period
            auto pstep = [&](auto bar, int t, i32x4 (&a0)[4], i32x4 (&b0)[8], i32x4 (&na)[4], i32x4 (&nb)[8]) {
                i32x4 a1[4], b1[8], bp[8];
                const int ws0 = t % NWS, ws1 = (t + 1) % NWS, ws2 = (t + 2) % NWS;
                if constexpr (!(ABL & 8)) frags(hs1, tap1, ws1, a1, b1);
                advance();
                mfma_group(a0, b0);
                sched(std::integral_constant<int, 12>{}, std::integral_constant<int, 1>{});
                if constexpr (!(ABL & 8)) frags_lo(hi_half ? ws1 : ws0, bp);
                mfma_group(a1, b1);
                sched(std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{});
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        a0[i][d] = (int)__builtin_amdgcn_permlane32_swap((unsigned)a0[i][d], (unsigned)a1[i][d], false,
                                                                         false)[0];
                if constexpr (!(ABL & 8)) frags(hs1, tap1, ws2, na, nb);
                advance();
                mfma_group(a0, bp);
                sched(std::integral_constant<int, 12>{}, std::integral_constant<int, 1>{});
                if constexpr (!(ABL & 4) && decltype(bar)::value) {
                    if constexpr ((ABL & 128) != 0) pt0 = __builtin_amdgcn_s_memtime();
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if constexpr ((ABL & 128) != 0) pt1 = __builtin_amdgcn_s_memtime();
                    barrier_raw();
                    if constexpr ((ABL & 128) != 0) {
                        const unsigned long long pt2 = __builtin_amdgcn_s_memtime();
                        p_work += pt0 - ptp;
                        p_wait += pt1 - pt0;
                        p_bar += pt2 - pt1;
                        ptp = pt2;
                    }
                }
            };
            for (int kt = 0; kt < nmine; ++kt) {
                for (int s = 0; s < spt; s += 4, t += 4) {   // spt % 4 == 0 (launch_stream)
                    pstep(std::bool_constant<BP == 2>{}, t, fa, fb, na, nb);
                    pstep(std::true_type{}, t + 2, na, nb, fa, fb);
                }
                tile_origin(kt, cur_clip0, cur_oy0, cur_ox0);
                epilogue(cur_clip0, cur_oy0, cur_ox0);
            }
        } else {
            for (int kt = 0; kt < nmine; ++kt) {
                for (int s = 0; s < spt; s += 2, t += 2) {
                    cstep(std::bool_constant<BP == 1>{}, t, fa, fb, na, nb);
                    cstep(std::true_type{}, t + 1, na, nb, fa, fb);
                }
                tile_origin(kt, cur_clip0, cur_oy0, cur_ox0);
                epilogue(cur_clip0, cur_oy0, cur_ox0);
            }
        }
        if constexpr ((ABL & 128) != 0)
            if (lane == 0) {
                unsigned long long* pr = a.prof + ((size_t)blockIdx.x * 8 + wave) * 4;
                pr[0] = p_work; pr[1] = p_wait; pr[2] = p_bar; pr[3] = (unsigned long long)t;
            }
        if constexpr (S16) range_report(a.range_flag, a.range_bit, range_bad);
        return;
    }
    // fragment geometry (v_mfma_f32_32x32x16_bf16: lane l holds row/column l & 31 and k-half hi = l >> 5).
    // Wave w owns blocks 2w, 2w+1; block row r = 4 q + 2 dy + dx is pixel (2 (q >> 2) + dy, 2 (q & 3) + dx)
    // of the block: rows 4q..4q+3 are 2x2 pool window q
    const int r32 = lane & 31, hi = lane >> 5;
    int ab;   // halo byte offset of this lane's pixel at tap (0,0) in block 0
    {
        const int b = 2 * w;
        const int cl = b / BPC, bb = b % BPC;
        const int q = r32 >> 2;
        const int y = 4 * (bb / BPR) + 2 * (q >> 2) + ((r32 >> 1) & 1);
        const int x = 8 * (bb % BPR) + 2 * (q & 3) + (r32 & 1);
        ab = ((cl * HH + y) * HW + x) * 64;
    }
    constexpr int blk1 = ((4 * (1 / BPR)) * HW + 8 * (1 % BPR)) * 64;   // block 2w+1 relative to block 2w
    const int ylo = 2 * ((r32 >> 4) & 1) + ((r32 >> 1) & 1);          // this lane's pixel y mod 4
    int boffm[2];                                                      // + 2048 jb for column block jb
#pragma unroll
    for (int m = 0; m < 2; ++m) boffm[m] = r32 * 64 + (((2 * m + hi) ^ wswz<M16>(r32)) << 4);
    // fragments of K-slice (chunk slot hs, tap) with weights in ring slot ws: fa[2 i + m] = block i,
    // channels 16 m .. 16 m + 15 of the slice; fb[2 jb + m] = output channels 32 jb .., same channels
    auto frags = [&](int hs, int tap, int ws, i32x4 (&fa)[4], i32x4 (&fb)[8]) {
        const int ky = tap / KS, kx = tap % KS;
        const int sw = hsw<M16>(ylo + ky);
        const char* hp = halo + hs * CSLOT + ab + (ky * HW + kx) * 64;
        const char* wp = wring + ws * WSLOT;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int pos = ((2 * m + hi) ^ sw) << 4;
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[2 * i + m] = *reinterpret_cast<const i32x4*>(hp + i * blk1 + pos);
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) fb[2 * jb + m] = *reinterpret_cast<const i32x4*>(wp + boffm[m] + 2048 * jb);
        }
    };
    float sc[4], sh[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        sc[jb] = a.scale[co0 + 32 * jb + r32];
        sh[jb] = a.shift[co0 + 32 * jb + r32];
    }
    barrier_raw();   // the loaders' prologue

    // never assigned a constant: a tile's first step accumulates onto the MFMA's inline zero instead,
    // so the register allocator keeps each accumulator in place across the whole MFMA chain
    f32x16 acc[2][4];
    const int Wp = a.Wc / 2;
    // scale >= 0 (host sign fold), so pooling the raw accumulators then one FMA equals BN-then-pool
    // exactly; LeakyReLU(0.3) = max(x, 0.3 x); 32-bit offsets into a buffer resource over the tile's
    // clips (stores past the last clip of a ragged 4-clip tile fall outside it and are dropped).
    // Accumulator register 4g + e of block i, column block jb = row 8g + 4 hi + e = pool window 2g + hi.
    auto epilogue = [&](int clip0, int oy0, int ox0) {
        const long long cb = a.out_clip_stride * 2;
        const __amdgpu_buffer_rsrc_t ors =
            make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip0 * cb, (long long)(a.N - clip0) * cb);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int b = 2 * w + i;
            const int cl = b / BPC, bb = b % BPC;
            const int py0 = (oy0 + 4 * (bb / BPR)) / 2, px0 = (ox0 + 8 * (bb % BPR)) / 2;
            const int cbase = cl * (int)a.out_clip_stride + a.out_c_off + co0;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const int co = 32 * jb + r32;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int q = 2 * g + hi;
                    const int py = py0 + (q >> 2), px = px0 + (q & 3);
                    const float mx = fmaxf(fmaxf(acc[i][jb][4 * g], acc[i][jb][4 * g + 1]),
                                           fmaxf(acc[i][jb][4 * g + 2], acc[i][jb][4 * g + 3]));
                    float x = fmaf(mx, sc[jb], sh[jb]);
                    x = fmaxf(x, LRELU * x);
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16_t)x), ors,
                                                          (cbase + (py * Wp + px) * a.out_pix_stride + co) * 2, 0, 0);
                }
            }
        }
    };

    unsigned long long ptp = (ABL & 128) ? __builtin_amdgcn_s_memtime() : 0, pt0 = 0, pt1 = 0, p_work = 0, p_wait = 0,
                       p_bar = 0;
    // next slice (tap1 of the chunk in halo slot hs1)
    int tap1 = 1, hs1 = 0;
    i32x4 fa[4], fb[8], na[4], nb[8];
    frags(0, 0, 0, fa, fb);
    if constexpr ((ABL & 8) != 0) frags(0, 0, 0, na, nb);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();   // slice 0 read: the loaders may now overwrite weight slot 0

    // first: the tile's first step (accumulate onto zero); bar: the step closes a BP-step group
    auto cstep = [&](auto first, auto bar, int t, i32x4 (&ca)[4], i32x4 (&cb)[8], i32x4 (&xa)[4], i32x4 (&xb)[8]) {
        // fragments of the next slice (weights in ring slot (t+1) % NWS), interleaved with the 16 MFMAs
        if constexpr (!(ABL & 8)) frags(hs1, tap1, (t + 1) & (NWS - 1), xa, xb);
        if constexpr (!(ABL & 16))
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb)
                        acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                            __builtin_bit_cast(bf16x8, ca[2 * i + m]), __builtin_bit_cast(bf16x8, cb[2 * jb + m]),
                            (decltype(first)::value && m == 0) ? (f32x16){} : acc[i][jb], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(ABL & 4) && decltype(bar)::value) {
            if constexpr ((ABL & 128) != 0) pt0 = __builtin_amdgcn_s_memtime();
            // LDS reads only: the epilogue's global stores (vmcnt on gfx9) are never waited for
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr ((ABL & 128) != 0) pt1 = __builtin_amdgcn_s_memtime();
            barrier_raw();
            if constexpr ((ABL & 128) != 0) {
                const unsigned long long pt2 = __builtin_amdgcn_s_memtime();
                p_work += pt0 - ptp;
                p_wait += pt1 - pt0;
                p_bar += pt2 - pt1;
                ptp = pt2;
            }
        }
        if (++tap1 == NTAP) {
            tap1 = 0;
            hs1 = hs1 == 2 ? 0 : hs1 + 1;
        }
    };
    int t = 0;
    int cur_clip0, cur_oy0, cur_ox0;
    using BAR0 = std::bool_constant<BP == 1>;
    for (int kt = 0; kt < nmine; ++kt) {
        cstep(std::true_type{}, BAR0{}, t, fa, fb, na, nb);
        cstep(std::false_type{}, std::true_type{}, t + 1, na, nb, fa, fb);
        t += 2;
        for (int s = 2; s < spt; s += 2, t += 2) {
            cstep(std::false_type{}, BAR0{}, t, fa, fb, na, nb);
            cstep(std::false_type{}, std::true_type{}, t + 1, na, nb, fa, fb);
        }
        tile_origin(kt, cur_clip0, cur_oy0, cur_ox0);
        epilogue(cur_clip0, cur_oy0, cur_ox0);
    }
    if constexpr ((ABL & 128) != 0)
        if (lane == 0) {
            unsigned long long* pr = a.prof + ((size_t)blockIdx.x * 8 + wave) * 4;
            pr[0] = p_work; pr[1] = p_wait; pr[2] = p_bar; pr[3] = (unsigned long long)t;
        }
}

// split-f16: two slice pairs per barrier (a 9-slot weight ring fits beside the 3 halo slots; v_conv2 3.64 -> 3.49 ms).
// The 3x3 layers' halo pieces land in time at BP 4 only with LAT 4 (a split step is ~3x a bf16 step, so 4 steps still
// cover the load latency): v_conv3 / v_conv4 / v_conv5 0.688 / 0.337 / 0.170 -> 0.665 / 0.324 / 0.165 ms
#ifndef AVSE_S16_BP5
#define AVSE_S16_BP5 4
#endif
#ifndef AVSE_S16_BP3
#define AVSE_S16_BP3 4
#endif
#ifndef AVSE_S16_LAT3
#define AVSE_S16_LAT3 4
#endif
template <int KS, int TH, int TW, int NCLIP, bool M16, bool S16 = false>
int launch_stream(const HaloArgs& a, hipStream_t s) {
    constexpr int BP = S16 ? (KS == 5 ? AVSE_S16_BP5 : AVSE_S16_BP3) : 1;
    constexpr int LAT = (S16 && KS == 3) ? AVSE_S16_LAT3 : StreamGeom<KS, TH, TW, NCLIP>::LAT;
    using G = StreamGeom<KS, TH, TW, NCLIP, LAT, BP, S16>;
    constexpr auto kern = k_conv_stream<KS, TH, TW, NCLIP, M16, G::LAT, 0, BP, S16>;
    if (int rc = ensure_lds_attr((const void*)kern, G::LDS + 1024)) return rc;
    if (a.Hc % TH || a.Wc % TW || a.Co % 128 || a.Ci % 64) {   // an even number of 32-channel chunks
        set_error("stream conv: tile does not divide the layer");
        return 3;
    }
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = ((a.N + NCLIP - 1) / NCLIP) * (a.Hc / TH) * (a.Wc / TW);
    const int cob = a.Co / 128;
    // one workgroup per CU; gx a multiple of 8 keeps a tile's co-blocks on one XCD (shared L2 window)
    int gx = ncu / cob;
    gx = gx >= 8 ? gx / 8 * 8 : (gx < 1 ? 1 : gx);
    if (gx > tiles) gx = tiles;
    if ((a.Ci / 32) % G::CPI || (S16 && ((a.out_mode != OUT_S16 && a.out_mode != OUT_F32) || (a.Ci / 32 * KS * KS) % 4))) {
        set_error("stream conv: split-f16 operands write split or f32 outputs, over slice counts divisible by 4");
        return 3;
    }
    hipLaunchKernelGGL(kern, dim3(gx, cob), dim3(512), G::LDS + 1024, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

int launch_conv_stream(const HaloArgs& a, hipStream_t s) {
    const bool m32 = a.mfma32 != 0;   // v_mfma_f32_32x32x16_bf16 compute waves (A/B variant, Options::mfma32)
    if (a.split) {   // split-f16 operands (a.Ci counts halves: 2 x the layer's channels)
        switch (a.variant) {
            case HALO_K5: return launch_stream<5, 16, 16, 1, true, true>(a, s);
            case HALO_K3_16: return launch_stream<3, 16, 16, 1, true, true>(a, s);
            case HALO_K3_8: return launch_stream<3, 8, 8, 4, true, true>(a, s);
        }
        set_error("stream conv: unsupported variant");
        return 3;
    }
    switch (a.variant) {
        case HALO_K5: return m32 ? launch_stream<5, 16, 16, 1, false>(a, s) : launch_stream<5, 16, 16, 1, true>(a, s);
        case HALO_K3_16: return m32 ? launch_stream<3, 16, 16, 1, false>(a, s) : launch_stream<3, 16, 16, 1, true>(a, s);
        case HALO_K3_8: return m32 ? launch_stream<3, 8, 8, 4, false>(a, s) : launch_stream<3, 8, 8, 4, true>(a, s);
    }
    set_error("stream conv: unsupported variant");
    return 3;
}

}  // namespace avse
