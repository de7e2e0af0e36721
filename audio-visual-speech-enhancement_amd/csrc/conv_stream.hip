// Persistent, warp-specialised MFMA convolution for the bf16 video encoder layers v_conv2..v_conv5
// (network.py:145-167: Conv2D 'same' -> BatchNorm -> LeakyReLU(0.3) -> MaxPooling2D(2x2)), gfx950.
//
// Design (every choice measured with tools/halo_ablate.hip / tools/stream_ablate.hip at the v_conv2
// bench shape; MFMA work alone runs at ~90% of the bf16 peak, so everything else must hide under it):
//   * 512 threads = 4 compute waves + 4 loader waves, one of each per SIMD (244 VGPRs: two waves fit).
//     Compute waves only read fragments from LDS, issue v_mfma_f32_32x32x16_bf16 (32-cycle MFMAs leave
//     24 issue cycles each) and run the epilogue; they hold issue priority.  Loader waves do all address
//     arithmetic, global loads and LDS stores.  With one wave per SIMD doing both, that work (~120
//     instructions per step) did not fit in the MFMA shadow and cost +60%;
//   * each compute wave owns 64 conv pixels x 128 output channels (2 x 4 blocks of 32 x 32): per
//     32-channel K-slice it reads 4 A + 8 B fragments (12 KB for 16 MFMAs), 25% fewer LDS bytes per
//     FLOP than 8 waves of 64 x 64, and keeps its 128 accumulators in place for the whole tile;
//   * the workgroup is persistent over tiles; one K-slice per step, one barrier per step;
//   * per step each loader lane issues three 16-byte loads — weights of the slice LAT+2 steps ahead,
//     one 1-KB piece of the input window of the chunk after next — into a ring of LAT register sets and
//     stores the set loaded LAT steps earlier.  vmcnt retires in issue order, so the input window's HBM
//     latency would stall the weights behind it with a short ring (LAT 4: +14%); register staging costs a
//     few issue cycles where an LDS-DMA (buffer_load ... lds) costs its wave 100-200;
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
__device__ __forceinline__ int wswz(int row) { return (row >> 2) & 3; }
__device__ __forceinline__ int hsw(int y) { return y & 3; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}

__device__ __forceinline__ i32x4 ld16(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
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

// LAT (load -> LDS store distance, steps): 10 for 5x5 (100 slices per 128-channel tile), 6 for 3x3
// (36 / 72 slices; the halo deadline below caps it at 10).  Measured on v_conv2: LAT 4 / 5 / 10 / 20 =
// 1.14 / 1.04-1.13 / 1.00 / 1.27 ms (20 spills).
template <int KS, int TH, int TW, int NCLIP, int LAT_ = (KS == 5 ? 10 : 6)>
struct StreamGeom {
    static constexpr int HH = TH + KS - 1, HW = TW + KS - 1;
    static constexpr int HPIX = NCLIP * HH * HW;              // halo pixels per chunk
    static constexpr int HPIECES = (HPIX * 64 + 1023) / 1024;  // 1-KB pieces per chunk
    static constexpr int HPW = (HPIECES + 3) / 4;              // pieces per wave per chunk
    static constexpr int NTAP = KS * KS;
    static constexpr int CSLOT = HPIECES * 1024;               // bytes per halo chunk slot
    static constexpr int WSLOT = 8192;                         // one K-slice of 128 co x 32 ci
    // LAT: steps between a load and its LDS write (the loop is unrolled by LAT); weights are loaded
    // WD = LAT + 2 steps ahead of their slice and land in a 2-slot LDS ring; 3 halo chunk slots;
    // + one 1-KB dummy row per wave for the zero pieces of steps without a real one
    static constexpr int LAT = LAT_, WD = LAT + 2, NHS = 3;
    static constexpr int LDS = NHS * CSLOT + 2 * WSLOT + 4 * 1024;
    static_assert(LDS > 80 * 1024 && LDS <= 160 * 1024, "one persistent workgroup per CU");
    static_assert(NCLIP * TH * TW == 256, "tile = 256 conv pixels (4 waves x 4 fragments)");
    // chunk g+2's pieces are loaded at taps 0..HPW-1 of chunk g and written LAT steps later, before
    // the first fragment read of chunk g+2 at step NTAP-1 of chunk g+1
    static_assert(HPW <= NTAP && HPW - 1 + LAT <= 2 * NTAP - 2, "halo pieces must land in time");
};

// ABL: ablation mask for tools/stream_ablate.hip only (0 in the library): 1 = no halo pieces in the
// loop, 2 = no weight streaming in the loop, 4 = no barrier/wait, 8 = no fragment reads, 16 = no MFMAs,
// 32 = every in-loop piece is a zero fill (all piece instructions, no input traffic), 64 = every tile
// reads clip 0's window (L2-resident input)
template <int KS, int TH, int TW, int NCLIP, int LAT_ = StreamGeom<KS, TH, TW, NCLIP>::LAT, int ABL = 0>
__global__ __launch_bounds__(512, 1) void k_conv_stream(HaloArgs a) {
    using G = StreamGeom<KS, TH, TW, NCLIP, LAT_>;
    constexpr int HH = G::HH, HW = G::HW, HPIX = G::HPIX, HPW = G::HPW, NTAP = G::NTAP;
    constexpr int CSLOT = G::CSLOT, WSLOT = G::WSLOT, LAT = G::LAT, WD = G::WD;
    constexpr int BPR = TW / 8, BPC = (TH / 4) * BPR;     // 4x8-pixel blocks (32 MFMA rows) per row / clip
    static_assert(TW % 8 == 0 && TH % 4 == 0 && BPC % 2 == 0, "a wave's two blocks share their y origin mod 4");
    constexpr int PAD = (KS - 1) / 2;

    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const halo = lds;                    // [NHS][CSLOT]
    char* const wring = lds + G::NHS * CSLOT;  // [2][WSLOT]
    char* const dummy = wring + 2 * WSLOT;     // [4 loader waves][1 KB]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;                    // index within the role

    const int nch = a.Ci / 32;                 // 32-channel chunks per tile
    const int spt = nch * NTAP;                // K-slices per tile (a multiple of 4: 4 | nch)
    const int tiles_x = a.Wc / TW, tiles_y = a.Hc / TH;
    const int tiles_per_clip = tiles_x * tiles_y;
    const int ntiles = ((a.N + NCLIP - 1) / NCLIP) * tiles_per_clip;
    const int nmine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    if (nmine <= 0) return;
    const int nchunks = nmine * nch;
    const int total = nmine * spt;
    const int co0 = blockIdx.y * 128;
    const long long clip_bytes = (long long)a.Hc * a.Wc * a.Ci * 2;

    auto tile_origin = [&](int k, int& clip0, int& oy0, int& ox0) {
        const int t = (int)blockIdx.x + k * (int)gridDim.x;
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
        const int wslice = a.Co * 64;
        int wvoff[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = 32 * w + 16 * u + (lane >> 2), sl = lane & 3;
            wvoff[u] = row * 64 + ((sl ^ wswz(row)) << 4);
        }
        auto wdst = [&](int slot, int u) { return wring + slot * WSLOT + 2048 * w + 1024 * u + lane * 16; };
        auto tile_rsrc = [&](int clip0) {
            return make_rsrc(reinterpret_cast<const char*>(a.in) + (long long)clip0 * clip_bytes,
                             (long long)(a.N - clip0) * clip_bytes);
        };
        // source offset (per lane) and LDS destination (uniform) of piece pc of this loader (P = w + 4 pc)
        // of chunk c of the tile at (oy0, ox0); not real: a zero load bound for this loader's dummy row
        const int ci2 = a.Ci * 2, hc = a.Hc, wc = a.Wc;
        auto piece_addr = [&](bool real, int oy0, int ox0, int c, int slot, int pc, int& voff, char*& dst) {
            const int P = w + 4 * pc;
            const int p = P * 16 + (lane >> 2), sl = lane & 3;
            const int cl = p / (HH * HW), rr = p - cl * (HH * HW);
            const int y = rr / HW, x = rr - y * HW;
            const int iy = oy0 + y - PAD, ix = ox0 + x - PAD;
            const int off = ((cl * hc + iy) * wc + ix) * ci2 + c * 64 + ((sl ^ hsw(y)) << 4);
            const int ok = (int)real & (int)(p < HPIX) & (int)((unsigned)iy < (unsigned)hc) & (int)((unsigned)ix < (unsigned)wc);
            const int mask = -ok;
            voff = (off & mask) | (kOOB & ~mask);
            dst = (real ? halo + slot * CSLOT + P * 1024 : dummy + w * 1024) + lane * 16;
        };

        // tile origins: the current slice's tile and the next one (chunk g+2 may belong to it)
        int cur_clip0, cur_oy0, cur_ox0, nxt_clip0, nxt_oy0, nxt_ox0;
        tile_origin(0, cur_clip0, cur_oy0, cur_ox0);
        tile_origin(1, nxt_clip0, nxt_oy0, nxt_ox0);
        __amdgpu_buffer_rsrc_t cur_rs = tile_rsrc(cur_clip0), nxt_rs = tile_rsrc(nxt_clip0);

        // prologue: chunks 0, 1 of the first tile (nch >= 4) and weight slices 0, 1 straight to LDS;
        // weight slices 2 .. LAT+1 into the register ring (stored by steps 0 .. LAT-1)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc)
#pragma unroll
            for (int pc = 0; pc < HPW; ++pc)
                if (w + 4 * pc < G::HPIECES) {
                    int voff;
                    char* dst;
                    piece_addr(true, cur_oy0, cur_ox0, cc, cc, pc, voff, dst);
                    st16(dst, ld16(cur_rs, voff, 0));
                }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int u = 0; u < 2; ++u) st16(wdst(s, u), ld16(wrs, wvoff[u], (s % spt) * wslice));
        i32x4 rw[LAT][2], rp[LAT];
        char* pdst[LAT];
#pragma unroll
        for (int S = 0; S < LAT; ++S) {
#pragma unroll
            for (int u = 0; u < 2; ++u) rw[S][u] = ld16(wrs, wvoff[u], ((S + 2) % spt) * wslice);
            rp[S] = (i32x4){0, 0, 0, 0};
            pdst[S] = dummy + w * 1024 + lane * 16;
        }
        wait_vm_lgkm0<0>();
        barrier_raw();
        barrier_raw();   // the compute waves have read slice 0 (weight slot 0 is overwritten at step 0)

        // state of the step being issued: its slice (k, c, tap) in halo slot hs; wsa = weight slice
        // loaded by it (step + WD, mod spt)
        int k = 0, c = 0, tap = 0, hs = 0;
        int wsa = WD % spt;
        int pv_voff;
        char* pv_dst;
        __amdgpu_buffer_rsrc_t pv_rs;
        // the piece a step loads: chunk g+2 of its slice's chunk g, piece index = its tap
        auto piece_prep = [&]() {
            const bool real = !(ABL & 32) & (w + 4 * tap < G::HPIECES) & (k * nch + c + 2 < nchunks);
            const bool nx = c + 2 >= nch;
            piece_addr(real, nx ? nxt_oy0 : cur_oy0, nx ? nxt_ox0 : cur_ox0, nx ? c + 2 - nch : c + 2,
                       hs == 0 ? 2 : hs - 1, tap < HPW ? tap : 0, pv_voff, pv_dst);
            pv_rs = nx ? nxt_rs : cur_rs;
        };
        auto lstep = [&](auto sidx, int t) {
            constexpr int S = decltype(sidx)::value;
            // 1. LDS stores of the set loaded LAT steps ago: weights of slice t+2 into ring slot t&1
            //    (slice t's, read during step t-1) and that step's piece
            if constexpr (!(ABL & 2))
#pragma unroll
                for (int u = 0; u < 2; ++u) st16(wdst(t & 1, u), rw[S][u]);
            if constexpr (!(ABL & 1)) st16(pdst[S], rp[S]);
            // 2. this step's loads
            if constexpr (!(ABL & 2))
#pragma unroll
                for (int u = 0; u < 2; ++u) rw[S][u] = ld16(wrs, wvoff[u], wsa * wslice);
            if constexpr (!(ABL & 1)) {
                piece_prep();
                rp[S] = ld16(pv_rs, pv_voff, 0);
                pdst[S] = pv_dst;
            }
            // 3. loads issued LAT-1 or more steps ago have landed (the next step stores the set loaded
            //    LAT-1 steps before it); this step's stores are visible after the barrier
            if constexpr (!(ABL & 4)) {
                wait_vm_lgkm0<(ABL & 3) == 3 ? 0 : (ABL & 3) ? (LAT - 1) * ((ABL & 1) ? 2 : 1) : 3 * (LAT - 1)>();
                barrier_raw();
            }
            // 4. advance to the next slice (a new tile moves the tile origins on)
            if (++wsa == spt) wsa = 0;
            if (++tap == NTAP) {
                tap = 0;
                hs = hs == 2 ? 0 : hs + 1;
                if (++c == nch) {
                    c = 0;
                    ++k;
                    cur_oy0 = nxt_oy0;
                    cur_ox0 = nxt_ox0;
                    cur_rs = nxt_rs;
                    tile_origin(k + 1, nxt_clip0, nxt_oy0, nxt_ox0);
                    nxt_rs = tile_rsrc(nxt_clip0);
                }
            }
        };
        for (int t = 0; t < total; t += LAT)   // total % LAT == 0 (host check)
            [&]<int... S>(std::integer_sequence<int, S...>) {
                (lstep(std::integral_constant<int, S>{}, t + S), ...);
            }(std::make_integer_sequence<int, LAT>{});
        wait_vm_lgkm0<0>();   // loads still in flight target registers and rows nobody reads
        return;
    }

    // =============================== compute waves ===============================
    // the MFMA stream gets issue priority over the co-resident loader wave of its SIMD (-2% time)
    __builtin_amdgcn_s_setprio(2);
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
    for (int m = 0; m < 2; ++m) boffm[m] = r32 * 64 + (((2 * m + hi) ^ wswz(r32)) << 4);
    // fragments of K-slice (chunk slot hs, tap) with weights in ring slot ws: fa[2 i + m] = block i,
    // channels 16 m .. 16 m + 15 of the slice; fb[2 jb + m] = output channels 32 jb .., same channels
    auto frags = [&](int hs, int tap, int ws, i32x4 (&fa)[4], i32x4 (&fb)[8]) {
        const int ky = tap / KS, kx = tap % KS;
        const int sw = hsw(ylo + ky);
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

    // next slice (tap1 of the chunk in halo slot hs1)
    int tap1 = 1, hs1 = 0;
    i32x4 fa[4], fb[8], na[4], nb[8];
    frags(0, 0, 0, fa, fb);
    if constexpr ((ABL & 8) != 0) frags(0, 0, 0, na, nb);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();   // slice 0 read: the loaders may now overwrite weight slot 0

    auto cstep = [&](auto first, int t, i32x4 (&ca)[4], i32x4 (&cb)[8], i32x4 (&xa)[4], i32x4 (&xb)[8]) {
        // fragments of the next slice (weights in ring slot (t+1)&1), interleaved with the 16 MFMAs
        if constexpr (!(ABL & 8)) frags(hs1, tap1, (t + 1) & 1, xa, xb);
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
        if constexpr (!(ABL & 4)) {
            // LDS reads only: the epilogue's global stores (vmcnt on gfx9) are never waited for
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();
        }
        if (++tap1 == NTAP) {
            tap1 = 0;
            hs1 = hs1 == 2 ? 0 : hs1 + 1;
        }
    };
    int t = 0;
    int cur_clip0, cur_oy0, cur_ox0;
    for (int kt = 0; kt < nmine; ++kt) {
        cstep(std::true_type{}, t, fa, fb, na, nb);
        cstep(std::false_type{}, t + 1, na, nb, fa, fb);
        t += 2;
        for (int s = 2; s < spt; s += 2, t += 2) {
            cstep(std::false_type{}, t, fa, fb, na, nb);
            cstep(std::false_type{}, t + 1, na, nb, fa, fb);
        }
        tile_origin(kt, cur_clip0, cur_oy0, cur_ox0);
        epilogue(cur_clip0, cur_oy0, cur_ox0);
    }
}

template <int KS, int TH, int TW, int NCLIP>
int launch_stream(const HaloArgs& a, hipStream_t s) {
    using G = StreamGeom<KS, TH, TW, NCLIP>;
    static bool attr = false;
    if (!attr) {
        AVSE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_stream<KS, TH, TW, NCLIP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr = true;
    }
    if (a.Hc % TH || a.Wc % TW || a.Co % 128 || a.Ci % 32 || ((a.Ci / 32) * KS * KS) % G::LAT) {
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
    hipLaunchKernelGGL((k_conv_stream<KS, TH, TW, NCLIP>), dim3(gx, cob), dim3(512), G::LDS, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

int launch_conv_stream(const HaloArgs& a, hipStream_t s) {
    switch (a.variant) {
        case HALO_K5: return launch_stream<5, 16, 16, 1>(a, s);
        case HALO_K3_16: return launch_stream<3, 16, 16, 1>(a, s);
        case HALO_K3_8: return launch_stream<3, 8, 8, 4>(a, s);
    }
    set_error("stream conv: unsupported variant");
    return 3;
}

}  // namespace avse
