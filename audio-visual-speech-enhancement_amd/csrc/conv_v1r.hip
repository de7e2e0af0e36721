// v_conv1 (network.py:139-143: Conv2D(128, 5x5, 'same') on the normalised 5-frame mouth crops ->
// BatchNorm -> LeakyReLU(0.3) -> MaxPooling2D(2x2)) fused with VideoNormalizer.normalize
// (data_processor.py:208-212) and the f32 -> bf16 cast, gfx950 — dense-K formulation.
//
// K = 5 x 5 taps x 5 frames = 125 runs as 4 K-slices of 32 (128, 3 zero weights), 16 groups of 8 k
// (V1_GMAP, avse_common.h).  The normalised window is stored in LDS with 10-byte pixels (frames 0..4,
// bf16), so kernel row ky of output pixel (y, x) is the 50 contiguous bytes at window pixel (y + ky, x):
// groups 0..14 are the first 24 elements of each row run in thirds (16 B each).  A 16-B run starts at a
// 2-byte boundary when x is odd, so the window is stored twice — copy 1 shifted by 2 bytes — and every
// A fragment is four dword reads (ds_read2_b32 pairs) from the copy that aligns it.  The 5 leftover
// elements (kx = 4, frame 4 of each kernel row) form group 15, read from a column-major "frame-4 plane"
// (column x, 2 bytes per window row, two copies shifted by 2 bytes): frame 4 of window pixels
// (y .. y + 4, x + 4) are 5 consecutive entries of column x + 4; the 16-B read's 3 extra entries meet zero
// weights.  Row pitch 208 B, plane column pitch 48 B, image bases = 0 mod 128 B and the V1_GMAP pairing
// leave one 2-way bank conflict (group 15's half-wave) on the A reads (exhaustive search).
//   * 512 threads: 4 compute waves (v_mfma_f32_16x16x32_bf16, issue priority) + 4 loader waves;
//   * weights: 4 slices x 128 co x 32 k bf16 (32 KB) resident in LDS for the whole launch;
//   * compute wave w owns conv-pixel rows 4w .. 4w+3 of the 16 x 16 tile as 4 blocks of 4x4 pixels x 128
//     output channels; block row r = 4 q + 2 dy + dx is pixel (2 (q >> 1) + dy, 2 (q & 1) + dx), so a
//     lane's 4 accumulator rows are one 2x2 pool window (raw maxima: BN scale >= 0 after the host sign
//     fold).  Tile k's pool maxima go to LDS staging (f32) interleaved with tile k+1's first K-slice, whose
//     MFMAs overwrite the accumulators right after their maxima are taken (2 VALU per MFMA: the MFMA
//     shadow); one workgroup barrier per tile, after that slice;
//   * loader waves, per tile: window k+1 (f32 loaded three tiles ahead, normalised with the prepared
//     (1/std, -mean/std) table, bf16, both copies and the frame-4 plane), output pass of tile k-2 (BN +
//     LeakyReLU on the staged maxima in packed f32 math, bf16, 16-B stores), loads of window k+4.  The
//     loaders' VALU work shares each SIMD's issue with the compute wave's MFMA shadows, but unlike the
//     compute wave's (tied to the accumulators' lifetime) it can land anywhere in the tile.
// Persistent over tiles in XCD-aware order (as conv_stream.hip).
#include "avse_common.h"

namespace avse {
namespace {

constexpr float LRELU = 0.3f;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
constexpr int kOOB = 0x7fffff00;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const int nrec = bytes > kOOB ? kOOB : (bytes < 0 ? 0 : (int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ void barrier_raw() { asm volatile("s_barrier" ::: "memory"); }
// weights image: row (slice, co) 64 B, 16-B k-group s at s ^ wsw(co) (conflict-free for the 16x16x32
// B-operand lane groups, tools/lds_swizzle_search.py)
__device__ __forceinline__ int wsw(int co) { return 2 * ((co >> 2) & 1); }

constexpr int TH = 16, TW = 16, KS = 5, PAD = 2, NF = 5;
constexpr int HH = TH + KS - 1, HW = TW + KS - 1, HPIX = HH * HW;   // 20 x 20 window
constexpr int RP = 208;                                             // window row pitch (10-B pixels)
constexpr int CP = 48;                                              // frame-4 plane column pitch (2-B rows)
constexpr int NSL = 4;                                              // K-slices per tile
constexpr int WIMG = NSL * 128 * 64;                                // 32 KB resident weights
// one window slot: copy 0 | copy 1 (bytes shifted by 2) | plane copy 0 | plane copy 1 (shifted by 2)
constexpr int C1OFF = 4224, PL0 = 8448, PL1 = 9472, WSLOT = 10496, NWS = 3;
// pooled f32 tile (8 x 8 px x 128 co), row pitch 576 B: the compute waves' ds_write_b32 (pixels P, P+1 in
// one 32-lane group) land 16 banks apart
constexpr int SPITCH = 576, STG = 64 * SPITCH;
constexpr int WIN = WIMG, STAGE = WIN + NWS * WSLOT, SSHO = STAGE + 2 * STG;
constexpr int LDS_BYTES = SSHO + 1024;
static_assert(WIN % 128 == 0 && WSLOT % 128 == 0 && C1OFF % 128 == 0 && PL0 % 128 == 0 && PL1 % 128 == 0,
              "bank alignment of the image bases");
static_assert(HH * RP + 2 <= C1OFF && C1OFF + HH * RP <= PL0 && PL0 + HW * CP + 2 <= PL1 && PL1 + HW * CP <= WSLOT &&
                  2 * 22 + 2 <= CP,
              "images (plane columns hold rows 0..22: 20 written, 3 zero for the last 16-B reads)");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
constexpr int PPL = 2;   // window pixels per loader lane (400 of 512)
constexpr int HC = 128, TX = HC / TW, TPC = TX * (HC / TH);         // the network's 128 x 128 crops (launch check)

// loader lane -> window pixel (wy | wx << 8, 0xffff = none) for pixel slot e (0: even columns, 1: odd):
// 8 groups of 25 pixels per slot, one per 32-lane half-wave (the ds_write lane group), chosen by annealing
// so the window-copy and frame-4-plane stores of a group are at most 2-way bank conflicted
__device__ const unsigned short kLoaderPix[2][256] = {
    {
     0x0c04, 0x0402, 0x0a0a, 0x0206, 0x0a11, 0x0002, 0x0e02, 0x120d, 0x0205, 0x000d, 0x0601, 0x0600, 0x0208, 0x0c0f, 0x0c12, 0x0606, 
     0x0008, 0x0c05, 0x0805, 0x0003, 0x0e0c, 0x0a10, 0x0204, 0x0e0e, 0x000c, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0c0e, 0x1006, 0x1004, 0x0c08, 0x0a04, 0x0401, 0x1206, 0x0202, 0x0000, 0x0802, 0x1200, 0x0e0b, 0x020f, 0x000a, 0x0603, 0x0e0f, 
     0x0c0b, 0x1011, 0x120a, 0x0406, 0x0c02, 0x0400, 0x0803, 0x0009, 0x040c, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x1001, 0x0602, 0x0a0c, 0x0801, 0x0810, 0x000e, 0x1203, 0x0a01, 0x0609, 0x0e0a, 0x0608, 0x120e, 0x0a12, 0x0e0d, 0x1010, 0x0209, 
     0x020b, 0x0e13, 0x0800, 0x0403, 0x0e12, 0x040b, 0x1012, 0x0807, 0x0e09, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0c06, 0x0a06, 0x020a, 0x060a, 0x0c07, 0x1002, 0x1204, 0x0405, 0x0203, 0x060e, 0x0e10, 0x0411, 0x0a0d, 0x0806, 0x1208, 0x080a, 
     0x0410, 0x0607, 0x0812, 0x080f, 0x0811, 0x1000, 0x1003, 0x1205, 0x0e05, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x060f, 0x000b, 0x0c13, 0x040e, 0x0813, 0x0c01, 0x040d, 0x0213, 0x0407, 0x0c0a, 0x0a0e, 0x0a0b, 0x0408, 0x080d, 0x0a05, 0x0e01, 
     0x0613, 0x0808, 0x000f, 0x0e04, 0x0a07, 0x0c10, 0x0211, 0x060c, 0x0005, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x1207, 0x100b, 0x0409, 0x0a0f, 0x100d, 0x040a, 0x120b, 0x0e08, 0x1005, 0x0011, 0x0a08, 0x0612, 0x1213, 0x0605, 0x0a09, 0x1211, 
     0x1212, 0x0013, 0x0809, 0x1202, 0x0e11, 0x0404, 0x0010, 0x1201, 0x100c, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0012, 0x1210, 0x0004, 0x0a13, 0x0a03, 0x120f, 0x120c, 0x1007, 0x0c0d, 0x0804, 0x0201, 0x0200, 0x080c, 0x0e03, 0x080b, 0x080e, 
     0x0e00, 0x0c00, 0x0c11, 0x0c09, 0x100f, 0x1009, 0x0610, 0x0a02, 0x0210, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0e06, 0x0611, 0x0c0c, 0x0207, 0x020d, 0x060b, 0x020e, 0x0a00, 0x0604, 0x040f, 0x0e07, 0x100e, 0x1013, 0x0007, 0x060d, 0x0212, 
     0x1008, 0x1209, 0x100a, 0x0c03, 0x020c, 0x0001, 0x0413, 0x0412, 0x0006, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, },
    {
     0x0502, 0x0908, 0x0511, 0x0f01, 0x0b0b, 0x0d0d, 0x030e, 0x0f00, 0x0913, 0x0f05, 0x0d06, 0x0708, 0x010a, 0x0508, 0x0313, 0x010f, 
     0x0912, 0x0302, 0x0f0c, 0x0503, 0x0907, 0x0310, 0x0309, 0x0105, 0x070f, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x1102, 0x1100, 0x1101, 0x0106, 0x0111, 0x0f0b, 0x030c, 0x0113, 0x0909, 0x0f12, 0x0b0a, 0x1303, 0x0110, 0x0d11, 0x0710, 0x1308, 
     0x0509, 0x0706, 0x0d0a, 0x1103, 0x0b0e, 0x0d0e, 0x0f0f, 0x0f09, 0x0704, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0d00, 0x0b0f, 0x1111, 0x0b0d, 0x1310, 0x0312, 0x1307, 0x0d01, 0x1113, 0x1311, 0x0308, 0x0108, 0x050b, 0x0906, 0x0712, 0x0713, 
     0x090e, 0x0f0d, 0x0905, 0x0109, 0x0510, 0x1112, 0x090b, 0x1110, 0x0d13, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0b05, 0x050f, 0x0705, 0x110e, 0x0f02, 0x0b12, 0x0b13, 0x130d, 0x090c, 0x0d05, 0x0107, 0x070a, 0x050c, 0x0711, 0x1306, 0x0b04, 
     0x0d10, 0x0104, 0x0f07, 0x070c, 0x0911, 0x0900, 0x0d12, 0x010b, 0x0b09, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x010c, 0x0d08, 0x030b, 0x0d0c, 0x070e, 0x0f08, 0x0d07, 0x030f, 0x0100, 0x1105, 0x010e, 0x0101, 0x070b, 0x0103, 0x0504, 0x0707, 
     0x0512, 0x0b07, 0x0702, 0x0b01, 0x0513, 0x010d, 0x070d, 0x0b00, 0x0305, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0501, 0x0f04, 0x130a, 0x0709, 0x1107, 0x0700, 0x0d09, 0x0507, 0x0d04, 0x0904, 0x1109, 0x0b06, 0x0d02, 0x0b02, 0x1106, 0x0901, 
     0x0f06, 0x0b08, 0x0300, 0x0d0f, 0x0d0b, 0x0f0a, 0x090d, 0x0506, 0x0903, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x0703, 0x130b, 0x110b, 0x0102, 0x0303, 0x0f10, 0x0910, 0x1301, 0x050a, 0x0d03, 0x0f11, 0x090a, 0x0304, 0x030a, 0x130e, 0x0f03, 
     0x0301, 0x0b0c, 0x1305, 0x0f13, 0x130c, 0x0902, 0x0311, 0x110f, 0x1302, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 
     0x1309, 0x0701, 0x0f0e, 0x1104, 0x1304, 0x0500, 0x0b03, 0x0307, 0x110d, 0x0505, 0x130f, 0x110a, 0x050e, 0x1300, 0x0b11, 0x030d, 
     0x0b10, 0x1312, 0x110c, 0x050d, 0x1313, 0x090f, 0x0306, 0x1108, 0x0112, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, 0xffff, },
};

// V1_GMAP packed 4 bits per (slice, k-group): group of (s, kg) = (kGmap >> (4 (4 s + kg))) & 15
constexpr unsigned long long pack_gmap() {
    unsigned long long v = 0;
    for (int s = 0; s < 4; ++s)
        for (int kg = 0; kg < 4; ++kg) v |= (unsigned long long)V1_GMAP[s][kg] << (4 * (4 * s + kg));
    return v;
}
constexpr unsigned long long kGmap = pack_gmap();
static_assert(V1_GMAP[3][3] == 15, "group 15 (the frame-4 plane: its own block step) is k-group 3 of slice 3");

// ABL: ablation mask for tools/v1r_ablate.hip only (0 in the library): 1 = loaders skip the output pass,
// 2 = loaders skip the per-tile window work, 4 = no MFMAs, 8 = no barrier in the tile loop,
// 16 = s_memtime phase stamps summed per wave into a.prof[(block * 8 + wave) * 8 + phase], 64 = no A-fragment
// reads, 128 = no B-fragment reads, 256 = no maxima
template <int ABL = 0>
__global__ __launch_bounds__(512, 1) void k_conv_v1r(HaloArgs a) {
    extern __shared__ __attribute__((aligned(1024))) char lds[];
    char* const wimg = lds;
    char* const stg = lds + STAGE;                  // [2][STG] pooled raw maxima, compute -> loader
    float* const ssh = reinterpret_cast<float*>(lds + SSHO);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wave & 3;

    const int ntiles = a.N * TPC;
    const int gxs = (int)gridDim.x;
    const int slot = (gxs % 8 == 0) ? ((int)blockIdx.x % 8) * (gxs / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = (ntiles - slot + gxs - 1) / gxs;
    if (nmine <= 0) return;
    auto tile_origin = [&](int k, int& clip, int& oy0, int& ox0) {
        const int t = slot + k * gxs;
        clip = t / TPC;
        const int tt = t % TPC;
        oy0 = (tt / TX) * TH;
        ox0 = (tt % TX) * TW;
    };
    unsigned long long pacc[8] = {}, plast = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int i) {
        if constexpr ((ABL & 16) != 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            pacc[i] += t - plast;
            plast = t;
        }
    };
    auto stamps_out = [&]() {
        if constexpr ((ABL & 16) != 0)
            if (lane == 0)
                for (int i = 0; i < 8; ++i) a.prof[((size_t)blockIdx.x * 8 + wave) * 8 + i] = pacc[i];
    };

    if (wave >= 4) {
        // =============================== loader waves ===============================
        if constexpr ((ABL & 1024) != 0) __builtin_amdgcn_s_setprio(3);
        const int L = w * 64 + lane;
        {   // resident weights [slice][co][32] (host packing) and the BN tail
            const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, (long long)WIMG);
#pragma unroll
            for (int i = 0; i < WIMG / 16 / 256; ++i) {
                const int C = L + 256 * i, row = C >> 2, sl = C & 3;
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, C * 16, 0, 0);
                *reinterpret_cast<i32x4*>(wimg + row * 64 + ((sl ^ wsw(row & 127)) << 4)) = v;
            }
            if (L < 128) {
                ssh[L] = a.scale[L];
                ssh[128 + L] = a.shift[L];
            }
            // the window slots are zeroed once: bytes no pixel store reaches (row pads, plane rows 20..22) are
            // read against zero weights and must hold finite values
            for (int i = L; i < NWS * WSLOT / 4; i += 256) reinterpret_cast<int*>(lds + WIN)[i] = 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();   // Z: zeroing done before any wave stores pixels
        }
        const long long clip_bytes = (long long)a.Hc * a.Wc * NF * 4;
        const bool norm = a.vrn != nullptr;
        const __amdgpu_buffer_rsrc_t nrs = make_rsrc(norm ? a.vrn : a.video, norm ? (long long)a.Hc * a.Wc * 8 : 0);
        // window pixel of (lane, e): kLoaderPix (e = 0 even columns, e = 1 odd: one store pattern per wave)
        int pwy[PPL], pwx[PPL];
        bool pv[PPL];
#pragma unroll
        for (int e = 0; e < PPL; ++e) {
            const unsigned v = kLoaderPix[e][L];
            pv[e] = v != 0xffffu;
            pwy[e] = pv[e] ? (int)(v & 255) : 0;
            pwx[e] = pv[e] ? (int)(v >> 8) : e;
        }
        // three register sets: window t lives in set t % 3 from its loads (three tiles ahead) to its store.
        // Out-of-image pixels load as zeros (buffer range check): video 0 and table (0, 0) -> normalised 0
        f32x4 v4[3][PPL];
        float v1[3][PPL];
        f32x2 rn[3][PPL];
        auto win_load = [&](auto set, int k) {
            constexpr int Q = decltype(set)::value;
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const __amdgpu_buffer_rsrc_t vrs =
                make_rsrc(reinterpret_cast<const char*>(a.video) + (long long)clip * clip_bytes, clip_bytes);
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                const int iy = oy0 + pwy[e] - PAD, ix = ox0 + pwx[e] - PAD;
                const bool ok = pv[e] & ((unsigned)iy < (unsigned)HC) & ((unsigned)ix < (unsigned)HC);
                const int pix = iy * HC + ix;
                const int voff = ok ? pix * NF * 4 : kOOB, noff = ok ? pix * 8 : kOOB;
                v4[Q][e] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, voff, 0, 0));
                v1[Q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, voff, 16, 0));
                rn[Q][e] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(nrs, noff, 0, 0));
            }
        };
        // VideoNormalizer: fma(v, 1/std, -mean/std), bf16; copy 0 at 10 x, copy 1 at 10 x - 2; frame 4 into
        // both plane copies (column x, row y)
        auto win_store = [&](auto set, int hs) {
            constexpr int Q = decltype(set)::value;
            char* const base = lds + WIN + hs * WSLOT;
#pragma unroll
            for (int e = 0; e < PPL; ++e) {
                if (!pv[e]) continue;
                const f32x2 r = rn[Q][e];
                f32x2 n01 = {v4[Q][e][0], v4[Q][e][1]}, n23 = {v4[Q][e][2], v4[Q][e][3]};
                float n4 = v1[Q][e];
                if (norm) {
                    n01 = __builtin_elementwise_fma(n01, (f32x2){r[0], r[0]}, (f32x2){r[1], r[1]});
                    n23 = __builtin_elementwise_fma(n23, (f32x2){r[0], r[0]}, (f32x2){r[1], r[1]});
                    n4 = fmaf(n4, r[0], r[1]);
                }
                const unsigned d0 = __builtin_bit_cast(unsigned, __builtin_convertvector(n01, bf16x2));
                const unsigned d1 = __builtin_bit_cast(unsigned, __builtin_convertvector(n23, bf16x2));
                const unsigned d2 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){n4, 0.f}, bf16x2));
                const unsigned e0 = __builtin_amdgcn_alignbyte(d1, d0, 2);   // (h1, h2)
                const unsigned e1 = __builtin_amdgcn_alignbyte(d2, d1, 2);   // (h3, h4)
                const int off = pwy[e] * RP + 10 * pwx[e];
                char* const c0 = base + off;
                char* const c1 = base + C1OFF + off - 2;
                if (e == 0) {   // even column: copy 0 4-byte aligned, copy 1 2 bytes past
                    *reinterpret_cast<unsigned*>(c0) = d0;
                    *reinterpret_cast<unsigned*>(c0 + 4) = d1;
                    *reinterpret_cast<unsigned short*>(c0 + 8) = (unsigned short)d2;
                    *reinterpret_cast<unsigned short*>(c1) = (unsigned short)d0;
                    *reinterpret_cast<unsigned*>(c1 + 2) = e0;
                    *reinterpret_cast<unsigned*>(c1 + 6) = e1;
                } else {
                    *reinterpret_cast<unsigned short*>(c0) = (unsigned short)d0;
                    *reinterpret_cast<unsigned*>(c0 + 2) = e0;
                    *reinterpret_cast<unsigned*>(c0 + 6) = e1;
                    *reinterpret_cast<unsigned*>(c1) = d0;
                    *reinterpret_cast<unsigned*>(c1 + 4) = d1;
                    *reinterpret_cast<unsigned short*>(c1 + 8) = (unsigned short)d2;
                }
                const int poff = pwx[e] * CP + 2 * pwy[e];
                *reinterpret_cast<unsigned short*>(base + PL0 + poff) = (unsigned short)d2;
                *reinterpret_cast<unsigned short*>(base + PL1 + poff - 2) = (unsigned short)d2;
            }
        };
        // output pass of tile k: BN (|scale|, shift) + LeakyReLU(0.3) on the pooled raw maxima the compute waves
        // left in staging slot k & 1, bf16, 16-B stores (16 lanes = one pooled pixel's 256 bytes).  Packed f32
        // math in asm: the BN pair broadcasts through op_sel, and no canonicalising maxima
        const int c8 = (L & 15) * 8;
        f32x2 obn[8];   // (scale, shift) of channel c8 + e
        const int Wp = HC / 2;
        auto out_pass = [&](int k) {
            int clip, oy0, ox0;
            tile_origin(k, clip, oy0, ox0);
            const long long cb = a.out_clip_stride * 2;
            const __amdgpu_buffer_rsrc_t ors = make_rsrc(reinterpret_cast<const char*>(a.out) + (long long)clip * cb, cb);
            const char* sbase = stg + (k & 1) * STG + (L >> 4) * SPITCH + c8 * 4;
            const int obase = ((oy0 >> 1) * Wp + (ox0 >> 1) + ((L >> 4) & 7)) * a.out_pix_stride + a.out_c_off + c8;
#pragma unroll
            for (int r = 0; r < 4; ++r) {   // pooled pixel P = 16 r + (L >> 4) = (2 r + (L >> 7), (L >> 4) & 7)
                const f32x4 m0 = *reinterpret_cast<const f32x4*>(sbase + 16 * r * SPITCH);
                const f32x4 m1 = *reinterpret_cast<const f32x4*>(sbase + 16 * r * SPITCH + 16);
                const float m[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
                i32x4 o;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    // channels c8 + 2h, c8 + 2h + 1: (m, m') * (sc, sc') + (sh, sh'), max(x, 0.3 x), bf16 pair
                    const f32x2 mm = {m[2 * h], m[2 * h + 1]};
                    const f32x2 sc = {obn[2 * h][0], obn[2 * h + 1][0]}, sh = {obn[2 * h][1], obn[2 * h + 1][1]};
                    f32x2 x, t;
                    float y0, y1;
                    asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(mm), "v"(sc), "v"(sh));
                    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(t) : "v"(x), "s"((f32x2){LRELU, LRELU}));
                    asm("v_max_f32 %0, %1, %2" : "=v"(y0) : "v"(x[0]), "v"(t[0]));
                    asm("v_max_f32 %0, %1, %2" : "=v"(y1) : "v"(x[1]), "v"(t[1]));
                    o[h] = __builtin_bit_cast(int, __builtin_convertvector((f32x2){y0, y1}, bf16x2));
                }
                __builtin_amdgcn_raw_buffer_store_b128(
                    o, ors, (obase + (2 * r + (L >> 7)) * Wp * a.out_pix_stride) * 2, 0, 0);
            }
        };
        using Q0 = std::integral_constant<int, 0>;
        using Q1 = std::integral_constant<int, 1>;
        using Q2 = std::integral_constant<int, 2>;
        // prologue: window 0 in LDS; windows 1, 2, 3 in flight (sets 1, 2, 0)
        win_load(Q0{}, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        win_store(Q0{}, 0);
        if (nmine > 1) win_load(Q1{}, 1);
        if (nmine > 2) win_load(Q2{}, 2);
        if (nmine > 3) win_load(Q0{}, 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();   // P: weights, BN tail, window 0
#pragma unroll
        for (int e = 0; e < 8; ++e) obn[e] = (f32x2){ssh[c8 + e], ssh[128 + c8 + e]};
        // iteration k (between barriers B_{k-1} and B_k; set (k+1) % 3 holds window k+1): window k+1 -> slot
        // (k+1) % 3, tile k-2's output pass (maxima staged before B_{k-1}), window k+4's loads into the freed set
        auto iter = [&](auto set, int k) {
            stamp(7);
            if (k + 1 < nmine && !(ABL & 2)) {
                // younger than window k+1's loads (vmcnt counts stores too): iterations k-2 and k-1, each an output
                // pass (4 stores, from iteration 2 on) and a window's loads (6)
                const int n = ((k >= 4 && !(ABL & 1)) ? 4 : 0) + (k + 2 < nmine ? 6 : 0) + ((k >= 3 && !(ABL & 1)) ? 4 : 0) +
                              (k + 3 < nmine ? 6 : 0);
                switch (n) {
                    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
                    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
                    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
                    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
                    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
                    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
                    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
                    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
                    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
                }
                stamp(0);
                win_store(set, (k + 1) % NWS);
                stamp(1);
            }
            if (k >= 2 && !(ABL & 1)) out_pass(k - 2);
            stamp(3);
            if (k + 4 < nmine && !(ABL & 2)) win_load(set, k + 4);
            stamp(4);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stamp(5);
            if constexpr (!(ABL & 8)) barrier_raw();   // B_k
            stamp(6);
        };
        for (int k = 0; k < nmine; k += 3) {
            iter(Q1{}, k);
            if (k + 1 < nmine) iter(Q2{}, k + 1);
            if (k + 2 < nmine) iter(Q0{}, k + 2);
        }
        if (nmine >= 2 && !(ABL & 1)) out_pass(nmine - 2);
        barrier_raw();   // B_end: the last tile's maxima are staged
        if (!(ABL & 1)) out_pass(nmine - 1);
        stamps_out();
        return;
    }

    // =============================== compute waves ===============================
    if constexpr (!(ABL & 512)) __builtin_amdgcn_s_setprio(2);
    const int r16 = lane & 15, kg = lane >> 4;
    const int q = r16 >> 2, dy = (r16 >> 1) & 1, dx = r16 & 1;
    const int py = 4 * w + 2 * (q >> 1) + dy, px = 2 * (q & 1) + dx;   // block 0; block i is 4 pixels right
    // A-fragment byte offsets per K-slice within a window slot (< 64 KB: two per VGPR — the compute waves
    // run at the 256-register limit)
    unsigned aoff01, aoff23;
    {
        int ao[NSL];
#pragma unroll
        for (int s = 0; s < NSL; ++s) {
            const int g = (int)((kGmap >> (4 * (4 * s + kg))) & 15);
            ao[s] = g < 15 ? (py + g / 3) * RP + 10 * px + 16 * (g % 3) + ((px & 1) ? C1OFF - 2 : 0)
                           : (px + 4) * CP + 2 * py + ((py & 1) ? PL1 - 2 : PL0);
        }
        aoff01 = (unsigned)ao[0] | ((unsigned)ao[1] << 16);
        aoff23 = (unsigned)ao[2] | ((unsigned)ao[3] << 16);
    }
    auto aoff = [&](int s) { return (int)(((s < 2 ? aoff01 : aoff23) >> (16 * (s & 1))) & 0xffff); };
    // block step (4 pixels right): 40 B in the window, 4 plane columns for group 15
    const int step3 = kg == 3 ? 4 * CP : 40;
    const int bbase = r16 * 64 + ((kg ^ wsw(r16)) << 4);   // + slice * 8192 + 1024 j
    barrier_raw();   // Z
    barrier_raw();   // P

    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // pool: the 4 accumulator rows of a lane are one 2x2 window; inline asm keeps the compiler from
    // canonicalising the operands (2 instead of 4 instructions per window)
    auto max4 = [](f32x4 v) {
        float r;
        asm volatile("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, %0, %4" : "=&v"(r) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
        return r;
    };
    // staging: pooled pixel P = (2w + (kg >> 1)) * 8 + 2i + (kg & 1), channel 16 j + r16 at P * SPITCH + 4 co
    char* const sl0 = stg + ((2 * w + (kg >> 1)) * 8 + (kg & 1)) * SPITCH + r16 * 4;
    i32x4 fa[4], na[4], fb[8];
    // one K-slice as 16 units of two MFMAs (j, i0) and (j, i0 + 1), j = p / 2, i0 = 2 (p % 2), each in program
    // order behind a sched_barrier: next-slice A block p (p < 4) into xa; after the last MFMA on column block j
    // (odd p), the next slice's B block j into the same registers (B is single-buffered).  Slice 0 (F) starts
    // every chain from a zero C operand and first stages the previous tile's 2x2 maxima of the two blocks
    // (max3 + max each: 2 VALU per MFMA, the MFMA shadow).  VS: the next slice is slice 3 (per-lane block step)
    auto slice = [&](auto first, auto vstep, int sb_slot, int abyte, int wbyte, i32x4 (&ca)[4], i32x4 (&xa)[4]) {
        constexpr bool F = decltype(first)::value, VS = decltype(vstep)::value;
        char* const sb = sl0 + sb_slot * STG;
        // opaque, provably non-negative base: the block / dword offsets fold into ds_read2_b32 immediates
        asm volatile("" : "+v"(abyte));
        abyte &= 0x3ffff;
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            const int j = p >> 1, i0 = 2 * (p & 1);
            if constexpr (F && !(ABL & 256)) {
                const float m0 = max4(acc[i0][j]), m1 = max4(acc[i0 + 1][j]);
                *reinterpret_cast<float*>(sb + 2 * i0 * SPITCH + 64 * j) = m0;
                *reinterpret_cast<float*>(sb + 2 * (i0 + 1) * SPITCH + 64 * j) = m1;
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (!(ABL & 4)) {
#pragma unroll
                for (int i = i0; i < i0 + 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ca[i]),
                                                                        __builtin_bit_cast(bf16x8, fb[j]),
                                                                        F ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
            }
            if (p < 4 && !(ABL & 64)) {
                const unsigned* qa = reinterpret_cast<const unsigned*>(lds + abyte + (VS ? p * step3 : 40 * p));
                xa[p] = (i32x4){(int)qa[0], (int)qa[1], (int)qa[2], (int)qa[3]};
            }
            __builtin_amdgcn_sched_barrier(0);
            if ((p & 1) && !(ABL & 128)) {
                fb[j] = *reinterpret_cast<const i32x4*>(wimg + wbyte + 1024 * j);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    using T = std::true_type;
    using Fl = std::false_type;
    {   // tile 0's slice-0 fragments
        const int ab = WIN + aoff(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned* qa = reinterpret_cast<const unsigned*>(lds + ab + 40 * i);
            fa[i] = (i32x4){(int)qa[0], (int)qa[1], (int)qa[2], (int)qa[3]};
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[j] = *reinterpret_cast<const i32x4*>(wimg + bbase + 1024 * j);
    }
    // tile k: slice 0 (+ tile k-1's maxima into staging slot (k-1) & 1; tile 0 stages its zero accumulators
    // into a slot nobody reads before tile 1 rewrites it), barrier B_k, slices 1..3; slice 3 reads tile k+1's
    // slice 0
    for (int k = 0; k < nmine; ++k) {
        const int wb = __builtin_amdgcn_readfirstlane(WIN + (k % NWS) * WSLOT);
        const int wbn = __builtin_amdgcn_readfirstlane(WIN + ((k + 1) % NWS) * WSLOT);
        stamp(3);
        slice(T{}, Fl{}, (k - 1) & 1, wb + aoff(1), bbase + 8192, fa, na);
        stamp(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(1);
        if constexpr (!(ABL & 8)) barrier_raw();   // B_k: tile k-1's maxima staged
        stamp(2);
        slice(Fl{}, Fl{}, 0, wb + aoff(2), bbase + 2 * 8192, na, fa);
        slice(Fl{}, T{}, 0, wb + aoff(3), bbase + 3 * 8192, fa, na);
        slice(Fl{}, Fl{}, 0, wbn + aoff(0), bbase, na, fa);
    }
    {   // the last tile's maxima
        char* const sb = sl0 + ((nmine - 1) & 1) * STG;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) *reinterpret_cast<float*>(sb + 2 * i * SPITCH + 64 * j) = max4(acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();   // B_end
    stamp(3);
    stamps_out();
}

__global__ void k_vnorm_prep(const float* __restrict__ mean, const float* __restrict__ stdv, f32x2* __restrict__ rn,
                             int npix) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    const float r = 1.f / stdv[p];
    rn[p] = (f32x2){r, -mean[p] * r};
}

}  // namespace

int launch_conv_v1r(const HaloArgs& a, hipStream_t s) {
    if (int rc = ensure_lds_attr((const void*)k_conv_v1r<0>, LDS_BYTES)) return rc;
    if (a.Hc != HC || a.Wc != HC || a.Co != 128 || a.Ci != NF || !a.w) {
        set_error("v_conv1 dense-K kernel: unexpected layer shape or missing packing");
        return 3;
    }
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = a.N * TPC;
    int gx = ncu >= 8 ? ncu / 8 * 8 : ncu;
    if (gx > tiles) gx = tiles;
    hipLaunchKernelGGL(k_conv_v1r<0>, dim3(gx), dim3(512), LDS_BYTES, s, a);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

int launch_vnorm_prep(const float* mean, const float* stdv, float* rn, int npix, hipStream_t s) {
    hipLaunchKernelGGL(k_vnorm_prep, dim3((npix + 255) / 256), dim3(256), 0, s, mean, stdv,
                       reinterpret_cast<f32x2*>(rn), npix);
    AVSE_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace avse
