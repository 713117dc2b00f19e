// Tile geometry and kernel arguments shared by the bilateral, joint-bilateral and
// adaptive-bilateral kernels (gfx950).
//
// Layout in LDS (one workgroup per CU):
//   [0, 96 KiB)      colour LUT, 768 entries x 32 interleaved copies (word d*32 + c)
//                    -> every ds_read_b32 half-wave is bank-conflict free.
//                    The adaptive kernel uses 1536 entries x 16 copies (same 96 KiB).
//   [96 KiB, ...)    RGBX tile plane(s): (TH + 2R) rows x S words, one u32 per pixel
//                    (byte 3 = 0 so v_sad_u8 sees exactly |db|+|dg|+|dr|).
//                    S = round_up(TW + 2L, 8) + 4 words (S = 4 mod 8): the 16 lanes of a
//                    ds_read_b128 group land on disjoint banks.
// Thread mapping: wave w covers tile rows 4w..4w+3, lane l -> row 4w + l/16, columns
// 8*(l%16) .. 8*(l%16)+7 (P = 8 horizontally adjacent outputs per thread).
#pragma once

#include <type_traits>
#include <utility>

#include "vip_common.hpp"

namespace vip {

constexpr int kMaxRadius = 15;            // ksize <= 31 (BASELINE C5 uses ksize 31)
constexpr int kWsStride = kMaxRadius + 1; // spatial weights stored as ws[|ky|][|kx|]
constexpr int kP = 8;                     // outputs per thread
constexpr int kTW = 16 * kP;              // tile width in pixels
constexpr int kLdsBudget = 160 * 1024;
// joint kernel: folded tables behind a saturating address (SatLut) up to this radius. 7 and 8
// work with 16-copy tables (sat_fold_copies), bit-exact, but measured slower than the
// 768 x 16 LUT those radii keep: texture JBF R = 7 186.6 -> 207.8 us, R = 8 242.0 -> 274.7
// (profiles/r06_jbf_fold16_ab.txt)
#ifndef VIP_JBF_SAT_MAX_R
#define VIP_JBF_SAT_MAX_R 6
#endif
constexpr int kSatMaxR = VIP_JBF_SAT_MAX_R;
constexpr int kFoldEntries = 32;  // the handle's folded tables hold d < 32 (zeros past the colour LUT's end)
// Largest distance the folded SatLut stores (measurement knob). A larger DZ (51 at R = 4,
// with 64-entry tables) means fewer saturated lanes and fewer 2-way conflicts on copy 31's
// bank, but measured no faster: C4 frame 674.8 -> 678.9 us (profiles/r03_sat_variants.txt).
#ifndef VIP_JBF_SAT_DZMAX
#define VIP_JBF_SAT_DZMAX (kFoldEntries - 1)
#endif
constexpr int kSatFoldDz = VIP_JBF_SAT_DZMAX;
static_assert(kSatFoldDz < kFoldEntries, "folded tables hold d < kFoldEntries");

// Folded joint-bilateral LUT behind a saturating address (SAT). One table per distinct
// squared tap distance r^2 (NTAB of them) holds RN(ws(r^2) * wc[d]), 32 interleaved
// copies each; the tables of one distance d sit side by side, S = NTAB * 128 bytes per d,
// from LDS byte T on: entry (d, table k, copy c) at T + d*S + 128k + 4c. A tap's address
// is one v_mad_legacy_u16 with the clamp bit, min(d*S + B0 + 4c, 65535), plus the
// compile-time T - B0 + 128k in the ds_read immediate. Up to d = DZ that is the entry
// itself; every larger d saturates to 65535, which B0 = 65535 - DZ*S - 124 places on entry
// (DZ, k, 31) -- an exact zero whenever the colour LUT is zero from DZ on (the texture
// filter's sigma_color sqrt(3): zero from d = 25; DZ = 31 at R <= 5, 26 at R = 6). A
// saturated lane reads the bank of copy 31: a 2-way conflict when that lane does not
// saturate. So the clamp costs no instruction and
// the spatial multiply is folded away: per tap v_sad_u8, v_mad_legacy_u16, ds_read,
// 3 v_fma, v_add (the 32-copy reads stay bank-conflict free; lanes that saturate read one
// broadcast word). T = B0 rounded up to 16 keeps the immediate small and >= 0; the tile
// planes (PB bytes) go below the tables when they fit under B0, else after them.
// NTAB_ = 1, DZMAX = 511: the unfolded colour LUT of the plain filter (zero from d <= 511,
// e.g. sigma_color 30: zero from 432) as 512 entries x 32 copies -- 64 KiB instead of 96,
// the v_lshl_or of the address replaced by the (fast-class) v_mad_legacy_u16.
// COPIES_ (round 6): 16 instead of 32 copies per table halve S, so the 16-bit address reaches
// twice the distances -- the folded tables of radius 7 and 8 (24 and 30 of them) then still
// hold d <= 31 >= 25, the texture JBF's zero point, where 32 copies stop at 21 and 17. Lanes l
// and l + 16 of a half-wave then share a copy (<= 2-way bank conflicts, as the 768 x 16 LUT
// those radii used before); the last copy is 4 * (COPIES - 1) bytes into an entry.
template <int R, int PB, int NTAB_ = disc_r2_count(R), int DZMAX = kSatFoldDz, int COPIES_ = 32>
struct SatLut {
    static constexpr int NTAB = NTAB_;
    static constexpr int COPIES = COPIES_;
    static constexpr int S = NTAB * 4 * COPIES;
    static constexpr int LAST = 4 * (COPIES - 1);
    static constexpr int DZ = (65535 - LAST) / S < DZMAX ? (65535 - LAST) / S : DZMAX;  // tables hold d <= DZMAX
    static constexpr int B0 = 65535 - DZ * S - LAST;
    static constexpr int T = round_up(B0, 16);
    static constexpr int PL = PB <= B0 ? 0 : round_up(T + (DZ + 1) * S, 16);  // plane offset
    static constexpr int BYTES = PB <= B0 ? T + (DZ + 1) * S : PL + PB;
    static_assert(COPIES == 16 || COPIES == 32, "copies");
    static_assert(DZ >= 0 && T - B0 + (NTAB - 1) * 4 * COPIES <= 65535, "ds_read immediate range");
};
// Copies of the joint kernel's folded tables at radius R: 32 (conflict-free) up to R = 6, 16
// beyond (the address range, above)
template <int R>
constexpr int sat_fold_copies() { return R <= 6 ? 32 : 16; }
static_assert(SatLut<6, 0>::DZ >= 25 && SatLut<8, 0, disc_r2_count(8), kSatFoldDz, 16>::DZ >= 25 &&
                  SatLut<7, 0, disc_r2_count(7), kSatFoldDz, 32>::DZ < 25,
              "folded tables reach the texture JBF's zero point (d = 25) with sat_fold_copies");

// Frames one launch of the plain bilateral / adaptive kernels may filter (the
// *_run_rows_batch entry points; a shard's B frames per RCCL group, vip_shard_run_batch).
constexpr int kMaxBatchFrames = 6;
// Radii whose plain / adaptive kernels have a multi-frame form (the small-slab radii; a
// batch of larger radii launches frame by frame)
constexpr int kBatchMaxRadius = 8;

struct StencilArgs {
    const uint8_t* src;
    const uint8_t* guide;  // == src for the plain filters
    uint8_t* dst;
    long long src_pitch, guide_pitch, dst_pitch;
    int width;
    int out_rows;          // output rows to produce
    int src_row0;          // source row of output row 0
    int row_lo, row_hi;    // neighbour rows clamp to [row_lo, row_hi)
    int tiles_x;
    int tiles_total;       // tiles_x * tiles_y (persistent workgroups stride over them)
    int aligned;           // src/guide base and pitch are 4-byte aligned -> dword tile loads
    int dst_aligned;       // dst base and pitch are 8-byte aligned -> qword stores
    const float* color;    // colour LUT in device memory
    int lut_nonzero;       // entries [lut_nonzero, end) of the colour LUT are exactly 0
    const float* fold;     // or null: [disc_r2_count(R)][kFoldEntries] = RN(ws(r^2) * colour[d])
    int inflight;          // host only: frames in flight on this device (the small-frame tiling's model)
    // Multi-frame launch: frame f < nframes reads fsrc[f] and writes fdst[f] (fsrc[0] == src,
    // fdst[0] == dst; same geometry and pitches); launch tile t is tile t - f * tiles_frame of
    // frame f, so the persistent workgroups run straight from one frame's tiles into the
    // next one's (one prologue, the next tile's loads under the current one's taps).
    int nframes;
    int tiles_frame;       // tiles per frame (set by the launcher)
    int free_cus;          // host only: persistent workgroups leave this many CUs to concurrent work
    // Last-round split (multi-frame kernels, plan_tail): launch tiles [tail_full, tiles_total)
    // run in the last round as 2^tail_shift pieces each, a piece being a run of the tile's
    // waves; tail_full == tiles_total and tail_shift == 0 when the rounds come out even.
    int tail_full, tail_shift;
    const uint8_t* fsrc[kMaxBatchFrames];
    uint8_t* fdst[kMaxBatchFrames];
    float ws[kWsStride * kWsStride];  // spatial LUT, |ky|-major, in the kernarg segment (scalar loads)
};

// Runtime-radius kernel (vip_stencil_rt.hip): radius 0 and the radii above the
// templated set, up to the reference's largest (bilateral ksize 65).
constexpr int kRtMaxRadius = 32;

struct RtArgs {
    const uint8_t* src;
    const uint8_t* guide;  // == src for the plain filters
    uint8_t* dst;
    long long src_pitch, guide_pitch, dst_pitch;
    int width, out_rows, src_row0, row_lo, row_hi;  // as StencilArgs
    int aligned, dst_aligned;
    const float* color;    // colour LUT (768 or 1536 entries)
    const float* wsrow;    // [2R+1][wst]: ws(kx, ky) at [ky + R][kx + ra], 0 outside the disc
    const int* hw;         // [R+1]: disc half-width of row |ky|
    int R, wst, ra;
    int L, S, tiles_x;     // set by the launcher
};
int launch_stencil_rt(const RtArgs& a, bool joint, bool adaptive, bool fma, hipStream_t stream);
int stencil_rt_max_radius(bool joint, bool adaptive);

// One workgroup per CU of the current device (the 96 KiB LUT fills most of the CU's
// LDS), each striding over tiles; fewer blocks than CUs when the frame has fewer tiles.
inline int device_cus() {
    static std::atomic<int> cus_by_dev[64];  // CU count per device, 0 = not queried yet
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    int cus = cus_by_dev[dev & 63].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        cus_by_dev[dev & 63].store(cus, std::memory_order_relaxed);
    }
    return cus;
}

// free_cus: CUs the launch leaves to concurrent work (StencilArgs::free_cus)
inline int persistent_blocks(int tiles, int free_cus = 0) {
    int cus = device_cus() - (free_cus > 0 ? free_cus : 0);
    cus = cus > 0 ? cus : 1;
    return tiles < cus ? tiles : cus;
}

constexpr int lut_words(bool adaptive) { return adaptive ? 1536 * 16 : 768 * 32; }

#ifndef VIP_TAIL_SPLIT  // build knob: 0 runs the last round's tiles whole
#define VIP_TAIL_SPLIT 1
#endif
// A persistent launch of T tiles on B workgroups runs ceil(T / B) rounds; when the last
// holds k = T mod B tiles, B - k workgroups idle through it while k run a whole tile each
// (a C2 slab batch at 8 GPUs: 1,530 tiles on 248 workgroups, 6.17 rounds run as 7). The
// last round's tiles are cut into m = 2^s pieces of WAVES / m waves each, the largest m
// with k * m <= B, so that k * m workgroups share them; a piece's workgroup still loads
// the whole tile plane (the apron rows its waves read) and its other waves skip the taps.
// m divides WAVES (a 12-wave tile is cut in 2 or 4, never 8). Returns s (0: no cut).
constexpr int tail_shift(int tiles, int blocks, int waves) {
    if (blocks <= 0 || tiles % blocks == 0) return 0;
    const long long k = tiles % blocks;
    int s = 0;
    while (waves % (2 << s) == 0 && (k << (s + 1)) <= blocks) ++s;
    return s;
}
static_assert(tail_shift(1530, 248, 16) == 2, "C2 slab batch at 8 GPUs: 42 tiles in 4 pieces");
static_assert(tail_shift(1530, 255, 16) == 0 && tail_shift(100, 100, 16) == 0, "even rounds: no cut");
static_assert(tail_shift(7 + 2 * 256, 256, 16) == 4 && tail_shift(7 + 2 * 256, 256, 12) == 2, "pieces divide WAVES");
static_assert(tail_shift(200 + 256, 256, 16) == 0, "k > blocks / 2: whole tiles");
inline void plan_tail(StencilArgs& a, int blocks, int waves) {
    const int s = VIP_TAIL_SPLIT ? tail_shift(a.tiles_total, blocks, waves) : 0;
    a.tail_full = s ? a.tiles_total - a.tiles_total % blocks : a.tiles_total;
    a.tail_shift = s;
}

// Tile filtered by a persistent workgroup at `slot` (= blockIdx.x + k * gridDim.x, round
// k). In full rounds each XCD (workgroups are dispatched round-robin over the 8 XCDs,
// b % 8) gets a run of gridDim.x / 8 consecutive row-major tiles, so horizontally
// adjacent tiles, whose aprons share cache lines, meet in the same L2. The last,
// partial round keeps the identity map. Placement affects speed only, never results.
__device__ __forceinline__ int xcd_tile(int slot, int total) {
    const int grid = (int)gridDim.x, b = (int)blockIdx.x;
    const int base = slot - b;
#ifdef VIP_NO_XCD_MAP
    return slot;
#endif
    if ((grid & 7) != 0 || base + grid > total) return slot;
    return base + (b & 7) * (grid >> 3) + (b >> 3);
}

// P outputs per thread (8, or 4 for register-heavy kernels), TPR threads per tile row:
// 16 (a wave covers 4 tile rows, the default) or 64 ("wide": one 256-pixel row per wave,
// P = 4 -- half the serial work per thread, for frames too small to fill the chip).
// S makes the ds_read_b128 row loads conflict-free: with P = 8 the 16 lanes of a
// b128 group read words tx*8 + 4c of rows ty, ty+1 -> S = 4 (mod 8); with P = 4 and
// 16 threads per row they read 64 contiguous words per row -> S = 0 (mod 64); with 64
// threads per row a wave reads 256 contiguous words of ONE row, whose lane groups
// ({0-3, 12-15, 20-27} ...) always cover 64 distinct banks -> any S.
template <int R, int P = kP, int TPR = 16>
struct Geom {
    static_assert((P == 8 && TPR == 16) || (P == 4 && (TPR == 16 || TPR == 64)), "P, TPR");
    static constexpr int TW = TPR * P;                       // tile width in pixels
    static constexpr int RPW = 64 / TPR;                     // tile rows per wave
    static constexpr int L = round_up(R, 4);                 // left/right apron, 4-px aligned
    static constexpr int S = P == 8 ? round_up(TW + 2 * L, 8) + 4
                                    : (TPR == 64 ? round_up(TW + 2 * L, 4) : round_up(TW + 2 * L, 64));
    static constexpr int GROUPS = (TW + 2 * L) / 4;          // 4-pixel groups per tile row
};

// Largest wave count (<= MAXW: 16, 12, 8 or 4) whose LUT (LUTW words) + plane(s) fit
// the CU's LDS.
template <int R, int PLANES, int MAXW = 16, int LUTW = lut_words(false), int P = kP, int TPR = 16>
constexpr int pick_waves() {
    constexpr int cand[4] = {16, 12, 8, 4};
    for (int w : cand) {
        if (w > MAXW) continue;
        const long long bytes =
            4LL * LUTW + 4LL * PLANES * (w * Geom<R, P, TPR>::RPW + 2 * R) * Geom<R, P, TPR>::S;
        if (bytes <= kLdsBudget) return w;
    }
    return 0;
}

template <int R, int WAVES, int PLANES, int LUTW = lut_words(false), int P = kP, int TPR = 16>
constexpr int lds_bytes() {
    return 4 * LUTW + 4 * PLANES * (WAVES * Geom<R, P, TPR>::RPW + 2 * R) * Geom<R, P, TPR>::S;
}

// Calls f(std::integral_constant<int, HW>) for the runtime circle half-width hw.
// circle_hw is non-increasing in |ky|, so deduplicating neighbours instantiates
// each distinct row body once.
template <int R, int KY>
struct HwDispatch {
    template <class F>
    __device__ __forceinline__ static void run(int hw, F&& f) {
        constexpr int H = circle_hw(R, KY);
        if constexpr (KY == 0 || circle_hw(R, KY - 1) != H) {
            if (hw == H) {
                f(std::integral_constant<int, H>{});
                return;
            }
        }
        if constexpr (KY < R) HwDispatch<R, KY + 1>::run(hw, static_cast<F&&>(f));
    }
};

// Runs f(ky, integral_constant<hw>) for the tile rows ky = -R..R, in order.
// UNROLL: every row is straight-line code with a compile-time half-width, so the
// accumulators stay in their registers from row to row (the caller fences them at
// each row end, see fence_accumulators). Otherwise a runtime row loop dispatches to
// one body per distinct half-width -- half the code, but the register allocator then
// copies every accumulator at each join (2 x 32 v_mov per row for 8 outputs, found
// in the ISA). Measured: bilateral r=7 240 -> 226 us, joint r=4 94 -> 85 us unrolled;
// r=15 (C5, 16384 x 2048 slab) 3283 -> 3211 us; adaptive r=7 384 -> 368 us.
template <int R, bool UNROLL, class F>
__device__ __forceinline__ void for_each_row(F&& f) {
    if constexpr (UNROLL) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
            ((f(I - R, std::integral_constant<int, circle_hw(R, I < R ? R - I : I - R)>{}),
              __builtin_amdgcn_sched_barrier(0)), ...);
        }(std::make_integer_sequence<int, 2 * R + 1>{});
    } else {
        for (int ky = -R; ky <= R; ++ky) {
            const int aky = ky < 0 ? -ky : ky;
            HwDispatch<R, 0>::run(circle_hw(R, aky), [&](auto hwc) { f(ky, hwc); });
        }
    }
}

// 12 bytes (4 RGB pixels) -> 4 RGBX words.
__device__ __forceinline__ uint4 unpack_rgb4(uint32_t a, uint32_t b, uint32_t c) {
    uint4 r;
    r.x = a & 0xffffffu;
    r.y = __builtin_amdgcn_alignbyte(b, a, 3) & 0xffffffu;
    r.z = __builtin_amdgcn_alignbyte(c, b, 2) & 0xffffffu;
    r.w = c >> 8;
    return r;
}

__device__ __forceinline__ uint32_t load_rgb(const uint8_t* row, int x) {
    const uint8_t* p = row + 3 * x;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}

// N sliding sums of K consecutive terms of x (integer: the add/subtract slide is exact)
template <int N, int K>
__device__ __forceinline__ void win_sum(const uint32_t (&x)[N + K - 1], uint32_t (&o)[N]) {
    uint32_t s = x[0];
#pragma unroll
    for (int k = 1; k < K; ++k) s += x[k];
    o[0] = s;
#pragma unroll
    for (int j = 1; j < N; ++j) {
        s = s + x[j + K - 1] - x[j - 1];
        o[j] = s;
    }
}

// Correctly rounded (float)s / d for an integer box sum s and the constant d = k^2
// (or 3): q0 = s*rd, one fma residual, one fma correction. Equal to the IEEE quotient
// for every s in [0, k^2 * 255], k <= 31 -- checked exhaustively in
// tests/test_oracle.py::test_constant_division_is_exact (rd = RN(1/d)).
__device__ __forceinline__ float div_exact(uint32_t s, float d, float rd) {
    const float f = (float)s;
    const float q0 = f * rd;
    return __builtin_fmaf(__builtin_fmaf(-q0, d, f), rd, q0);
}

// Register-staged prefetch of one tile plane: source rows
// [ty0 + src_row0 - R, +ROWS) x columns [tx0 - L, tx0 - L + TW + 2L) of `img`, rows
// clamped to [row_lo, row_hi), columns to [0, width) (the reference's replicate
// border, src/bilateral_filter_impl.cu:47-56). issue() starts the global loads
// (3 dwords per 4-pixel group when the group is interior and dword aligned,
// byte loads otherwise) and returns at once; commit() unpacks RGB to RGBX words
// and writes the LDS plane. A persistent workgroup issues tile t+1 before it
// computes tile t, so HBM latency hides under the VALU-bound tap loop.
template <int R, int ROWS, int NT, int P = kP, int TPR = 16>
struct TilePrefetch {
    using G = Geom<R, P, TPR>;
    static constexpr int NG = ROWS * G::GROUPS;
    static constexpr int K = (NG + NT - 1) / NT;
    uint32_t raw[K][3];

    __device__ __forceinline__ void issue(const uint8_t* img, long long pitch, const StencilArgs& a, int tx0,
                                          int ty0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int g = (int)threadIdx.x + k * NT;
            if (NG % NT != 0 && k == K - 1 && g >= NG) continue;
            const int r = g / G::GROUPS;
            const int gc = g - r * G::GROUPS;
            const int sy = clampi(ty0 + a.src_row0 - R + r, a.row_lo, a.row_hi - 1);
            const uint8_t* row = img + (long long)sy * pitch;
            const int x = tx0 - G::L + 4 * gc;
#ifdef VIP_ABL_NOLOAD  // timing ablation only (wrong output): no HBM reads, the apron included
            if (true) {
                raw[k][0] = (uint32_t)g * 0x01030507u;
                raw[k][1] = (uint32_t)(g + x) * 0x07050301u;
                raw[k][2] = (uint32_t)(g ^ sy) * 0x01010101u;
            } else
#endif
            if (a.aligned && x >= 0 && x + 3 < a.width) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(row + 3 * x);
                raw[k][0] = w[0];
                raw[k][1] = w[1];
                raw[k][2] = w[2];
            } else {
                const uint32_t q0 = load_rgb(row, clampi(x + 0, 0, a.width - 1));
                const uint32_t q1 = load_rgb(row, clampi(x + 1, 0, a.width - 1));
                const uint32_t q2 = load_rgb(row, clampi(x + 2, 0, a.width - 1));
                const uint32_t q3 = load_rgb(row, clampi(x + 3, 0, a.width - 1));
                raw[k][0] = q0 | (q1 << 24);
                raw[k][1] = (q1 >> 8) | (q2 << 16);
                raw[k][2] = (q2 >> 16) | (q3 << 8);
            }
        }
    }

    __device__ __forceinline__ void commit(uint32_t* plane) const {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int g = (int)threadIdx.x + k * NT;
            if (NG % NT != 0 && k == K - 1 && g >= NG) continue;
            const int r = g / G::GROUPS;
            const int gc = g - r * G::GROUPS;
            *reinterpret_cast<uint4*>(plane + r * G::S + 4 * gc) = unpack_rgb4(raw[k][0], raw[k][1], raw[k][2]);
        }
    }
};

// Fill the interleaved colour LUT: word d*COPIES + c = color[d], for
// 768 entries x 32 copies (bilateral, 96 KiB), 768 x 16 (joint bilateral when the
// halved LUT buys more waves, 48 KiB) or 1536 x 16 (adaptive, 96 KiB).
// load() issues all of a thread's LUT reads at once (a compile-time count), store()
// writes them: a kernel calls load() before its first tile's HBM reads, so the LUT
// words arrive during one round trip instead of one dependent L2 round trip per store
// (the earlier runtime loop waited on vmcnt(0) -- the tile prefetch included -- at each
// of its 6 iterations).
template <int NT, int ENTRIES, int COPIES>
struct LutStage {
    static_assert(COPIES == 16 || COPIES == 32, "copies");
    static constexpr int SHIFT = COPIES == 32 ? 3 : 2;  // log2(COPIES / 4 words per store)
    static constexpr int N = ENTRIES * COPIES / 4;        // uint4 stores
    static constexpr int K = (N + NT - 1) / NT;
    uint32_t v[K];

    __device__ __forceinline__ void load(const float* color) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = (int)threadIdx.x + k * NT;
            if (N % NT == 0 || q < N) v[k] = __float_as_uint(color[q >> SHIFT]);
        }
    }
    __device__ __forceinline__ void store(uint32_t* lut) const {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = (int)threadIdx.x + k * NT;
            if (N % NT == 0 || q < N) *reinterpret_cast<uint4*>(lut + 4 * q) = make_uint4(v[k], v[k], v[k], v[k]);
        }
    }
};

// SatLut staging: the fold tables ([NTAB][kFoldEntries] in device memory) into the
// [d][table][copy] layout, d = 0..DZ, at LDS byte T (the store() argument points there).
template <int NT, class SL>
struct SatStage {
    static constexpr int WPD = SL::NTAB * SL::COPIES;   // words per distance
    static constexpr int N = (SL::DZ + 1) * WPD / 4;    // uint4 stores
    static constexpr int K = (N + NT - 1) / NT;
    uint32_t v[K];

    __device__ __forceinline__ void load(const float* fold) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = (int)threadIdx.x + k * NT;
            const int w = 4 * q, d = w / WPD, t = (w - d * WPD) / SL::COPIES;
            if (N % NT == 0 || q < N) v[k] = __float_as_uint(fold[t * kFoldEntries + d]);
        }
    }
    __device__ __forceinline__ void store(uint32_t* lut) const {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int q = (int)threadIdx.x + k * NT;
            if (N % NT == 0 || q < N) *reinterpret_cast<uint4*>(lut + 4 * q) = make_uint4(v[k], v[k], v[k], v[k]);
        }
    }
};

// min(d * s + bias, 65535) in one VALU op (the clamp bit saturates the u16 result);
// the legacy encoding zeroes the destination's high half (checked on gfx950 by
// microbench/sat_addr.hip, which also measures its issue rate in the tap mix).
#ifndef VIP_SAT_INSN
#define VIP_SAT_INSN "v_mad_legacy_u16"
#endif
__device__ __forceinline__ uint32_t sat_addr(uint32_t d, uint32_t s, uint32_t bias) {
    uint32_t r;
    __asm__(VIP_SAT_INSN " %0, %1, %2, %3 clamp" : "=v"(r) : "v"(d), "s"(s), "v"(bias));
    return r;
}

template <int NT, int ENTRIES, int COPIES>
__device__ __forceinline__ void stage_lut(uint32_t* lut, const float* color) {
    LutStage<NT, ENTRIES, COPIES> s;
    s.load(color);
    s.store(lut);
}

// Neighbour words of one tile row, columns [4*C0, 4*C0 + 4*NC), read from LDS in
// 4-word chunks (row_off is 16-byte aligned; indexing as uint4 gives ds_read_b128).
// row_taps loads a chunk only a few columns before its first use, so just a short
// window of the row is live in registers (the whole row of a large radius is not:
// 40 words per plane at R = 15, which spilled).
template <int C0, int NC, bool TWO>
struct RowStream {
    // volatile: keep every load a full ds_read_b128 (hipcc otherwise narrows the
    // edge chunks to the words the row uses and re-pairs them as misaligned,
    // bank-conflicting ds_read2_b32)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const volatile u32x4 lds_u32x4;
    lds_u32x4* g;
    lds_u32x4* s;
    uint32_t gw[4 * NC], sw[4 * NC];

    __device__ __forceinline__ RowStream(const uint32_t* gplane, const uint32_t* splane, int row_off)
        : g((lds_u32x4*)(gplane) + (row_off >> 2) + C0), s((lds_u32x4*)(splane) + (row_off >> 2) + C0) {}

    __device__ __forceinline__ void load(int q) {
        const u32x4 v = g[q];
        gw[4 * q + 0] = v.x; gw[4 * q + 1] = v.y; gw[4 * q + 2] = v.z; gw[4 * q + 3] = v.w;
        if constexpr (TWO) {
            const u32x4 u = s[q];
            sw[4 * q + 0] = u.x; sw[4 * q + 1] = u.y; sw[4 * q + 2] = u.z; sw[4 * q + 3] = u.w;
        }
    }
    // word k (relative to column 4*C0) of the guide / source plane
    __device__ __forceinline__ uint32_t guide(int k) const { return gw[k]; }
    __device__ __forceinline__ uint32_t source(int k) const { return TWO ? sw[k] : gw[k]; }
};

// Progress-based wave priority. The SIMD arbiter serves ready waves by priority,
// then age, so with equal priorities the oldest wave of each SIMD races through
// the tile and idles at the tile barrier while the youngest finishes alone
// (measured with s_memtime stamps: 67K vs 116K cycles for the same work).
// Lowering a wave's priority as it advances through the tile's rows hands the
// issue slots to the waves that are behind, so all reach the barrier together.
// `band` is 0..3 (first quarter of the rows .. last quarter).
__device__ __forceinline__ void set_progress_priority(int band) {
#ifndef VIP_NO_PRIO_BANDS
    switch (band) {  // s_setprio takes an immediate; band is wave-uniform
        case 0: __builtin_amdgcn_s_setprio(3); break;
        case 1: __builtin_amdgcn_s_setprio(2); break;
        case 2: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
    }
#else
    (void)band;
#endif
}

// LUT-read lookahead of the tap loop, in neighbour columns (build knob).
#ifndef VIP_PIPE_DEPTH
#define VIP_PIPE_DEPTH 1
#endif

// The tap loop of one tile row for the thread's kP outputs, software-pipelined
// VIP_PIPE_DEPTH neighbour columns ahead: while column j's weights are
// accumulated, the colour-LUT reads of columns j+1..j+D are already in flight
// (the LDS latency is hidden inside the wave, not only across waves).
// `widx(g, n01, n21, i, kx)` returns the LDS byte address of the colour weight of
// guide word g (source floats {b, g}, {r, 1}) for output i at tap column kx. FOLD: the
// word read is already the tap's full weight ws[ky,kx] * wc[d] (a per-r^2 table, see
// bilateral_kernel), so the spatial multiply is skipped. Accumulation order per output is
// ascending kx, as in the reference's row-major loop.
typedef float f2 __attribute__((ext_vector_type(2)));

// Pins the accumulators at a row boundary: their row's updates happen before this
// point and none move across it (with every row unrolled, the compiler otherwise
// sinks all accumulation below all LUT reads and spills every weight).
template <int P>
__device__ __forceinline__ void fence_accumulators(f2 (&a01)[P], f2 (&a2k)[P]) {
#pragma unroll
    for (int i = 0; i < P; ++i) __asm__ volatile("" : "+v"(a01[i]), "+v"(a2k[i]));
}

// PK: accumulate with v_pk_fma_f32 ({s0,s1} and {s2,sk} pairs). Measured on gfx950:
// slower for every kernel (bilateral -10 %; adaptive 381 us scalar vs 446 us packed,
// together with packed offset subtracts) -- VOP3P ops do not pair with the other
// VALU work -- so both kernels use PK = false; kept as a knob.
// TWO: separate guide and source planes (joint bilateral); otherwise one plane.
#ifndef VIP_ROW_LOOKAHEAD
#define VIP_ROW_LOOKAHEAD 4  // columns between a chunk's LDS read and its first use
#endif
// ABS: widx returns an absolute LDS byte address (the kernel's dynamic LDS starts at 0),
// read through an address-space-3 pointer, so a constant part of it lands in the ds_read
// immediate instead of a v_add of the LDS base.
template <int HW, int L, int C0, int NC, bool FMA, bool PK, int P, bool TWO, class WIdx, bool FOLD = false,
          int D = VIP_PIPE_DEPTH, bool ABS = false>
__device__ __forceinline__ void row_taps(const uint32_t* gplane, const uint32_t* splane, int row_off,
                                         const float (&wsv)[HW + 1], const char* lut, WIdx&& widx,
                                         f2 (&a01)[P], f2 (&a2k)[P]) {
    constexpr int NB = D + 1;            // ring of in-flight columns
    constexpr int J0 = L - HW;           // first neighbour column relative to the thread's P
    constexpr int J1 = L + P - 1 + HW;   // last
    constexpr int LA = D + VIP_ROW_LOOKAHEAD;
    static_assert(J0 >= 4 * C0 && J1 < 4 * (C0 + NC), "row chunk range");
    auto chunk = [](int j) constexpr { return (j - 4 * C0) >> 2; };
    constexpr int PRE = chunk(J0 + LA < J1 ? J0 + LA : J1);  // chunks read before the loop
    RowStream<C0, NC, TWO> row(gplane, splane, row_off);
#pragma unroll
    for (int q = 0; q <= PRE; ++q) row.load(q);
    float wc[NB][P];
    f2 n01[NB], n21[NB];                 // {b, g} and {r, 1} of the neighbour (source image)
    auto issue = [&](int j) {
        const uint32_t g = row.guide(j - 4 * C0);
        const uint32_t p = row.source(j - 4 * C0);
        const int b = (j - J0) % NB;
        n01[b].x = (float)(p & 0xffu);
#ifdef VIP_ABL_CVT  // timing ablation only (wrong output): one byte conversion per column
        n01[b].y = n01[b].x;
        n21[b].x = n01[b].x;
#else
        n01[b].y = (float)((p >> 8) & 0xffu);
        n21[b].x = (float)((p >> 16) & 0xffu);
#endif
        n21[b].y = 1.0f;
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const int kx = j - L - i;
            if (kx < -HW || kx > HW) continue;
            if constexpr (ABS)
                wc[b][i] = *reinterpret_cast<const __attribute__((address_space(3))) float*>(
                    (size_t)widx(g, n01[b], n21[b], i, kx));
            else
                wc[b][i] = *reinterpret_cast<const float*>(lut + widx(g, n01[b], n21[b], i, kx));
        }
    };
#pragma unroll
    for (int j = J0; j < J0 + D && j <= J1; ++j) issue(j);
#pragma unroll
    for (int j = J0; j <= J1; ++j) {
        if (j + LA <= J1 && ((j + LA) & 3) == 0 && chunk(j + LA) > PRE) row.load(chunk(j + LA));
        if (j + D <= J1) issue(j + D);
        const int b = (j - J0) % NB;
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const int kx = j - L - i;
            if (kx < -HW || kx > HW) continue;
            const float w = FOLD ? wc[b][i] : wc[b][i] * wsv[kx < 0 ? -kx : kx];
            if constexpr (FMA && PK) {
                // v_pk_fma_f32: {s0,s1} += {b,g}*w and {s2,sk} += {r,1}*w; each half is an
                // IEEE fma, and fma(1, w, sk) == sk + w exactly
                const f2 w2 = {w, w};
                a01[i] = __builtin_elementwise_fma(n01[b], w2, a01[i]);
                a2k[i] = __builtin_elementwise_fma(n21[b], w2, a2k[i]);
            } else if constexpr (FMA) {
                a01[i].x = __builtin_fmaf(n01[b].x, w, a01[i].x);
                a01[i].y = __builtin_fmaf(n01[b].y, w, a01[i].y);
                a2k[i].x = __builtin_fmaf(n21[b].x, w, a2k[i].x);
                a2k[i].y = a2k[i].y + w;
            } else {
                a01[i].x = a01[i].x + n01[b].x * w;
                a01[i].y = a01[i].y + n01[b].y * w;
                a2k[i].x = a2k[i].x + n21[b].x * w;
                a2k[i].y = a2k[i].y + w;
            }
        }
#ifndef VIP_NO_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
}

// RN(sqrt(x)) for x = 0 or x in [1, 2^24) (the texture gradient's integer sums of
// squares): the hardware v_sqrt_f32 result s and one neighbour check each way -- the
// refinement LLVM's correctly rounded sqrtf expansion applies, without its denormal
// scaling and special-value handling, which these arguments never need. 9 VALU
// instead of 17; microbench/div_check.hip verifies it against sqrtf for EVERY integer
// in [0, 2^20) (the gradient sums stay below 6 * 255^2 = 390150).
__device__ __forceinline__ float sqrt_int_exact(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float s1 = __builtin_fmaf(-sm, s, x) <= 0.f ? sm : s;
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    return __builtin_fmaf(-sp, s, x) > 0.f ? sp : s1;
}

// 2^(j/64), j = 0..63, correctly rounded to double (staged into LDS by the kernels that
// call exp_tab_f32; internal linkage, one copy per translation unit).
static __constant__ double kExp2Tab64[64] = {
#include "vip_exp_tab64.inc"
};

// (float)exp((double)x) for float x in [0, 32) -- the texture guide's alpha argument
// sigma_alpha * (rtv - rtv_min) lies in [0, 255 / (5 ksize)] -- in 14 double ops:
// x = (k/64) ln2 + r with |r| <= ln2/128 (two-part Cody-Waite; k < 2^12, so k * HI is
// exact), exp(r) - 1 by its degree-5 Taylor polynomial (truncation < 2^-54), times
// 2^(k mod 64 / 64) from `etab` (kExp2Tab64 in LDS) and 2^(k / 64). microbench/div_check
// compares it with (float)exp((double)x) for EVERY float in [0, 32).
__device__ __forceinline__ float exp_tab_f32(float xf, const double* etab) {
    const double x = (double)xf;
    const double kd = __builtin_rint(x * 0x1.71547652b82fep+6);  // 64 / ln2
    const int k = (int)kd;
    double r = __builtin_fma(-kd, 0x1.62e42fefa3000p-7, x);       // ln2/64, 12 low bits clear
    r = __builtin_fma(-kd, 0x1.3de6af278ece6p-48, r);             // ln2/64 - HI
    double q = __builtin_fma(r, 1.0 / 120, 1.0 / 24);
    q = __builtin_fma(r, q, 1.0 / 6);
    q = __builtin_fma(r, q, 0.5);
    const double p = __builtin_fma(r * r, q, r);                  // exp(r) - 1
    const double t = etab[k & 63];
    return (float)__builtin_ldexp(__builtin_fma(t, p, t), k >> 6);
}

// clampi((int)v, 0, 255) written into byte `sel` of `word`: floor (the int conversion's
// truncation for v >= 0, and below 0 either way) then v_cvt_pk_u8_f32, whose float->u8
// conversion saturates (an integral input, so its rounding is moot) and packs in the same
// instruction. microbench/div_check compares it with the clamp for every float |v| < 2048.
__device__ __forceinline__ uint32_t pack_u8_clamped(float v, uint32_t sel, uint32_t word) {
    return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_floorf(v), sel, word);
}

// RN(1/k) for k in [1, 2^38): hardware rcp (1 ulp) + one Newton step. Verified
// exhaustively over every float of that range by microbench/div_check.hip.
__device__ __forceinline__ float recip_exact(float k) {
    const float y0 = __builtin_amdgcn_rcpf(k);
    return __builtin_fmaf(__builtin_fmaf(-k, y0, 1.0f), y0, y0);
}

// (float)(n / d) with the IEEE double quotient: the texture guide stage's rtv (CUDA profile,
// src/bilateral_texture_filter_impl.cu:99-101), n = (double)num in [0, 2^18), d =
// (double)msum + 1e-9 in [1e-9, 2^20): no scaling is ever needed. Two Newton steps from
// v_rcp_f64 give r = 1/d to within a few 2^-53 (the first two steps of the compiler's own
// f64 division), so q = RN(n r) is within 4 double ulps of n/d, and RN_f(q) equals
// RN_f(RN_d(n/d)) unless n/d lies within that distance of a float rounding midpoint --
// which q's 29 low mantissa bits show (midpoint: 2^28). Those lanes (about 2^-23 of them)
// take the IEEE division. 7 f64 ops + 3 integer ops against the division's 11 f64 ops.
// microbench/div_check compares it with (float)(n / d) on 2^30 inputs, half of them at
// midpoints.
__device__ __forceinline__ float rtv_quotient(double n, double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r0, 1.0);
    double r = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = n * r;
    const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned long long, q);
    if (__builtin_expect(((lo & 0x1fffffffu) - (0x10000000u - 64u)) < 128u, 0)) return (float)(n / d);
    return (float)q;
}

// RN(s / k) given y = RN(1/k) (Markstein): q0 = RN(s y) is within 1 ulp of s/k, the
// residual s - k q0 is exact under fma, and one correction rounds correctly. Needs
// no over/underflow: s in [0, 255 k], k in [1, 1024). Cross-checked on 2^30 random
// and near-midpoint quotients by microbench/div_check.hip.
__device__ __forceinline__ float div_by_sumk(float s, float k, float y) {
    const float q0 = s * y;
    return __builtin_fmaf(__builtin_fmaf(-k, q0, s), y, q0);
}

// dst = u8(sum_c / sumk + 0.5f) for the P outputs, packed as RGBX words. RCP: the
// window holds its centre tap with weight exactly 1 (bilateral, joint), so sumk is in
// [1, 1024) and the three divides share one exact reciprocal; the adaptive filter's
// sumk may be tiny or 0 and keeps the IEEE divide.
template <int P, bool RCP = false>
__device__ __forceinline__ void finish_outputs(const f2 (&a01)[P], const f2 (&a2k)[P], uint32_t (&o)[P]) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const float sk = a2k[i].y;
        if constexpr (RCP) {
            const float y = recip_exact(sk);
            o[i] = f2u8(div_by_sumk(a01[i].x, sk, y) + 0.5f) | (f2u8(div_by_sumk(a01[i].y, sk, y) + 0.5f) << 8) |
                   (f2u8(div_by_sumk(a2k[i].x, sk, y) + 0.5f) << 16);
        } else {
            o[i] = f2u8(a01[i].x / sk + 0.5f) | (f2u8(a01[i].y / sk + 0.5f) << 8) | (f2u8(a2k[i].x / sk + 0.5f) << 16);
        }
    }
}

// Frame f and its tile index of launch tile mt (multi-frame launches; wave-uniform).
struct FrameTile {
    int f, t;
};
// MULTI = false (every one-frame kernel): tile mt of frame 0, no extra instruction.
template <bool MULTI>
__device__ __forceinline__ FrameTile frame_tile(const StencilArgs& a, int mt) {
    int f = 0;
    if constexpr (!MULTI) return {f, mt};
    // a one-frame launch has tiles_frame == tiles_total > mt; never loops on tiles_frame <= 0
    while (mt >= a.tiles_frame && a.tiles_frame > 0 && f < kMaxBatchFrames - 1) {
        mt -= a.tiles_frame;
        ++f;
    }
    return {f, mt};
}
// Multi-frame kernels take the StencilArgs as their only argument, so it starts the kernel
// argument segment: frame f's pointer is one scalar load from there (indexing the by-value
// argument through a reference would copy the whole struct to scratch).
template <class T>
__device__ __forceinline__ T kernarg_at(size_t byte_offset) {
    typedef const __attribute__((address_space(4))) char kchar;
    typedef const __attribute__((address_space(4))) T kT;
    kchar* base = (kchar*)__builtin_amdgcn_kernarg_segment_ptr();
    return *(kT*)(base + byte_offset);
}

// Work items of a persistent launch: the tiles of the full rounds, then the last round's
// tiles in 2^tail_shift pieces each (plan_tail; one-frame kernels: the tiles).
template <bool MULTI>
__device__ __forceinline__ int launch_items(const StencilArgs& a) {
    if constexpr (!MULTI) return a.tiles_total;
    return a.tail_full + ((a.tiles_total - a.tail_full) << a.tail_shift);
}
// Launch tile of item v (the XCD map in full rounds, the identity in the last)
template <bool MULTI>
__device__ __forceinline__ int item_tile(const StencilArgs& a, int v) {
    if constexpr (!MULTI) return xcd_tile(v, a.tiles_total);
    return v < a.tail_full ? xcd_tile(v, a.tiles_total) : a.tail_full + ((v - a.tail_full) >> a.tail_shift);
}
// Does wave `wave` of a WAVES-wave workgroup filter item v? Every wave of a whole tile; of
// a last-round piece p, waves [p * WAVES / m, (p + 1) * WAVES / m). Wave-uniform.
template <bool MULTI, int WAVES>
__device__ __forceinline__ bool item_wave(const StencilArgs& a, int v, int wave) {
    if constexpr (!MULTI) return true;
    if (v < a.tail_full) return true;
    const int span = WAVES >> a.tail_shift;
    const int piece = (v - a.tail_full) & ((1 << a.tail_shift) - 1);
    return static_cast<unsigned>(wave - piece * span) < static_cast<unsigned>(span);
}

// Output base of item `item`'s frame, derived again at the store: keeping the frame
// index live across the tap loop costs scalar registers the loop's spatial weights use
// (measured +1 % on the 4K r=7 launch).
template <bool MULTI>
__device__ __forceinline__ uint8_t* frame_dst(const StencilArgs& a, int item) {
    if constexpr (!MULTI) return a.dst;
    __asm__ volatile("" : "+s"(item));  // recompute here, not from the tile's start
    int mt = item_tile<MULTI>(a, item), f = 0;
    while (mt >= a.tiles_frame && a.tiles_frame > 0 && f < kMaxBatchFrames - 1) {
        mt -= a.tiles_frame;
        ++f;
    }
    // one scalar load at the store, nothing held across the taps
    return f == 0 ? a.dst : kernarg_at<uint8_t*>(offsetof(StencilArgs, fdst) + f * sizeof(uint8_t*));
}

// fsrc[f] / fdst[f] by uniform selects (no dynamic index into the kernel arguments)
// frame f's source (fsrc[f]; p0 for frame 0)
template <bool MULTI>
__device__ __forceinline__ const uint8_t* frame_src(const uint8_t* p0, int f) {
    if constexpr (!MULTI) return p0;
    return f == 0 ? p0 : kernarg_at<const uint8_t*>(offsetof(StencilArgs, fsrc) + f * sizeof(const uint8_t*));
}

// Write P RGB outputs (3P bytes) of row oy starting at column x to dst (A: StencilArgs or
// RtArgs -- out_rows, width, dst_pitch, dst_aligned).
template <int P, class A>
__device__ __forceinline__ void store_px_to(const A& a, uint8_t* dst, int oy, int x, const uint32_t (&o)[P]) {
    if (oy >= a.out_rows || x >= a.width) return;
    uint8_t* row = dst + (long long)oy * a.dst_pitch;
    if constexpr (P == 4) {
        if (a.dst_aligned && x + P <= a.width) {  // 12 bytes at a 4-byte aligned address
            uint32_t* p = reinterpret_cast<uint32_t*>(row + 3 * x);
            p[0] = o[0] | (o[1] << 24);
            p[1] = (o[1] >> 8) | (o[2] << 16);
            p[2] = (o[2] >> 16) | (o[3] << 8);
            return;
        }
    } else if (a.dst_aligned && x + P <= a.width) {
        uint32_t w[6];
        w[0] = o[0] | (o[1] << 24);
        w[1] = (o[1] >> 8) | (o[2] << 16);
        w[2] = (o[2] >> 16) | (o[3] << 8);
        w[3] = o[4] | (o[5] << 24);
        w[4] = (o[5] >> 8) | (o[6] << 16);
        w[5] = (o[6] >> 16) | (o[7] << 8);
        uint2* p = reinterpret_cast<uint2*>(row + 3 * x);
        p[0] = make_uint2(w[0], w[1]);
        p[1] = make_uint2(w[2], w[3]);
        p[2] = make_uint2(w[4], w[5]);
        return;
    }
    {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            if (x + i < a.width) {
                uint8_t* p = row + 3 * (x + i);
                p[0] = (uint8_t)(o[i]);
                p[1] = (uint8_t)(o[i] >> 8);
                p[2] = (uint8_t)(o[i] >> 16);
            }
        }
    }
}

template <int P, class A>
__device__ __forceinline__ void store_px(const A& a, int oy, int x, const uint32_t (&o)[P]) {
    store_px_to(a, a.dst, oy, x, o);
}

}  // namespace vip
