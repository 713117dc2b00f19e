// Bilateral and joint-bilateral filter kernels for gfx950 (MI355X).
//
// Behaviour follows src/bilateral_filter_impl.cu:7-202 of the reference
// (yuyuyu-bot/various_image_processings): per output pixel and per tap in
// row-major order, w = ws[ky,kx] * wc[|db|+|dg|+|dr|], sum_c += p_c * w,
// sumk += w, dst_c = u8(sum_c / sumk + 0.5f), replicate border. Taps outside
// the disc carry an exact zero weight in the reference and are skipped here,
// which leaves every sum bit-identical (x + 0*p == x).
//
// MI355X design: the kernel is FP32-VALU bound, not HBM bound,
// so everything is arranged to minimise VALU instructions per (output, tap):
//   v_sad_u8 (colour L1 distance of packed RGBX) -> v_lshl_or (LUT address)
//   -> ds_read_b32 (32-copy LUT, bank-conflict free) -> v_mul (spatial weight
//   from an SGPR) -> 3 x v_fma + v_add.
// Neighbour pixels are read once per thread-row with ds_read_b128 and shared by
// the thread's 8 horizontally adjacent outputs.
#include "vip_stencil.hpp"

namespace vip {

#ifdef VIP_STAMPS
// diagnostic build only: [block][wave][tile][3] shader-clock stamps
__device__ unsigned long long vip_stamps[256 * 16 * 8 * 3];
__device__ __forceinline__ void vip_stamp(int blk, int wave, int t, int k) {
    if ((threadIdx.x & 63) == 0 && t < 8 && blk < 256)
        vip_stamps[((blk * 16 + wave) * 8 + t) * 3 + k] = __builtin_amdgcn_s_memtime();
}
#define VIP_STAMP(t, k) vip_stamp(blockIdx.x, wave, t, k)
// [block][entry shader clock, entry 100 MHz real time, exit clock, exit real time]
__device__ unsigned long long vip_rt[256 * 4];
__device__ __forceinline__ void vip_rt_stamp(int k) {
    if (threadIdx.x == 0 && blockIdx.x < 256) {
        vip_rt[blockIdx.x * 4 + 2 * k] = __builtin_amdgcn_s_memtime();
        vip_rt[blockIdx.x * 4 + 2 * k + 1] = __builtin_amdgcn_s_memrealtime();
    }
}
#define VIP_RT_STAMP(k) vip_rt_stamp(k)
#else
#define VIP_STAMP(t, k)
#define VIP_RT_STAMP(k)
#endif

#ifndef VIP_BIL_UNROLL_MAX_R
#define VIP_BIL_UNROLL_MAX_R 15
#endif
#ifndef VIP_BIL_PIPE_DEPTH  // plain bilateral: LUT reads this many neighbour columns ahead
#define VIP_BIL_PIPE_DEPTH VIP_PIPE_DEPTH
#endif
#ifndef VIP_BIL_RCP  // epilogue: one exact reciprocal per output instead of 3 IEEE divides
#define VIP_BIL_RCP 1
#endif
// NE: colour-LUT entries held in LDS. 768 (every L1 distance), or 32 when the
// handle's LUT is exactly zero from entry 31 on (small sigma_color: the texture
// filter's JBF has sigma_color sqrt(3), nonzero up to d = 24): the distance is then
// clamped to 31 (one v_min_u32 per tap) and the 32-copy table takes 4 KiB.
// FOLD (with SAT, NE = 32): one table per distinct squared tap distance r^2, holding
// the full weight RN(ws(r^2) * wc[d]) -- the same float product the unfolded taps
// form, so bit-identical -- addressed by the tap's compile-time table offset (the
// ds_read immediate) behind the saturating address (SatLut, vip_stencil.hpp): per tap
// v_sad_u8, v_mad_legacy_u16, 3 v_fma, v_add and no spatial v_mul, bank-conflict free.
// (Round 2 measured the folded tables behind a v_min clamp + v_lshl_or: 7 VALU, slower.)
template <int R>
struct FoldRank {  // table index of tap (|ky|, |kx|)
    int t[(R + 1) * (R + 1)];
    constexpr FoldRank() : t() {
        for (int y = 0; y <= R; ++y)
            for (int x = 0; x <= R; ++x) t[y * (R + 1) + x] = disc_r2_rank(R, x * x + y * y);
    }
};
// VIP_BIL_MIN_WPE (build knob, experiments): at least this many waves per SIMD, i.e. a
// VGPR cap of 512 / N, so that a smaller workgroup leaves registers for a second kernel
#ifdef VIP_BIL_MIN_WPE
#define VIP_BIL_WPE_ATTR __attribute__((amdgpu_waves_per_eu(VIP_BIL_MIN_WPE)))
#else
#define VIP_BIL_WPE_ATTR
#endif
// The kernel body; MULTI: a multi-frame launch (bilateral_frames_kernel), whose tiles run
// from one frame into the next (StencilArgs::nframes). The one-frame kernel compiles with
// MULTI = false, to exactly the code it had before multi-frame launches existed.
template <int R, int WAVES, bool JOINT, bool FMA, int COPIES, int P, int NE, bool FOLD, int TPR, bool SAT, bool MULTI>
__device__ __forceinline__ void bilateral_body(const StencilArgs& a) {
    using G = Geom<R, P, TPR>;
    constexpr int NT = WAVES * 64;
    constexpr int TH = WAVES * G::RPW;
    constexpr bool ROW_UNROLL = R <= VIP_BIL_UNROLL_MAX_R;  // straight-line rows (for_each_row)
    constexpr int ROWS = TH + 2 * R;
    constexpr int PLANE = ROWS * G::S;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* const lut = lds;
    constexpr int NTAB = FOLD ? disc_r2_count(R) : 1;
    static_assert(!FOLD || (SAT && NE == 32 && COPIES == sat_fold_copies<R>()), "folded tables: saturating address");
    // SAT: tables from byte SL::T, planes at SL::PL (folded: one table per r^2, d <= DZ;
    // unfolded: the colour LUT, d <= 511, times the spatial weight per tap)
    using SL = SatLut<R, 4 * (JOINT ? 2 : 1) * PLANE, FOLD ? disc_r2_count(R) : 1, FOLD ? kSatFoldDz : 511,
                      FOLD ? COPIES : 32>;
    uint32_t* const gplane = SAT ? lds + SL::PL / 4 : lds + NTAB * NE * COPIES;
    uint32_t* const splane = JOINT ? gplane + PLANE : gplane;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = lane % TPR;
    const int ty = wave * G::RPW + lane / TPR;
    const uint32_t lane4 = (uint32_t)(lane & (COPIES - 1)) << 2;  // this lane's LUT copy
#if VIP_SAT_SHARE31  // measurement knob: lanes 30/31 share copy 30, copy 31's bank holds only the saturation target
    const uint32_t sbias = (uint32_t)SL::B0 + (SAT && COPIES == 32 && lane4 == 124u ? 120u : lane4);
#else
    const uint32_t sbias = (uint32_t)SL::B0 + lane4;                // SAT: register bias of the address
#endif
    const char* const lut_bytes = reinterpret_cast<const char*>(lut);

    VIP_RT_STAMP(0);
    // persistent: workgroup b filters items b, b + grid, b + 2 grid, ... (item_tile: the
    // tiles; in a multi-frame launch the last round's tiles in pieces, plan_tail)
    int tile = blockIdx.x;
    const int items = launch_items<MULTI>(a);
    TilePrefetch<R, ROWS, NT, P, TPR> pg, ps;
    // once per workgroup; its reads go out first
    std::conditional_t<SAT, SatStage<NT, SL>, LutStage<NT, NTAB * NE, COPIES>> ls;
    ls.load(FOLD ? a.fold : a.color);
    // multi-frame launches (plain filter only: guide == src): frame f's tiles follow
    // frame f - 1's, so a workgroup's next tile may be the next frame's
    {
        const FrameTile ft = frame_tile<MULTI>(a, item_tile<MULTI>(a, tile));
        const int tx0 = (ft.t % a.tiles_x) * G::TW, ty0 = (ft.t / a.tiles_x) * TH;
        pg.issue(JOINT ? a.guide : frame_src<MULTI>(a.guide, ft.f), a.guide_pitch, a, tx0, ty0);
        if constexpr (JOINT) ps.issue(a.src, a.src_pitch, a, tx0, ty0);
    }
    ls.store(SAT ? lds + SL::T / 4 : lut);
    pg.commit(gplane);
    if constexpr (JOINT) ps.commit(splane);
    __syncthreads();

    for ([[maybe_unused]] int it = 0;; ++it) {
        VIP_STAMP(it, 0);
        const FrameTile ft = frame_tile<MULTI>(a, item_tile<MULTI>(a, tile));
        const int tx0 = (ft.t % a.tiles_x) * G::TW, ty0 = (ft.t / a.tiles_x) * TH;
        const int next = tile + (int)gridDim.x;
        if (next < items) {  // next tile's HBM reads fly under this tile's taps
            const FrameTile fn = frame_tile<MULTI>(a, item_tile<MULTI>(a, next));
            const int nx0 = (fn.t % a.tiles_x) * G::TW, ny0 = (fn.t / a.tiles_x) * TH;
            pg.issue(JOINT ? a.guide : frame_src<MULTI>(a.guide, fn.f), a.guide_pitch, a, nx0, ny0);
            if constexpr (JOINT) ps.issue(a.src, a.src_pitch, a, nx0, ny0);
        }
        // wave-uniform: skip rows past the frame, and other pieces' rows of a split tile
        if (ty0 + wave * G::RPW < a.out_rows && item_wave<MULTI, WAVES>(a, tile, wave)) {
            uint32_t ctr[P];  // centre pixels of the guide (== src for the plain filter)
            {
                const uint4* c = reinterpret_cast<const uint4*>(gplane + (ty + R) * G::S + tx * P + G::L);
#pragma unroll
                for (int q = 0; q < P / 4; ++q) {
                    const uint4 v = c[q];
                    ctr[4 * q + 0] = v.x; ctr[4 * q + 1] = v.y; ctr[4 * q + 2] = v.z; ctr[4 * q + 3] = v.w;
                }
            }
            f2 a01[P], a2k[P];  // {sum_b, sum_g}, {sum_r, sumk}
#pragma unroll
            for (int i = 0; i < P; ++i) a01[i] = a2k[i] = f2{0.f, 0.f};

            for_each_row<R, ROW_UNROLL>([&](const int ky, auto hwc) {
                    constexpr int HW = decltype(hwc)::value;
                    const int aky = ky < 0 ? -ky : ky;
                    set_progress_priority((ky + R) * 4 / (2 * R + 1));
                    const int row_off = (ty + R + ky) * G::S + tx * P;
                    const float* const ws = a.ws + aky * kWsStride;
                    constexpr int C0 = (G::L - HW) / 4, C1 = (G::L + P - 1 + HW) / 4;
                    constexpr int NC = C1 - C0 + 1;
                    float wsv[HW + 1];
#pragma unroll
                    for (int k = 0; k <= HW; ++k) wsv[k] = ws[k];
                    // colour weight address: v_sad_u8 (|db|+|dg|+|dr|) -> word d*COPIES + lane copy
                    auto widx = [&](uint32_t g, f2, f2, int i, int kx) {
                        uint32_t d = __builtin_amdgcn_sad_u8(g, ctr[i], 0u);
                        if constexpr (SAT) {  // min(d*S + bias, 65535) + table offset (immediate)
                            uint32_t off = (uint32_t)(SL::T - SL::B0);
                            if constexpr (FOLD) {
                                constexpr FoldRank<R> rank;
                                off += 4u * COPIES * rank.t[aky * (R + 1) + (kx < 0 ? -kx : kx)];
                            }
                            return sat_addr(d, SL::S, sbias) + off;
                        }
                        if constexpr (NE < 768) d = d < NE - 1 ? d : NE - 1;
                        return (d << (COPIES == 32 ? 7 : 6)) | lane4;
                    };
                    row_taps<HW, G::L, C0, NC, FMA, false, P, JOINT, decltype(widx)&, FOLD,
                             JOINT ? VIP_PIPE_DEPTH : VIP_BIL_PIPE_DEPTH, SAT>(
                        gplane, splane, row_off, wsv, lut_bytes, widx, a01, a2k);
                    if constexpr (ROW_UNROLL) fence_accumulators(a01, a2k);
            });

            uint32_t o[P];
            finish_outputs<P, VIP_BIL_RCP != 0>(a01, a2k, o);
            store_px_to(a, JOINT ? a.dst : frame_dst<MULTI>(a, tile), ty0 + ty, tx0 + tx * P, o);
        }
        VIP_STAMP(it, 1);
        if (next >= items) {
            VIP_RT_STAMP(1);
            break;
        }
        __syncthreads();  // every wave is done reading this tile
        pg.commit(gplane);
        if constexpr (JOINT) ps.commit(splane);
        __syncthreads();
        VIP_STAMP(it, 2);
        tile = next;
    }
}

template <int R, int WAVES, bool JOINT, bool FMA, int COPIES, int P, int NE = 768, bool FOLD = false, int TPR = 16,
          bool SAT = false>
__global__ __launch_bounds__(WAVES * 64) VIP_BIL_WPE_ATTR void bilateral_kernel(const StencilArgs a) {
    bilateral_body<R, WAVES, JOINT, FMA, COPIES, P, NE, FOLD, TPR, SAT, false>(a);
}
// multi-frame launches (vip_bilateral_run_rows_batch; plain filter, radius <= kBatchMaxRadius)
template <int R, int WAVES, bool JOINT, bool FMA, int COPIES, int P, int NE = 768, bool FOLD = false, int TPR = 16,
          bool SAT = false>
__global__ __launch_bounds__(WAVES * 64) VIP_BIL_WPE_ATTR void bilateral_frames_kernel(const StencilArgs a) {
    bilateral_body<R, WAVES, JOINT, FMA, COPIES, P, NE, FOLD, TPR, SAT, true>(a);
}

// The joint kernel holds two tile planes; when the full 32-copy LUT leaves room for
// fewer than 16 waves, a 16-copy LUT (lanes l and l+16 of a half-wave share a copy:
// at most 2-way bank conflicts) is used if it buys more waves (VIP_JBF_LUT16=0 disables).
#ifndef VIP_JBF_LUT16
#define VIP_JBF_LUT16 1
#endif
#ifndef VIP_JBF_MAXW
#define VIP_JBF_MAXW 16
#endif
// Outputs per thread: 8 for the plain filter. The joint filter's second plane and
// prefetch registers push 8 outputs past 128 VGPRs as the radius grows (spilled
// VGPRs: 0 up to R = 3, 1 at R = 4, 14 at R = 7, 36 at R = 8, 69+ beyond); 8 outputs
// still win up to R = 7 (measured: r=4 84 -> 79 us, r=7 214 -> 206 us), 4 above.
#ifndef VIP_JBF_P8_MAX_R
#define VIP_JBF_P8_MAX_R 7
#endif
#ifndef VIP_BIL_P
#define VIP_BIL_P 8
#endif
template <int R, int PLANES>
constexpr int outputs_per_thread() { return PLANES == 2 ? (R <= VIP_JBF_P8_MAX_R ? 8 : 4) : VIP_BIL_P; }
template <int R, int PLANES>
constexpr int lut_copies() {
    constexpr int P = outputs_per_thread<R, PLANES>();
    if (!VIP_JBF_LUT16 || PLANES == 1) return 32;
    return pick_waves<R, PLANES, VIP_JBF_MAXW, 768 * 16, P>() > pick_waves<R, PLANES, 16, 768 * 32, P>() ? 16 : 32;
}
// Plain filter above radius 8 (the row-loop radii, C5's r=15): wave cap (build knob;
// 12 waves allow 168 VGPRs, no spills)
#ifndef VIP_BIL_BIG_MAXW
#define VIP_BIL_BIG_MAXW 16
#endif
// Joint filter with 8 outputs per thread beyond radius 7 (VIP_JBF_P8_MAX_R > 7): wave cap
// (12 waves allow 168 VGPRs: no spills at R = 8..10). Measured round 6 on the texture JBF
// (profiles/r06_jbf_p8_big_r_ab.txt, 4K, interleaved): R = 8 239.7-240.0 us with 4 outputs
// on 16 waves against 266.4-266.6 (8 on 12 waves) and 285.9-286.6 (8 on 8); R = 10 379-380
// against 420 and 449. The default stays 4 outputs beyond radius 7.
#ifndef VIP_JBF_P8_BIG_MAXW
#define VIP_JBF_P8_BIG_MAXW 12
#endif
template <int R, int PLANES>
constexpr int max_waves() {
    return PLANES == 2 ? (R > 7 && R <= VIP_JBF_P8_MAX_R ? VIP_JBF_P8_BIG_MAXW : VIP_JBF_MAXW)
                       : (R > 8 ? VIP_BIL_BIG_MAXW : 16);
}

#ifndef VIP_JBF_WIDE  // joint kernel on wide tiles with the 32-copy LUT (measurement knob)
#define VIP_JBF_WIDE 0
#endif
#ifndef VIP_JBF_WIDE_MAX_R
#define VIP_JBF_WIDE_MAX_R 8
#endif

// Plain kernel on the 512-entry saturating-address LUT (SatLut, 64 KiB, v_mad_legacy_u16
// in place of the v_lshl_or) when the colour LUT allows it. Measured slower, so off: C2
// 172.3 -> 175.4 us, the C5 slab 3198 -> 3296 us (profiles/r03_sat_variants.txt).
#ifndef VIP_BIL_SAT
#define VIP_BIL_SAT 0
#endif

// Joint kernel on the 512-entry saturating-address LUT (SatLut, 32 copies: no bank
// conflicts) in place of the 16-copy 768-entry LUT, when the colour LUT is zero past 511
// (sigma_color 30: past 432) and the tables leave as many waves (measurement knob).
#ifndef VIP_JBF_SAT
#define VIP_JBF_SAT 0
#endif

#ifndef VIP_JBF_SHORT_LUT  // joint kernel: 32-entry clamped LUT when the colour LUT allows it
#define VIP_JBF_SHORT_LUT 0
#endif

// Small frames (plain filter, R <= VIP_BIL_SMALL_MAX_R): a frame with fewer 128 x 64
// tiles than CUs leaves CUs idle (C1's 512 x 512 lenna: 32 tiles on 256 CUs; a 270-row
// slab of the 4K frame at 8 GPUs: 150). Two ways to spread it: fewer waves per workgroup
// (8 or 4: 128 x 32 / 128 x 16 tiles, more CUs busy, fewer waves per SIMD), and the
// "wide" tiling -- one 256-pixel row per wave, 4 outputs per thread -- which halves the
// serial tap work of a thread, so a launch whose tiles fit in one round ends sooner
// (every thread of a 16-wave tile runs its 8 outputs x 149 taps back to back: ~47 us
// at r = 7, whatever the frame size). Chosen per launch by a per-CU time model,
// rounds * waves * cost(waves) * work(P): cost = 1, 1.25, 1.8 at 4, 2, 1 waves per SIMD,
// work = 1 for 8 outputs per thread, kWideWork for 4 (half the taps plus the extra byte
// conversions and apron rows). vip_bilateral_set_waves / VIP_BIL_WAVES and
// vip_bilateral_set_wide / VIP_BIL_WIDE force either.
#ifndef VIP_BIL_SMALL_MAX_R
#define VIP_BIL_SMALL_MAX_R 8
#endif
#ifndef VIP_BIL_WIDE_WORK
#define VIP_BIL_WIDE_WORK 0.55f
#endif
struct Tiling {
    int waves;
    bool wide;
};
// With F frames in flight (distinct streams among the device's recent launches,
// vip_capi.hip frames_in_flight) the frames share the chip, so a frame's rounds are counted
// on cus / F CUs: a small frame then takes the tiling that fills its share, not the one
// that ends soonest alone (C1 with 4 streams: 16-wave 256-px tiles, 61.8k against 27.3k
// Mpx/s for the one-frame choice, profiles/r03 small-frame tables in DESIGN.md section 4).
inline Tiling small_frame_tiling(int width, int out_rows, int inflight = 1, int nframes = 1) {
    const int forced = bilateral_forced_waves();
    const int fwide = bilateral_forced_wide();  // 0 auto, 1 narrow, 2 wide
    const int share = device_cus() / (inflight > 1 ? inflight : 1);  // CUs per launch
    const int cus = share > 0 ? share : 1;
    const int cand[3] = {16, 8, 4};
    const float cost[3] = {1.0f, 1.25f, 1.8f};
    Tiling best{16, false};
    float best_t = 0.f;
    bool first = true;
    for (int wide = 0; wide < 2; ++wide) {
        if ((fwide == 1 && wide) || (fwide == 2 && !wide) || (fwide == 0 && forced && wide)) continue;
        const int tw = wide ? 256 : 128, rpw = wide ? 1 : 4;
        const long long tiles_x = (width + tw - 1) / tw;
        for (int i = 0; i < 3; ++i) {
            if (forced && cand[i] != forced) continue;
            const int th = cand[i] * rpw;
            const long long tiles = tiles_x * ((out_rows + th - 1) / th) * (nframes > 1 ? nframes : 1);
            const float t = (float)((tiles + cus - 1) / cus) * cand[i] * cost[i] * (wide ? VIP_BIL_WIDE_WORK : 1.f);
            if (first || t < best_t) best = Tiling{cand[i], wide != 0}, best_t = t, first = false;
        }
    }
    return best;
}

template <int R, bool JOINT, bool FMA, int NE, bool FOLD, int WAVES, bool WIDE = false, bool SAT = false>
static int launch_bilateral_w(const StencilArgs& a, hipStream_t stream);

// LDS of a SAT launch (the saturating-address tables and the planes)
template <int R, int WAVES, int PLANES, int P, bool FOLD>
constexpr int sat_lds_bytes() {
    return SatLut<R, 4 * PLANES * (WAVES * Geom<R, P>::RPW + 2 * R) * Geom<R, P>::S, FOLD ? disc_r2_count(R) : 1,
                  FOLD ? kSatFoldDz : 511, FOLD ? sat_fold_copies<R>() : 32>::BYTES;
}
template <int R, int PLANES, int MAXW, int P, bool FOLD>
constexpr int pick_waves_sat() {
    if (MAXW >= 16 && sat_lds_bytes<R, 16, PLANES, P, FOLD>() <= kLdsBudget) return 16;
    if (MAXW >= 12 && sat_lds_bytes<R, 12, PLANES, P, FOLD>() <= kLdsBudget) return 12;
    if (MAXW >= 8 && sat_lds_bytes<R, 8, PLANES, P, FOLD>() <= kLdsBudget) return 8;
    return sat_lds_bytes<R, 4, PLANES, P, FOLD>() <= kLdsBudget ? 4 : 0;
}

template <int R, bool JOINT, bool FMA, int NE, bool FOLD = false, bool SAT = false>
static int launch_bilateral_ne(const StencilArgs& a, hipStream_t stream) {
    constexpr int PLANES = JOINT ? 2 : 1;
    constexpr int P = outputs_per_thread<R, PLANES>();
    constexpr int COPIES = FOLD ? sat_fold_copies<R>() : NE < 768 ? 32 : lut_copies<R, PLANES>();
    constexpr int LUTW = (FOLD ? disc_r2_count(R) : 1) * NE * COPIES;
    constexpr int WAVES = SAT ? pick_waves_sat<R, PLANES, max_waves<R, PLANES>(), P, FOLD>()
                              : pick_waves<R, PLANES, max_waves<R, PLANES>(), LUTW, P>();
    static_assert(WAVES > 0, "tile does not fit LDS");
    if constexpr (SAT) {
        return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, WAVES, false, true>(a, stream);
    } else {
#if VIP_JBF_WIDE
        // joint filter on wide tiles (P = 4, one 256-pixel row per wave): two planes of
        // 16 + 2R rows leave room for the 32-copy (bank-conflict free) LUT at 16 waves
        if constexpr (JOINT && !FOLD && NE == 768 && R <= VIP_JBF_WIDE_MAX_R)
            return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 16, true>(a, stream);
#endif
        if constexpr (!JOINT && !FOLD && NE == 768 && WAVES == 16 && R <= VIP_BIL_SMALL_MAX_R) {
            const Tiling t = small_frame_tiling(a.width, a.out_rows, a.inflight, a.nframes);
            if (t.wide) {
                if (t.waves == 16) return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 16, true>(a, stream);
                if (t.waves == 8) return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 8, true>(a, stream);
                return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 4, true>(a, stream);
            }
            if (t.waves == 8) return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 8>(a, stream);
            if (t.waves == 4) return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, 4>(a, stream);
        }
        return launch_bilateral_w<R, JOINT, FMA, NE, FOLD, WAVES>(a, stream);
    }
}

template <int R, bool JOINT, bool FMA, int NE, bool FOLD, int WAVES, bool WIDE, bool SAT>
static int launch_bilateral_w(const StencilArgs& a, hipStream_t stream) {
    constexpr int PLANES = JOINT ? 2 : 1;
    constexpr int P = WIDE ? 4 : outputs_per_thread<R, PLANES>();
    constexpr int TPR = WIDE ? 64 : 16;  // threads per tile row
    using G = Geom<R, P, TPR>;
    constexpr int COPIES = FOLD ? sat_fold_copies<R>()
                                : NE < 768 || (WIDE && pick_waves<R, PLANES, WAVES, 768 * 32, P, TPR>() == WAVES)
                                      ? 32
                                      : lut_copies<R, PLANES>();
    constexpr int LUTW = (FOLD ? disc_r2_count(R) : 1) * NE * COPIES;
    constexpr int TH = WAVES * G::RPW;
    constexpr int LDS = SAT ? sat_lds_bytes<R, WAVES, PLANES, P, FOLD>() : lds_bytes<R, WAVES, PLANES, LUTW, P, TPR>();
    static_assert(LDS <= kLdsBudget, "tile does not fit LDS");
    static_assert(!SAT || TPR == 16, "SAT: 128-pixel tiles");
    auto kern = bilateral_kernel<R, WAVES, JOINT, FMA, COPIES, P, NE, FOLD, TPR, SAT>;
    static std::atomic<unsigned long long> attr_devs{0};
    const bool multi = !JOINT && a.nframes > 1;
    if constexpr (!JOINT && !FOLD && R <= kBatchMaxRadius) {
        if (multi) {
            kern = bilateral_frames_kernel<R, WAVES, JOINT, FMA, COPIES, P, NE, FOLD, TPR, SAT>;
            static std::atomic<unsigned long long> attr_devs_frames{0};
            if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), LDS, attr_devs_frames, SAT))
                return rc;
        }
    } else {
        if (multi) return VIP_ERR_INVALID_ARGUMENT;  // no multi-frame form (the batch entry point loops frames)
    }
    if (!multi)
        if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), LDS, attr_devs, SAT)) return rc;
    note_launch(reinterpret_cast<const void*>(kern));
    StencilArgs args = a;
    args.tiles_x = (a.width + G::TW - 1) / G::TW;
    args.tiles_frame = args.tiles_x * ((a.out_rows + TH - 1) / TH);
    args.tiles_total = args.tiles_frame * (multi ? a.nframes : 1);
    if (args.tiles_total == 0) return 0;
    const int blocks = persistent_blocks(args.tiles_total, a.free_cus);
    args.tail_full = args.tiles_total;  // no cut: every item a whole tile on the XCD map
    args.tail_shift = 0;
    // the last round in pieces for one frame in flight only: with two streams the other
    // stream's launch already fills the CUs a whole-tile last round leaves idle, and the
    // pieces' fewer waves per CU cost more CU time (C2 slab at 8 GPUs, 6 frames per launch,
    // 8 CUs free: one stream 0.0256-0.0258 -> 0.0250 ms per frame, two streams 0.0222-0.0225
    // -> 0.0231-0.0233; profiles/r05_slab_batch_ab{,2}.txt)
    if (multi && a.inflight <= 1) plan_tail(args, blocks, WAVES);
    launch(kern, dim3(blocks), dim3(WAVES * 64), LDS, stream, args);
    return (int)hipGetLastError();
}

template <int R>
constexpr bool jbf_sat_fits() {
    constexpr int P = outputs_per_thread<R, 2>();
    return pick_waves_sat<R, 2, max_waves<R, 2>(), P, false>() >=
           pick_waves<R, 2, max_waves<R, 2>(), 768 * lut_copies<R, 2>(), P>();
}

template <int R, bool JOINT, bool FMA>
static int launch_bilateral_r(const StencilArgs& a, hipStream_t stream) {
    if constexpr (!JOINT && VIP_BIL_SAT) {  // plain filter, 128-pixel 16-wave tiles: 512 x 32 LUT (SatLut)
        if (a.lut_nonzero <= 511) {
            const Tiling t = R <= VIP_BIL_SMALL_MAX_R ? small_frame_tiling(a.width, a.out_rows, a.inflight, a.nframes)
                                                      : Tiling{16, false};
            if (t.waves == 16 && !t.wide) return launch_bilateral_ne<R, JOINT, FMA, 768, false, true>(a, stream);
        }
    }
    if constexpr (JOINT && R <= kSatMaxR)  // saturating-address folded tables (SatLut)
        if (a.fold && a.lut_nonzero <= SatLut<R, 0, disc_r2_count(R), kSatFoldDz, sat_fold_copies<R>()>::DZ)
            return launch_bilateral_ne<R, JOINT, FMA, 32, true, true>(a, stream);
    if constexpr (JOINT && VIP_JBF_SHORT_LUT)
        if (a.lut_nonzero <= 31) return launch_bilateral_ne<R, JOINT, FMA, 32>(a, stream);
    if constexpr (JOINT && VIP_JBF_SAT && jbf_sat_fits<R>())
        if (!a.fold && a.lut_nonzero <= 511) return launch_bilateral_ne<R, JOINT, FMA, 768, false, true>(a, stream);
    return launch_bilateral_ne<R, JOINT, FMA, 768>(a, stream);
}

template <bool JOINT, bool FMA>
static int launch_bilateral_dispatch(int radius, const StencilArgs& a, hipStream_t stream) {
    switch (radius) {
#define VIP_CASE(RR) \
    case RR: return launch_bilateral_r<RR, JOINT, FMA>(a, stream);
#ifdef VIP_ONLY_R7
        VIP_CASE(4) VIP_CASE(7) VIP_CASE(15)
#else
        VIP_CASE(1) VIP_CASE(2) VIP_CASE(3) VIP_CASE(4) VIP_CASE(5) VIP_CASE(6) VIP_CASE(7) VIP_CASE(8)
        VIP_CASE(9) VIP_CASE(10) VIP_CASE(11) VIP_CASE(12) VIP_CASE(13) VIP_CASE(14) VIP_CASE(15)
#endif
#undef VIP_CASE
        default: return VIP_ERR_UNSUPPORTED_KSIZE;
    }
}

// One translation unit per (JOINT, FMA) variant so the 15 radii compile in parallel.
#if defined(VIP_BIL_JOINT) && defined(VIP_BIL_FMA)
int launch_bilateral_joint_fma(int radius, const StencilArgs& a, hipStream_t s) {
    return launch_bilateral_dispatch<true, true>(radius, a, s);
}
#elif defined(VIP_BIL_JOINT)
int launch_bilateral_joint_mul(int radius, const StencilArgs& a, hipStream_t s) {
    return launch_bilateral_dispatch<true, false>(radius, a, s);
}
#elif defined(VIP_BIL_FMA)
int launch_bilateral_plain_fma(int radius, const StencilArgs& a, hipStream_t s) {
    return launch_bilateral_dispatch<false, true>(radius, a, s);
}
#ifdef VIP_STAMPS
}  // namespace vip
extern "C" int vip_debug_read_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vip::vip_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int vip_debug_read_rt(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vip::vip_rt), bytes, 0, hipMemcpyDeviceToHost);
}
namespace vip {
#endif
#else
int launch_bilateral_plain_mul(int radius, const StencilArgs& a, hipStream_t s) {
    return launch_bilateral_dispatch<false, false>(radius, a, s);
}
#endif

}  // namespace vip
