// Adaptive bilateral filter kernel for gfx950 (MI355X).
//
// Behaviour follows src/adaptive_bilateral_filter_impl.cu:7-115 of the reference:
//   mean_c   = (sum of the full k x k square, replicate border) / k^2   (float)
//   offset_c = ctr_c - mean_c
//   dist     = |(n0-c0) - o0| + |(n1-c1) - o1| + |(n2-c2) - o2|          (float)
//   w        = ws[ky,kx] * wc[int(dist)]   (circular spatial support)
//   dst_c    = u8(sum_c / sumk + 0.5f)
// dist = sum_c |n_c - 2 c_c + mean_c| reaches 1530, so the reference's full 1536-entry
// LUT (:5) is needed; it is held in LDS as 16 interleaved copies (96 KiB): the two
// lanes l, l+16 of a half-wave that share a copy can meet on one bank (<= 2-way).
// The window sums are exact integers: per-thread vertical column sums (16-bit
// packed R|B lanes when (2R+1)^2*255 < 2^16), then a horizontal sliding window.
#include "vip_stencil.hpp"

#ifndef VIP_ADA_P
#define VIP_ADA_P 4
#endif
#ifndef VIP_ADA_UNROLL  // straight-line tile rows (for_each_row): 384 -> 368 us with scalar taps
#define VIP_ADA_UNROLL 1
#endif

namespace vip {

// Separable box sums need VRB (TH x VW words) after the plane and VW u16 of VG in each
// plane row's unused tail (S - VW words): true up to R = 8 at 16 waves.
template <int R, int P, int WAVES, int LUTW = lut_words(true)>
constexpr bool adaptive_vbox() {
    using G = Geom<R, P>;
    constexpr int VW = G::GROUPS * 4;
    return VW <= 2 * (G::S - VW) && lds_bytes<R, WAVES, 1, LUTW, P>() + 4LL * (WAVES * 4) * VW <= kLdsBudget;
}

// NE: LUT entries in LDS (1536 x 16 copies; or 512 x 32 copies, bank-conflict free, when
// the colour LUT is exactly zero from entry 511 on -- sigma_color 30 underflows past
// d = 431 -- with the index clamped to 511: one v_min_u32 per tap).
// SAT (NE = 512, 32 copies): the index clamp costs no instruction -- the LUT address is
// one v_mad_legacy_u16 with the clamp bit, min(d*128 + B0 + 4c, 65535), in place of the
// v_lshl_or, and every d > 511 saturates onto entry (511, copy 31), an exact zero (the
// SatLut scheme of vip_stencil.hpp with one table). The table sits at LDS byte 16.
constexpr int kAdaSatB0 = 65535 - 511 * 128 - 124;  // 3
constexpr int kAdaSatT = 16;                         // round_up(kAdaSatB0, 16): table byte offset
template <int NE, bool SAT>
constexpr int ada_lut_words() { return NE * (NE < 1536 ? 32 : 16) + (SAT ? kAdaSatT / 4 : 0); }

// The kernel body; MULTI: a multi-frame launch (adaptive_frames_kernel, as bilateral_body)
template <int R, int WAVES, bool FMA, int P, int NE, bool SAT, bool MULTI>
__device__ __forceinline__ void adaptive_body(const StencilArgs& a) {
    static_assert(!SAT || NE == 512, "SAT: 512 entries x 32 copies");
    using G = Geom<R, P>;
    constexpr int NT = WAVES * 64;
    constexpr int TH = WAVES * 4;
    constexpr int ROWS = TH + 2 * R;
    constexpr int K = 2 * R + 1;
    constexpr bool PACK = K * K * 255 < 65536;
    constexpr int NCOL = P + 2 * R;            // columns touched by the thread's P windows
    constexpr int JB = G::L - R;               // first column relative to tx*P
    constexpr int CB0 = JB / 4, CB1 = (G::L + P - 1 + R) / 4;
    // VBOX: the k x k box sums are separable -- vertical K-row sums of the tile plane
    // are computed once per tile cooperatively (VRB: R|B<<16 per column, VG: G as u16 in
    // the plane rows' unused tail words), then each thread slides its K-column windows
    // over them. Fits the LDS for R <= 8; larger radii keep the per-thread square sums.
    constexpr int VW = G::GROUPS * 4;          // plane words in use per row (TW + 2L)
    constexpr bool VBOX = adaptive_vbox<R, P, WAVES, ada_lut_words<NE, SAT>()>();
    // straight-line rows where the separable box sums apply (R <= 8); the larger
    // radii keep the row loop (code size and build time)
    constexpr bool ROW_UNROLL = VIP_ADA_UNROLL != 0 && VBOX;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* const lut = lds + (SAT ? kAdaSatT / 4 : 0);
    constexpr int COPIES = NE < 1536 ? 32 : 16;
    uint32_t* const plane = lds + ada_lut_words<NE, SAT>();
    uint32_t* const vrb = plane + ROWS * G::S;  // VBOX: TH x VW words

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = lane & 15;
    const int ty = wave * 4 + (lane >> 4);
    const uint32_t lane16 = (uint32_t)(lane & (COPIES - 1)) << 2;
#if VIP_SAT_SHARE31  // measurement knob: lanes 30/31 share copy 30, copy 31's bank holds only the saturation target
    const uint32_t sbias = (uint32_t)kAdaSatB0 + (COPIES == 32 && lane16 == 124u ? 120u : lane16);
#else
    const uint32_t sbias = (uint32_t)kAdaSatB0 + lane16;  // SAT: register bias of the address
#endif
    const char* const lut_bytes = reinterpret_cast<const char*>(lut);

    int tile = blockIdx.x;  // persistent: items blockIdx.x + k * gridDim.x (item_tile)
    const int items = launch_items<MULTI>(a);
    TilePrefetch<R, ROWS, NT, P> pf;
    LutStage<NT, NE, COPIES> ls;  // LUT reads go out before the first tile's
    ls.load(a.color);
    {  // multi-frame launches: frame f's tiles follow frame f - 1's
        const FrameTile ft = frame_tile<MULTI>(a, item_tile<MULTI>(a, tile));
        pf.issue(frame_src<MULTI>(a.src, ft.f), a.src_pitch, a, (ft.t % a.tiles_x) * G::TW, (ft.t / a.tiles_x) * TH);
    }
    ls.store(lut);
    pf.commit(plane);
    __syncthreads();

    while (true) {
        const FrameTile ft = frame_tile<MULTI>(a, item_tile<MULTI>(a, tile));
        const int tx0 = (ft.t % a.tiles_x) * G::TW, ty0 = (ft.t / a.tiles_x) * TH;
        const int next = tile + (int)gridDim.x;
        if (next < items) {
            const FrameTile fn = frame_tile<MULTI>(a, item_tile<MULTI>(a, next));
            pf.issue(frame_src<MULTI>(a.src, fn.f), a.src_pitch, a, (fn.t % a.tiles_x) * G::TW,
                     (fn.t / a.tiles_x) * TH);
        }
        if constexpr (VBOX) {
            // ---- pass 1a (whole workgroup): vertical K-row sums, 4 output rows per run ----
            // output row r <-> plane rows r .. r + 2R; every sum is an exact integer
            for (int run = tid; run < VW * (TH / 4); run += NT) {
                const int c = run % VW, r0 = (run / VW) * 4;
                uint32_t rb[4 + K - 1], gg[4 + K - 1], orb[4], og[4];
        #pragma unroll
                for (int t = 0; t < 4 + K - 1; ++t) {
                    const uint32_t p = plane[(r0 + t) * G::S + c];
                    rb[t] = p & 0x00ff00ffu;            // K * 255 per 16-bit field
                    gg[t] = __builtin_amdgcn_ubfe(p, 8, 8);
                }
                win_sum<4, K>(rb, orb);
                win_sum<4, K>(gg, og);
        #pragma unroll
                for (int j = 0; j < 4; ++j) {
                    vrb[(r0 + j) * VW + c] = orb[j];
                    reinterpret_cast<uint16_t*>(plane + (r0 + j) * G::S + VW)[c] = (uint16_t)og[j];
                }
            }
            __syncthreads();
        }
        if (ty0 + wave * 4 < a.out_rows && item_wave<MULTI, WAVES>(a, tile, wave)) {
            uint32_t ctr[P];
            {
                const uint4* c = reinterpret_cast<const uint4*>(plane + (ty + R) * G::S + tx * P + G::L);
        #pragma unroll
                for (int q = 0; q < P / 4; ++q) {
                    const uint4 v = c[q];
                    ctr[4 * q + 0] = v.x; ctr[4 * q + 1] = v.y; ctr[4 * q + 2] = v.z; ctr[4 * q + 3] = v.w;
                }
            }
            float c0f[P], c1f[P], c2f[P], o0[P], o1[P], o2[P];
            const float kk = (float)(K * K);
            const float rkk = 1.f / kk;
            // offset = centre - box mean, as the reference (src/adaptive_bilateral_filter_impl.cu:88-92)
            auto set_offsets = [&](int i, uint32_t sr, uint32_t sg, uint32_t sb) {
                c0f[i] = (float)(ctr[i] & 0xffu);
                c1f[i] = (float)((ctr[i] >> 8) & 0xffu);
                c2f[i] = (float)((ctr[i] >> 16) & 0xffu);
                // opaque to the optimiser: otherwise fsub(uitofp n, uitofp c) in the tap
                // loop is rewritten as an integer v_sub_u32_sdwa + v_cvt_f32_i32 per
                // channel and pair (two slow ops instead of one v_sub_f32)
                __asm__("" : "+v"(c0f[i]), "+v"(c1f[i]), "+v"(c2f[i]));
                o0[i] = c0f[i] - div_exact(sr, kk, rkk);
                o1[i] = c1f[i] - div_exact(sg, kk, rkk);
                o2[i] = c2f[i] - div_exact(sb, kk, rkk);
            };
            if constexpr (VBOX) {
                // ---- pass 1b (per thread): K-column windows of the vertical sums ----
                constexpr int NCOLV = P + K - 1;
                uint32_t hrb[NCOLV], hg[NCOLV];
                const uint32_t* vrow = vrb + ty * VW + tx * P;
                const uint16_t* grow = reinterpret_cast<const uint16_t*>(plane + ty * G::S + VW) + tx * P;
        #pragma unroll
                for (int c = CB0; c <= CB1; ++c) {
                    const uint4 q4 = *reinterpret_cast<const uint4*>(vrow + 4 * c);
                    const uint2 g2 = *reinterpret_cast<const uint2*>(grow + 4 * c);
                    const uint32_t w4[4] = {q4.x, q4.y, q4.z, q4.w};
                    const uint32_t g4[4] = {g2.x & 0xffffu, g2.x >> 16, g2.y & 0xffffu, g2.y >> 16};
        #pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int j = 4 * c + t - JB;
                        if (j < 0 || j >= NCOLV) continue;
                        hrb[j] = w4[t];
                        hg[j] = g4[t];
                    }
                }
                uint32_t wg[P], wr[P], wb[P];
                win_sum<P, K>(hg, wg);
                if constexpr (PACK) {
                    uint32_t wrb[P];
                    win_sum<P, K>(hrb, wrb);
        #pragma unroll
                    for (int i = 0; i < P; ++i) {
                        wr[i] = wrb[i] & 0xffffu;
                        wb[i] = wrb[i] >> 16;
                    }
                } else {
                    uint32_t hr[NCOLV], hb[NCOLV];
        #pragma unroll
                    for (int t = 0; t < NCOLV; ++t) {
                        hr[t] = hrb[t] & 0xffffu;
                        hb[t] = hrb[t] >> 16;
                    }
                    win_sum<P, K>(hr, wr);
                    win_sum<P, K>(hb, wb);
                }
        #pragma unroll
                for (int i = 0; i < P; ++i) set_offsets(i, wr[i], wg[i], wb[i]);
            } else {
            // ---- pass 1: box sums over the full square ----
            // Column sums are kept only for the columns the sliding window adds or
            // drops (slot j < P-1 and j >= K); the window's other columns go straight
            // into one running sum, so registers stay O(P), not O(P + 2R).
            constexpr int HI0 = (K > P - 1) ? K : P - 1;     // first column with a "hi" slot
            constexpr int NSLOT = (P - 1) + (K + P - 1 - HI0);
            auto slot = [](int j) constexpr { return j < P - 1 ? j : (j >= HI0 ? P - 1 + j - HI0 : -1); };
            uint32_t vrb_[NSLOT], vg[NSLOT], vb[PACK ? 1 : NSLOT];
            uint32_t mrb = 0u, mg = 0u, mb = 0u;            // columns in [P-1, K) without a slot
        #pragma unroll
            for (int q = 0; q < NSLOT; ++q) { vrb_[q] = 0u; vg[q] = 0u; if constexpr (!PACK) vb[q] = 0u; }
            for (int r = 0; r < K; ++r) {
                const uint32_t* row = plane + (ty + r) * G::S + tx * P;
        #pragma unroll
                for (int c = CB0; c <= CB1; ++c) {
                    const uint4 q4 = *reinterpret_cast<const uint4*>(row + 4 * c);
                    const uint32_t w4[4] = {q4.x, q4.y, q4.z, q4.w};
        #pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int j = 4 * c + t - JB;  // window column of this word
                        if (j < 0 || j >= NCOL) continue;
                        const uint32_t p = w4[t];
                        const int q = slot(j);
                        uint32_t& arb = q >= 0 ? vrb_[q < 0 ? 0 : q] : mrb;
                        uint32_t& ag = q >= 0 ? vg[q < 0 ? 0 : q] : mg;
                        if constexpr (PACK) {
                            arb += p & 0x00ff00ffu;
                            ag += (p >> 8) & 0xffu;
                        } else {
                            uint32_t& ab = q >= 0 ? vb[q < 0 ? 0 : q] : mb;
                            arb += p & 0xffu;
                            ag += (p >> 8) & 0xffu;
                            ab += (p >> 16) & 0xffu;
                        }
                    }
                }
            }
            {
                uint32_t wrb = mrb, wg = mg, wb = mb;
        #pragma unroll
                for (int j = 0; j < K; ++j) {
                    const int q = slot(j);
                    if (q < 0) continue;
                    wrb += vrb_[q]; wg += vg[q]; if constexpr (!PACK) wb += vb[q];
                }
        #pragma unroll
                for (int i = 0; i < P; ++i) {
                    if (i > 0) {
                        const int qa = slot(i + K - 1), qd = slot(i - 1);
                        wrb += vrb_[qa] - vrb_[qd];
                        wg += vg[qa] - vg[qd];
                        if constexpr (!PACK) wb += vb[qa] - vb[qd];
                    }
                    set_offsets(i, PACK ? (wrb & 0xffffu) : wrb, wg, PACK ? (wrb >> 16) : wb);
                }
            }
            }

            // ---- pass 2: offset-weighted bilateral over the disc ----
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
                    // dist = |(n0-c0)-o0| + |(n1-c1)-o1| + |(n2-c2)-o2|; (float)(n-c) == f_n - f_c exactly.
                    // Index int(dist) <= 1530 -> word d*16 + (lane & 15) of the 1536 x 16 LUT.
                    auto widx = [&](uint32_t, f2 n01, f2 n21, int i, int) {
                        // scalar subtracts here and scalar fma accumulation (row_taps PK =
                        // false): the packed forms (v_pk_add_f32 {b, g} pairs, v_pk_fma_f32
                        // accumulation) measured 446 us per 4K frame against 381 us
                        const float d0 = (n01.x - c0f[i]) - o0[i];
                        const float d1 = (n01.y - c1f[i]) - o1[i];
                        const float d2 = (n21.x - c2f[i]) - o2[i];
                        const float dist = (__builtin_fabsf(d0) + __builtin_fabsf(d1)) + __builtin_fabsf(d2);
                        uint32_t d = (uint32_t)dist;
                        if constexpr (SAT) return sat_addr(d, 128u, sbias) + (uint32_t)(kAdaSatT - kAdaSatB0);
                        if constexpr (NE < 1536) d = d < NE - 1 ? d : NE - 1;
                        return (d << (COPIES == 32 ? 7 : 6)) | lane16;
                    };
                    row_taps<HW, G::L, C0, NC, FMA, false, P, false, decltype(widx)&, false, VIP_PIPE_DEPTH, SAT>(
                        plane, plane, row_off, wsv, lut_bytes, widx, a01, a2k);
                    if constexpr (ROW_UNROLL) fence_accumulators(a01, a2k);
            });

            uint32_t o[P];
            finish_outputs(a01, a2k, o);
            store_px_to(a, frame_dst<MULTI>(a, tile), ty0 + ty, tx0 + tx * P, o);
        }
        if (next >= items) break;
        __syncthreads();
        pf.commit(plane);
        __syncthreads();
        tile = next;
    }
}

template <int R, int WAVES, bool FMA, int P, int NE = 1536, bool SAT = false>
__global__ __launch_bounds__(WAVES * 64) void adaptive_kernel(const StencilArgs a) {
    adaptive_body<R, WAVES, FMA, P, NE, SAT, false>(a);
}
// multi-frame launches (vip_adaptive_run_rows_batch, radius <= kBatchMaxRadius)
template <int R, int WAVES, bool FMA, int P, int NE = 1536, bool SAT = false>
__global__ __launch_bounds__(WAVES * 64) void adaptive_frames_kernel(const StencilArgs a) {
    adaptive_body<R, WAVES, FMA, P, NE, SAT, true>(a);
}

#ifndef VIP_ADA_SHORT_LUT
#define VIP_ADA_SHORT_LUT 0
#endif
#ifndef VIP_ADA_SAT  // 512 x 32 conflict-free LUT behind the saturating address
#define VIP_ADA_SAT 1
#endif

template <int R, bool FMA, int NE, bool SAT = false>
static int launch_adaptive_ne(const StencilArgs& a, hipStream_t stream) {
    // P = 8 outputs per thread needs ~170 VGPRs (per-output centre/offset floats,
    // accumulators, pipelined LUT reads) -> 8 waves; P = 4 fits 128 -> 16 waves
    constexpr int P = VIP_ADA_P;
    using G = Geom<R, P>;
    constexpr int LUTW = ada_lut_words<NE, SAT>();
    constexpr int WAVES = pick_waves<R, 1, P == 8 ? 8 : 16, LUTW, P>();
    static_assert(WAVES > 0, "tile does not fit LDS");
    constexpr int TH = WAVES * 4;
    constexpr int LDS = lds_bytes<R, WAVES, 1, LUTW, P>() +
                        (adaptive_vbox<R, P, WAVES, LUTW>() ? 4 * TH * G::GROUPS * 4 : 0);
    static_assert(LDS <= kLdsBudget, "adaptive tile does not fit LDS");
    auto kern = adaptive_kernel<R, WAVES, FMA, P, NE, SAT>;
    static std::atomic<unsigned long long> attr_devs{0};
    const bool multi = a.nframes > 1;
    if constexpr (R <= kBatchMaxRadius) {
        if (multi) {
            kern = adaptive_frames_kernel<R, WAVES, FMA, P, NE, SAT>;
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
    // the last round in pieces (C3 slab at 8 GPUs, 6 frames per launch, 8 CUs free: one
    // stream 0.0500 -> 0.0477 ms per frame, two streams 0.0429-0.0430 both ways; at 4 GPUs
    // on two streams 0.0960 -> 0.0939; profiles/r05_slab_batch_ab{,2}.txt)
    if (multi) plan_tail(args, blocks, WAVES);
    launch(kern, dim3(blocks), dim3(WAVES * 64), LDS, stream, args);
    return (int)hipGetLastError();
}

template <int R, bool FMA>
static int launch_adaptive_r(const StencilArgs& a, hipStream_t stream) {
    if constexpr (VIP_ADA_SAT != 0)
        if (a.lut_nonzero <= 511) return launch_adaptive_ne<R, FMA, 512, true>(a, stream);
    if constexpr (VIP_ADA_SHORT_LUT != 0)
        if (a.lut_nonzero <= 511) return launch_adaptive_ne<R, FMA, 512>(a, stream);
    return launch_adaptive_ne<R, FMA, 1536>(a, stream);
}

template <bool FMA>
static int launch_adaptive_dispatch(int radius, const StencilArgs& a, hipStream_t stream) {
    switch (radius) {
#define VIP_CASE(RR) \
    case RR: return launch_adaptive_r<RR, FMA>(a, stream);
#ifdef VIP_ONLY_R7
        VIP_CASE(4) VIP_CASE(7)
#else
        VIP_CASE(1) VIP_CASE(2) VIP_CASE(3) VIP_CASE(4) VIP_CASE(5) VIP_CASE(6) VIP_CASE(7) VIP_CASE(8)
        VIP_CASE(9) VIP_CASE(10) VIP_CASE(11) VIP_CASE(12) VIP_CASE(13) VIP_CASE(14) VIP_CASE(15)
#endif
#undef VIP_CASE
        default: return VIP_ERR_UNSUPPORTED_KSIZE;
    }
}

#if defined(VIP_ADA_FMA)
int launch_adaptive_fma(int radius, const StencilArgs& a, hipStream_t s) { return launch_adaptive_dispatch<true>(radius, a, s); }
#else
int launch_adaptive_mul(int radius, const StencilArgs& a, hipStream_t s) { return launch_adaptive_dispatch<false>(radius, a, s); }
#endif

}  // namespace vip
