// Bilateral-texture-filter stages for gfx950 (MI355X): gradient magnitude,
// box blur + modified relative total variation (mRTV), and the guide image.
//
// Reference: src/gradient_impl.cu:7-112, src/bilateral_texture_filter_impl.cu:10-177
// (yuyuyu-bot/various_image_processings). Arithmetic is written out explicitly
// (the library is built with -ffp-contract=off) so that the oracle's CUDA
// profile reproduces it bit for bit:
//   gradient f32 : del = fmaf(d, d, del) per channel (nvcc contraction), sqrtf
//   mRTV         : (imax - imin) * mmax / ((double)msum + 1e-9) in double
//   guide        : exp evaluated as (float)exp(double) (correctly rounded expf),
//                  g = int(fmaf(alpha, B[argmin], (1 - alpha) * B) + 0.5f)
#include "vip_stencil.hpp"

namespace vip {

// ---------------------------------------------------------------------------
// gradient: one thread per pixel; neighbours come through L1/L2 (4 reads/pixel).
// ---------------------------------------------------------------------------
template <typename T, int CH, bool FMA>
__global__ __launch_bounds__(256) void gradient_kernel(const T* __restrict__ src, float* __restrict__ dst, int width,
                                                      int height) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= width || y >= height) return;
    const int xm = max(x - 1, 0), xp = min(x + 1, width - 1);
    const int ym = max(y - 1, 0), yp = min(y + 1, height - 1);
    const long long w = width;
    const T* r0 = src + (y * w) * CH;
    const T* rm = src + (ym * w) * CH;
    const T* rp = src + (yp * w) * CH;
    float dx = 0.f, dy = 0.f;
    if constexpr (sizeof(T) == 1) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int h = (int)r0[xp * CH + c] - (int)r0[xm * CH + c];
            const int v = (int)rp[x * CH + c] - (int)rm[x * CH + c];
            dx = dx + (float)(h * h);
            dy = dy + (float)(v * v);
        }
    } else if constexpr (FMA) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const float h = r0[xp * CH + c] - r0[xm * CH + c];
            dx = __builtin_fmaf(h, h, dx);
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const float v = rp[x * CH + c] - rm[x * CH + c];
            dy = __builtin_fmaf(v, v, dy);
        }
    } else {
        // include/cpp/gradient.hpp:16-25: sum += h*h + v*v per channel
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const float h = r0[xp * CH + c] - r0[xm * CH + c];
            const float v = rp[x * CH + c] - rm[x * CH + c];
            s = s + (h * h + v * v);
        }
        dst[y * w + x] = __builtin_sqrtf(s);
        return;
    }
    dst[y * w + x] = __builtin_sqrtf(dx + dy);
}

template <typename T, int CH, bool FMA>
static int launch_gradient_t(const T* src, float* dst, int width, int height, hipStream_t stream) {
    dim3 grid((width + 63) / 64, (height + 3) / 4);
    launch(gradient_kernel<T, CH, FMA>, grid, dim3(256), 0, stream, src, dst, width, height);
    return (int)hipGetLastError();
}

int launch_gradient_u8(const uint8_t* src, float* dst, int width, int height, int ch, hipStream_t stream) {
    if (ch == 1) return launch_gradient_t<uint8_t, 1, true>(src, dst, width, height, stream);
    if (ch == 3) return launch_gradient_t<uint8_t, 3, true>(src, dst, width, height, stream);
    return VIP_ERR_INVALID_ARGUMENT;
}

int launch_gradient_f32(const float* src, float* dst, int width, int height, int ch, bool fma, hipStream_t stream) {
    if (ch == 1) return fma ? launch_gradient_t<float, 1, true>(src, dst, width, height, stream)
                            : launch_gradient_t<float, 1, false>(src, dst, width, height, stream);
    if (ch == 3) return fma ? launch_gradient_t<float, 3, true>(src, dst, width, height, stream)
                            : launch_gradient_t<float, 3, false>(src, dst, width, height, stream);
    return VIP_ERR_INVALID_ARGUMENT;
}

// ---------------------------------------------------------------------------
// blur + mRTV: 64 x 4 outputs per block, (64+2r) x (4+2r) halo tile in LDS
// (image as RGBX words, magnitude as f32), one thread per output pixel.
// ---------------------------------------------------------------------------
constexpr int kBlurTW = 64, kBlurTH = 4;

template <bool CPP>
__global__ __launch_bounds__(256) void blur_rtv_kernel(const uint8_t* __restrict__ img, const float* __restrict__ mag,
                                                      float* __restrict__ blurred, float* __restrict__ rtv, int width,
                                                      int height, int ksize) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int radius = ksize / 2;
    const int tw = kBlurTW + 2 * radius, th = kBlurTH + 2 * radius;
    uint32_t* s_img = lds;
    float* s_mag = reinterpret_cast<float*>(lds + tw * th);
    const int x0 = blockIdx.x * kBlurTW, y0 = blockIdx.y * kBlurTH;
    for (int i = threadIdx.x; i < tw * th; i += 256) {
        const int r = i / tw, c = i - r * tw;
        const int yc = clampi(y0 - radius + r, 0, height - 1);
        const int xc = clampi(x0 - radius + c, 0, width - 1);
        const uint8_t* p = img + ((long long)yc * width + xc) * 3;
        s_img[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
        s_mag[i] = mag[(long long)yc * width + xc];
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int x = x0 + tx, y = y0 + ty;
    if (x >= width || y >= height) return;
    // channel sums are exact integers (== the reference's float sums, all < 2^24);
    // intensity extremes come from integer byte sums: x -> float(x)/3.f is monotonic,
    // so max_i(s_i/3.f) == (max_i s_i)/3.f and one divide replaces k*k of them
    // window 2*(ksize/2)+1 wide; the divisor below is ksize^2 even for even ksize
    const int kw = 2 * radius + 1;
    uint32_t s0 = 0, s1 = 0, s2 = 0, smax = 0, smin = 0xffffffffu;
    float mmax = 0.f, msum = 0.f;
    for (int ky = 0; ky < kw; ++ky) {
        const uint32_t* ri = s_img + (ty + ky) * tw + tx;
        const float* rm = s_mag + (ty + ky) * tw + tx;
        for (int kx = 0; kx < kw; ++kx) {
            const uint32_t p = ri[kx];
            s0 += p & 0xffu;
            s1 += (p >> 8) & 0xffu;
            s2 += (p >> 16) & 0xffu;
            const uint32_t s = __builtin_amdgcn_sad_u8(p, 0u, 0u);
            smax = s > smax ? s : smax;
            smin = s < smin ? s : smin;
            const float m = rm[kx];
            mmax = mmax < m ? m : mmax;
            msum = msum + m;  // row-major order, as the reference accumulates
        }
    }
    const float kk = (float)(ksize * ksize);
    float* b = blurred + ((long long)y * width + x) * 3;
    b[0] = (float)s0 / kk;
    b[1] = (float)s1 / kk;
    b[2] = (float)s2 / kk;
    const float imax = (float)(int)smax / 3.f, imin = (float)(int)smin / 3.f;
    const float num = (imax - imin) * mmax;
    rtv[(long long)y * width + x] = CPP ? num / (msum + 1e-9f) : (float)((double)num / ((double)msum + 1e-9));
}

int launch_blur_rtv(const uint8_t* img, const float* mag, float* blurred, float* rtv, int width, int height,
                    int ksize, bool cpp, hipStream_t stream) {
    const int radius = ksize / 2;
    const int lds = (kBlurTW + 2 * radius) * (kBlurTH + 2 * radius) * 8;
    dim3 grid((width + kBlurTW - 1) / kBlurTW, (height + kBlurTH - 1) / kBlurTH);
    if (cpp)
        launch(blur_rtv_kernel<true>, grid, dim3(256), lds, stream, img, mag, blurred, rtv, width, height,
                           ksize);
    else
        launch(blur_rtv_kernel<false>, grid, dim3(256), lds, stream, img, mag, blurred, rtv, width, height,
                           ksize);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// guide: first strict argmin of rtv over the clamped k x k window, alpha blend.
// ---------------------------------------------------------------------------
template <bool CPP>
__global__ __launch_bounds__(256) void guide_kernel(const float* __restrict__ blurred, const float* __restrict__ rtv,
                                                   uint8_t* __restrict__ guide, int width, int height, int ksize) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int radius = ksize / 2;
    const int tw = kBlurTW + 2 * radius, th = kBlurTH + 2 * radius;
    float* s_rtv = reinterpret_cast<float*>(lds);
    const int x0 = blockIdx.x * kBlurTW, y0 = blockIdx.y * kBlurTH;
    for (int i = threadIdx.x; i < tw * th; i += 256) {
        const int r = i / tw, c = i - r * tw;
        const int yc = clampi(y0 - radius + r, 0, height - 1);
        const int xc = clampi(x0 - radius + c, 0, width - 1);
        s_rtv[i] = rtv[(long long)yc * width + xc];
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int x = x0 + tx, y = y0 + ty;
    if (x >= width || y >= height) return;
    // CUDA initialises with 1e10f (:152), include/cpp with FLT_MAX (:97)
    float rmin = CPP ? 3.402823466e+38f : 1e10f;
    int mx = 0, my = 0;
    const int kw = 2 * radius + 1;  // window; sigma_alpha below uses ksize (even ksize too)
    for (int ky = 0; ky < kw; ++ky) {
        const float* rr = s_rtv + (ty + ky) * tw + tx;
        for (int kx = 0; kx < kw; ++kx) {
            const float v = rr[kx];
            if (rmin > v) {
                rmin = v;
                mx = kx;
                my = ky;
            }
        }
    }
    const int gx = clampi(x - radius + mx, 0, width - 1);
    const int gy = clampi(y - radius + my, 0, height - 1);
    const float sigma_alpha = 1.f / (float)(5 * ksize);
    const float arg = sigma_alpha * (s_rtv[(ty + radius) * tw + tx + radius] - rmin);
    const float e = (float)exp((double)arg);
    const float alpha = 2.f / (1.f + e) - 1.f;
    const float beta = 1.f - alpha;
    const float* bm = blurred + ((long long)gy * width + gx) * 3;
    const float* bc = blurred + ((long long)y * width + x) * 3;
    uint8_t* g = guide + ((long long)y * width + x) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v = CPP ? (alpha * bm[c] + beta * bc[c]) + 0.5f : __builtin_fmaf(alpha, bm[c], beta * bc[c]) + 0.5f;
        g[c] = (uint8_t)clampi((int)v, 0, 255);
    }
}

int launch_guide(const float* blurred, const float* rtv, uint8_t* guide, int width, int height, int ksize, bool cpp,
                 hipStream_t stream) {
    const int radius = ksize / 2;
    const int lds = (kBlurTW + 2 * radius) * (kBlurTH + 2 * radius) * 4;
    dim3 grid((width + kBlurTW - 1) / kBlurTW, (height + kBlurTH - 1) / kBlurTH);
    if (cpp)
        launch(guide_kernel<true>, grid, dim3(256), lds, stream, blurred, rtv, guide, width, height, ksize);
    else
        launch(guide_kernel<false>, grid, dim3(256), lds, stream, blurred, rtv, guide, width, height, ksize);
    return (int)hipGetLastError();
}

}  // namespace vip

namespace vip {

// ---------------------------------------------------------------------------
// Fused guide stage of one bilateral-texture iteration: X (u8x3) -> G (u8x3).
// gradient (src/gradient_impl.cu:7-66) -> box blur + mRTV
// (src/bilateral_texture_filter_impl.cu:10-104) -> argmin/alpha blend (:106-177),
// all in LDS: blurred and rtv never reach HBM (reads 3 B/px + halo, writes 3 B/px).
//
// Regions around the output tile T (64 x 16), R = ksize/2, each stored
// PRE-CLAMPED: entry q holds the stage's value at clamp(q), which is exactly what
// the reference stage reads through its own clamped coordinates. Inner loops then
// index the regions directly; a position outside the image only clamps its
// centre once.
//   XR : image pixels as RGBX words, T (+) (2R+1) (origin 4-px aligned)
//   MR : gradient magnitude, T (+) 2R
//   H  : horizontal window aggregates of the image rows of T (+) 2R at the blur
//        columns of T (+) R: {R|B<<16 sums, max|(1023-min)<<16 of the byte sums
//        r+g+b, G sums as u16} -- the separable part of the box blur and of the
//        intensity extremes (integer sums and max/min are order-free, so exact).
//        2.5 words per position, and MR stored over XR, keep the tile at 26 KiB:
//        6 workgroups per CU
//   BR, RR : blurred RGB and rtv, T (+) R (aliases XR/H once those are consumed)
// The magnitude sum is NOT separable: it is accumulated per blur position in the
// reference's row-major order. Bit-exact with the stage kernels: x/3.f is
// monotonic (extremes of integer sums), float divides by the constants ksize^2
// and 3 use an fma-corrected reciprocal that equals the correctly rounded
// quotient on every reachable numerator (verified exhaustively,
// tests/test_oracle.py::test_constant_division_is_exact), rtv divide in double
// (CUDA profile).
// ---------------------------------------------------------------------------
// Guide tile (TW x TH outputs) and workgroup size, per radius. The phases run one
// work item per thread where the counts allow it: 4 vertically adjacent blur
// positions per pass-2 run, 4 vertically adjacent guide outputs per guide run, so a
// (TW + 2R) x (TH + 2R) blur region of up to 1024 pass-2 runs fills 1024 threads once.
// 92 x 36 at R = 2 (k = 5, C4): 96 x 40 blur positions = 960 pass-2 runs (1.159 per
// output), 828 guide runs, 2160 = 60 tile rows exactly, 75 KiB of LDS -> two 16-wave
// workgroups per CU. Measured per 4K iteration (guide stage + JBF, round 2,
// profiles/r02_variants.txt): 64 x 16 / 256 threads 158.4-159.7 us, 124 x 28 / 1024
// 150.3-150.7 us (60 x 60: 157.5, 28 x 124: 154.2, 252 x 12: 177.0, 60 x 28 / 512: 165.3);
// round 5, per C4 frame on one stream, interleaved on one box
// (profiles/r05_gf_tiles_{a,b,c}.txt): 92 x 36 656.1-661.0 us against 124 x 28
// 661.7-667.2 (96 x 36 668-671, 124 x 24 673, 108 x 32 678-680, 80 x 40 697, 80 x 44 692,
// 60 x 60 693). VIP_GF_TW / _TH / _NT override R <= 2.
struct GfTile { int tw, th, nt; };
// Tiles per radius for R > 2 (texture ksize 6..24; the reference's default ksize 9 is R = 4).
// Round 6, kernel-stamped 4K launches interleaved on one box against the 64 x 16 / 256-thread
// tile (profiles/r06_guide_tiles_big_r_ab{,2}.txt): R = 3 92 x 32 / 1024 110.7 -> 91.1 us (fewer
// blur positions per output: 1.33 against 1.64); R = 4 the same tile with its VGPRs capped at 64
// (two workgroups per CU, 10 spilled) 134.4 -> 110.5; R = 5 92 x 32 216.6 -> 192.3 (uncapped:
// capped spills 37 and runs 211.5); R = 6 keeps 64 x 16 (60 x 36: 300.5, capped 261.6 against
// 263.8); R = 7 60 x 36 capped (49 spilled) 446.7 -> 394.5. Knobs: VIP_GF_T<R> = GfTile{tw, th,
// nt}, VIP_GF_WPE<R> = minimum waves per SIMD (8 caps the VGPRs at 64).
#ifndef VIP_GF_T3
#define VIP_GF_T3 GfTile{92, 32, 1024}
#endif
#ifndef VIP_GF_T4
#define VIP_GF_T4 GfTile{92, 32, 1024}
#endif
#ifndef VIP_GF_T5
#define VIP_GF_T5 GfTile{92, 32, 1024}
#endif
#ifndef VIP_GF_T6
#define VIP_GF_T6 GfTile{64, 16, 256}
#endif
#ifndef VIP_GF_T7
#define VIP_GF_T7 GfTile{60, 36, 1024}
#endif
#ifndef VIP_GF_WPE4
#define VIP_GF_WPE4 8
#endif
#ifndef VIP_GF_WPE5
#define VIP_GF_WPE5 1
#endif
#ifndef VIP_GF_WPE6
#define VIP_GF_WPE6 1
#endif
#ifndef VIP_GF_WPE7
#define VIP_GF_WPE7 8
#endif
constexpr GfTile gf_tile(int R) {
#if defined(VIP_GF_TW) && defined(VIP_GF_TH) && defined(VIP_GF_NT)
    if (R <= 2) return GfTile{VIP_GF_TW, VIP_GF_TH, VIP_GF_NT};
#else
    if (R <= 2) return GfTile{92, 36, 1024};
#endif
    switch (R) {
        case 3: return VIP_GF_T3;
        case 4: return VIP_GF_T4;
        case 5: return VIP_GF_T5;
        case 6: return VIP_GF_T6;
        case 7: return VIP_GF_T7;
        default: return GfTile{64, 16, 256};
    }
}
// minimum waves per SIMD the guide-stage kernel of radius R is compiled for (1: no cap)
constexpr int gf_min_waves(int R) {
    return R == 4 ? VIP_GF_WPE4 : R == 5 ? VIP_GF_WPE5 : R == 6 ? VIP_GF_WPE6 : R == 7 ? VIP_GF_WPE7 : 1;
}
constexpr int kGfH1 = 8;   // pass 1: horizontally adjacent window aggregates per thread
constexpr int kGfV2 = 4;   // pass 2: vertically adjacent blur positions per thread
constexpr int kGfRun = 4;  // guide: vertically adjacent outputs per thread

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// MRSEP_: the magnitudes get their own region beside XR (written as they are computed, no
// barrier between pass 1 and their store), when two workgroups still fit a CU.
template <int R, int TW_, int TH_, int NT_, bool MRSEP_ = false>
struct GfGeomT {
    static constexpr int TW = TW_, TH = TH_, NT = NT_;
    static constexpr bool MRSEP = MRSEP_;
    static_assert(TW % 4 == 0 && TH % 4 == 0, "guide tile: 4-pixel groups, 4-row runs");
    static constexpr int K = 2 * R + 1;
    static constexpr int BW = TW + 2 * R;               // BR/RR: T (+) R
    static constexpr int BH = TH + 2 * R;
    static constexpr int BHP = round_up(BH, kGfV2);     // + pass-2 overhang rows
    static constexpr int HWP = round_up(BW, kGfH1);     // H: blur columns, rows of T (+) 2R
    static constexpr int HH = BHP + 2 * R;
    static constexpr int MW = round_up(BW + 2 * R, 4);  // MR: T (+) 2R
    static constexpr int MH = HH;
    static constexpr int XL = round_up(2 * R + 1, 4);   // XR left apron (4-px aligned origin)
    static constexpr int XW = round_up(cmax(MW - 2 * R + XL + 1, HWP + XL), 4);
    static constexpr int XH = MH + 2;
    static constexpr int XR_WORDS = XW * XH;
    static constexpr int HPL = HWP * HH;                // one H plane
    static constexpr int BPL = BW * BHP;                // one BR/RR plane
    // XR, then MR in its place (gradients wait in registers until XR is consumed) or, with
    // MRSEP, beside it; H after them (RB, MX words + G as u16); BR/RR and the guide tile GT
    // reuse it all
    static constexpr int MR_AT = MRSEP ? XR_WORDS : 0;
    static constexpr int H_AT = XR_WORDS + (MRSEP ? MW * MH : 0);
    static constexpr int A_WORDS = cmax(H_AT + 2 * HPL + HPL / 2, 4 * BPL + TW * TH);
    static constexpr int WORDS = A_WORDS;
    // the exp table (64 doubles) after every region, read by the guide phase
    static constexpr int ETAB = round_up(WORDS, 4);
    static constexpr int WORDS_ALL = ETAB + 128;
    static_assert(MRSEP || MW * MH <= XR_WORDS, "MR reuses the XR region");
    static constexpr int NR1 = HH * (HWP / kGfH1);      // pass-1 runs
    static constexpr int NR2 = BW * (BHP / kGfV2);      // pass-2 runs
    static constexpr int IT2 = (NR2 + NT - 1) / NT;
};
// Measurement knob VIP_GF_MR_SEP: MR beside XR at R = 2 (92 x 36: 80,224 bytes, still two
// workgroups per CU), one barrier and the MR store phase fewer -- bit-exact and slower:
// 67.8-68.3 against 65.4-65.9 us per 4K launch, interleaved (profiles/r06_guide_barrier_cuts_ab.txt)
#ifdef VIP_GF_MR_SEP
constexpr bool kGfMrSep2 = true;
#else
constexpr bool kGfMrSep2 = false;
#endif
template <int R>
using GfGeom = GfGeomT<R, gf_tile(R).tw, gf_tile(R).th, gf_tile(R).nt, R == 2 && kGfMrSep2>;

typedef short gf_s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short gf_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(gf_u16x2, a),
                                                                  __builtin_bit_cast(gf_u16x2, b)));
}

// N sliding maxima (any associative, idempotent op) of K consecutive terms: blocks of
// K, suffix scans inside a block and prefix scans into the next, window j =
// op(suffix[j], prefix[j + K - 1]) (van Herk / Gil-Werman).
template <int N, int K, class T, class Op>
__device__ __forceinline__ void win_op(const T (&x)[N + K - 1], T (&o)[N], Op op) {
    constexpr int M = N + K - 1;
    T suf[M], pre[M];
#pragma unroll
    for (int b0 = 0; b0 < M; b0 += K) {
        const int b1 = (b0 + K < M ? b0 + K : M) - 1;
        suf[b1] = x[b1];
#pragma unroll
        for (int t = b1 - 1; t >= b0; --t) suf[t] = op(x[t], suf[t + 1]);
        pre[b0] = x[b0];
#pragma unroll
        for (int t = b0 + 1; t <= b1; ++t) pre[t] = op(pre[t - 1], x[t]);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = (j % K == 0) ? suf[j] : op(suf[j], pre[j + K - 1]);
}

#ifdef VIP_GF_STAMPS
// diagnostic build only: [workgroup][wave][16] shader-clock stamps -- kernel entry (0),
// the arrival of each wave at each of the 6 phase barriers (1-6), exit (7), XR loads
// issued (8), gradients done (9)
__device__ unsigned long long vip_gf_stamps[4096 * 16 * 16];
#define VIP_GF_STAMP(k)                                                                             \
    do {                                                                                            \
        const int wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                         \
        if ((threadIdx.x & 63) == 0 && wg_ < 4096)                                                  \
            vip_gf_stamps[(wg_ * 16 + (threadIdx.x >> 6)) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define VIP_GF_STAMP(k)
#endif

// Progress-based wave priority inside the long phases (set_progress_priority in
// vip_stencil.hpp): band 0..3 as the thread advances through its gradients, pass-3 rows
// and guide outputs, so the waves of a workgroup reach each phase barrier together.
// Measured 733 -> 714 us per 4K k=5 nitr=5 frame (profiles/r02_variants.txt).
#ifndef VIP_GF_NO_PRIO
#define VIP_GF_PROGRESS(band) set_progress_priority(band)
#else
#define VIP_GF_PROGRESS(band)
#endif

// Phase 1 of a guide tile. issue() starts the global loads of the XR region of the tile with origin (x0, y0) into
// registers (4-pixel groups, dword loads when interior and aligned, clamped bytes otherwise;
// every load of the thread issued before any is unpacked: one HBM latency per tile, not one
// per group), commit() unpacks them into XR as RGBX words.
template <class G, int R>
struct XrLoad {
    static constexpr int NG = G::XH * (G::XW / 4);
    static constexpr int KG = (NG + G::NT - 1) / G::NT;
    uint32_t raw[KG][3];

    __device__ __forceinline__ void issue(const uint8_t* __restrict__ img, int width, int lo, int hi, int aligned,
                                          int x0, int y0, int tid) {
        const int xr0 = x0 - G::XL, yr0 = y0 - 2 * R - 1;
        const int W1 = width - 1;
#pragma unroll
        for (int k = 0; k < KG; ++k) {
            const int g = tid + k * G::NT;
            if (NG % G::NT != 0 && g >= NG) continue;
            const int ry = g / (G::XW / 4), gx = g - ry * (G::XW / 4);
            const uint8_t* row = img + (long long)clampi(yr0 + ry, lo, hi - 1) * width * 3;
            const int x = xr0 + 4 * gx;
#ifdef VIP_GF_ABL_LOAD  // timing ablation only (wrong output): no HBM reads
            if (true) {
                raw[k][0] = g * 0x01010101u;
                raw[k][1] = (g + x) * 0x01010101u;
                raw[k][2] = (g ^ 7) * 0x01010101u;
            } else
#endif
#ifdef VIP_GF_ISA_HOT  // ISA-count builds only (scripts/isa_classes.py): the interior path alone
            if (true) {
#else
            if ((aligned & 1) && x >= 0 && x + 3 <= W1) {
#endif
                const uint32_t* w = reinterpret_cast<const uint32_t*>(row + 3 * x);
                raw[k][0] = w[0];
                raw[k][1] = w[1];
                raw[k][2] = w[2];
            } else {
                const uint32_t q0 = load_rgb(row, clampi(x, 0, W1)), q1 = load_rgb(row, clampi(x + 1, 0, W1));
                const uint32_t q2 = load_rgb(row, clampi(x + 2, 0, W1)), q3 = load_rgb(row, clampi(x + 3, 0, W1));
                raw[k][0] = q0 | (q1 << 24);
                raw[k][1] = (q1 >> 8) | (q2 << 16);
                raw[k][2] = (q2 >> 16) | (q3 << 8);
            }
        }
    }
    __device__ __forceinline__ void commit(uint32_t* XR, int tid) const {
#pragma unroll
        for (int k = 0; k < KG; ++k) {
            const int g = tid + k * G::NT;
            if (NG % G::NT != 0 && g >= NG) continue;
            const int ry = g / (G::XW / 4), gx = g - ry * (G::XW / 4);
            *reinterpret_cast<uint4*>(XR + ry * G::XW + 4 * gx) = unpack_rgb4(raw[k][0], raw[k][1], raw[k][2]);
        }
    }
};

// Row bands: rows [lo, hi) of the (dense, width*3 pitch) buffers are the valid
// frame rows -- every stage clamps into them, as the reference clamps into
// [0, height) -- and guide rows [gy0, gy1) are produced (a row slab of a sharded
// frame; the whole frame is lo = gy0 = 0, hi = gy1 = height).
// Phases 1-4 of one guide tile: G::TW x G::TH guide outputs with origin (x0, y0) in
// image coordinates, from the image rows [lo, hi) (every read clamps into them) in
// the G::WORDS words of LDS at `lds`; rows >= gy1 and columns past the image are not
// produced. Each guide word (RGBX) goes to sink(ty, tx, word), tile-relative. Ends
// after the guide phase WITHOUT a barrier (the caller's sink target decides).
// (A persistent guide kernel that issues its next tile's XrLoad right before the guide phase
// needs 72 more VGPRs than the 64 of two workgroups per CU and spills them: measured in round
// 6 at the compiler's resource report, not built.)
template <class G, int R, bool CPP, bool OPAQUE_TID = false, class Sink>
__device__ __forceinline__ void guide_tile(uint32_t* lds, const uint8_t* __restrict__ img, int width, int lo, int hi,
                                           int gy1, int ksize, int aligned, int x0, int y0, Sink&& sink) {
    constexpr int K = G::K;  // window width; the reference divides by ksize^2 and
                             // uses sigma_alpha = 1/(5 ksize) even when ksize is even
    constexpr bool PACKRB = K * K * 255 < 65536;  // R|B<<16 vertical sums stay in 16 bits
    uint32_t* XR = lds;
    uint32_t* H = lds + G::H_AT;                        // RB plane, MX plane (HPL words each)
    uint16_t* HG = reinterpret_cast<uint16_t*>(H + 2 * G::HPL);  // G sums (<= K * 255) as u16
    float* BR = reinterpret_cast<float*>(lds);          // 3 planes of BPL, aliases XR/H
    float* RR = BR + 3 * G::BPL;
    float* MR = reinterpret_cast<float*>(lds + G::MR_AT);  // (aliased: written once XR is consumed)
    double* const etab = reinterpret_cast<double*>(lds + G::ETAB);  // kExp2Tab64
    // OPAQUE_TID (the fused iteration kernel, which calls this three times): without it
    // the compiler keeps chunk 0's thread-index arithmetic live across the later chunks
    // (18 spilled VGPRs, ~90 MB of scratch writes per 4K launch); recomputing is cheaper.
    // The single-call guide stage keeps the plain index (and its known range).
    int tid = threadIdx.x;
    if constexpr (OPAQUE_TID) {
        __asm__ volatile("" : "+v"(tid));
        __builtin_assume(tid >= 0 && tid < G::NT);
    }
    // region origins (image coordinates)
    const int xr0 = x0 - G::XL, yr0 = y0 - 2 * R - 1;
    const int mr0x = x0 - 2 * R, mr0y = y0 - 2 * R;
    const int W1 = width - 1, H0 = lo, H1 = hi - 1;

    // 1. XR: 4-pixel groups (XrLoad)
    {
        XrLoad<G, R> xl;
        xl.issue(img, width, lo, hi, aligned, x0, y0, tid);
        VIP_GF_STAMP(8);
#ifndef VIP_GF_EXP_OCML
        if (tid < 64) etab[tid] = kExp2Tab64[tid];  // read in phase 4, after several barriers
#endif
        xl.commit(XR, tid);
        VIP_GF_STAMP(1);
        __syncthreads();
    }

    // 2a. MR[q] = gradient at c = clamp(q); XR is pre-clamped, so c's neighbours are
    //     read directly (XR[c +- e] == X(clamp(c +- e))). sum_c h^2 + v^2 is an exact
    //     integer (< 2^24), equal to the reference's float sums: v_dot2 on the
    //     {c0, c2} 16-bit difference pairs, a mad for c1.
    constexpr int NM = G::MW * G::MH, KM = (NM + G::NT - 1) / G::NT;
    float mrv[G::MRSEP ? 1 : KM];  // aliased MR: this thread's gradients, stored over XR after pass 1
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        VIP_GF_PROGRESS(k * 4 / KM);
        const int i = tid + k * G::NT;
        if (NM % G::NT != 0 && i >= NM) continue;
        const int qy = i / G::MW, qx = i - qy * G::MW;
        const int cx = clampi(mr0x + qx, 0, W1) - xr0, cy = clampi(mr0y + qy, H0, H1) - yr0;
        const uint32_t* c = XR + cy * G::XW + cx;
        const uint32_t L = c[-1], Rt = c[1], U = c[-G::XW], D = c[G::XW];
        const gf_s16x2 h02 = __builtin_bit_cast(gf_s16x2, Rt & 0x00ff00ffu) - __builtin_bit_cast(gf_s16x2, L & 0x00ff00ffu);
        const gf_s16x2 v02 = __builtin_bit_cast(gf_s16x2, D & 0x00ff00ffu) - __builtin_bit_cast(gf_s16x2, U & 0x00ff00ffu);
        const int h1 = (int)__builtin_amdgcn_ubfe(Rt, 8, 8) - (int)__builtin_amdgcn_ubfe(L, 8, 8);
        const int v1 = (int)__builtin_amdgcn_ubfe(D, 8, 8) - (int)__builtin_amdgcn_ubfe(U, 8, 8);
        const int ss = __builtin_amdgcn_sdot2(h02, h02, __builtin_amdgcn_sdot2(v02, v02, h1 * h1 + v1 * v1, false),
                                              false);
#ifdef VIP_GF_LLVM_SQRT  // the compiler's correctly rounded expansion (same result, 17 VALU)
        const float mag = __builtin_sqrtf((float)ss);
#else
        const float mag = sqrt_int_exact((float)ss);  // == sqrtf, exhaustively checked (microbench/div_check)
#endif
        if constexpr (G::MRSEP)
            MR[i] = mag;
        else
            mrv[k] = mag;
    }
    VIP_GF_STAMP(9);
    // 2b. pass 1: H = horizontal K-window aggregates, kGfH1 adjacent columns per thread.
    //     H row h <-> image row y0 - 2R + h (XR row h + 1); H column c <-> image column
    //     x0 - R + c, window XR columns c + XL - 2R .. c + XL.
    for (int run = tid; run < G::NR1; run += G::NT) {
        const int hr = run / (G::HWP / kGfH1), hc0 = (run - hr * (G::HWP / kGfH1)) * kGfH1;
        const uint32_t* xrow = XR + (hr + 1) * G::XW + hc0 + G::XL - 2 * R;
        constexpr int NX = kGfH1 + K - 1;
        uint32_t rb[NX], gg[NX], mx[NX];
#pragma unroll
        for (int t = 0; t < NX; ++t) {
            const uint32_t p = xrow[t];
            const uint32_t sb = __builtin_amdgcn_sad_u8(p, 0u, 0u);  // r + g + b
            rb[t] = p & 0x00ff00ffu;
            gg[t] = __builtin_amdgcn_ubfe(p, 8, 8);
            mx[t] = ((sb ^ 1023u) << 16) | sb;  // max of lo = max s, max of hi = 1023 - min s
        }
        uint32_t orb[kGfH1], og[kGfH1], omx[kGfH1];
        win_sum<kGfH1, K>(rb, orb);
        win_sum<kGfH1, K>(gg, og);
        win_op<kGfH1, K>(mx, omx, pk_max_u16);
        uint32_t* h = H + hr * G::HWP + hc0;
        static_assert(kGfH1 == 8, "one b128 store of 8 u16 G sums");
        *reinterpret_cast<uint4*>(HG + hr * G::HWP + hc0) =
            make_uint4(og[0] | (og[1] << 16), og[2] | (og[3] << 16), og[4] | (og[5] << 16), og[6] | (og[7] << 16));
#pragma unroll
        for (int j = 0; j < kGfH1; j += 4) {
            *reinterpret_cast<uint4*>(h + j) = make_uint4(orb[j], orb[j + 1], orb[j + 2], orb[j + 3]);
            *reinterpret_cast<uint4*>(h + G::HPL + j) = make_uint4(omx[j], omx[j + 1], omx[j + 2], omx[j + 3]);
        }
    }
    VIP_GF_STAMP(2);
    __syncthreads();  // XR is consumed (gradients and pass 1): MR takes its place
    if constexpr (!G::MRSEP) {
        VIP_GF_PROGRESS(0);
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            const int i = tid + k * G::NT;
            if (NM % G::NT != 0 && i >= NM) continue;
            MR[i] = mrv[k];
        }
        VIP_GF_STAMP(3);
        __syncthreads();
    }

    // 3. pass 2: blur + mRTV at the BR positions, kGfV2 vertically adjacent positions per
    //    thread (vertical windows of H, magnitude sums in row-major order). Blur
    //    position (p, c) <-> image (y0 - R + p, x0 - R + c): H rows p .. p + 2R, column c;
    //    MR rows p .. p + 2R, columns c .. c + 2R. Results stay in registers until every
    //    thread is done with H (BR/RR alias it).
    const float kk = (float)(ksize * ksize);
    // == 1.f / kk (RN(1/k) for every float k in [1, 2^38), microbench/div_check), 3 VALU
    // instead of the IEEE division's ~10
#ifndef VIP_GF_FAST_DIV
    const float rkk = 1.f / kk;
#else  // measurement knob, same values: 3 VALU instead of the IEEE division's ~10, but the
       // C4 frame measured 0.4 % slower with it and rtv_quotient (profiles/r04_gf_fast_div.txt)
    const float rkk = recip_exact(kk);
#endif
    constexpr float kThird = 0x1.555556p-2f;  // RN(1/3)
    float res[G::IT2][kGfV2][4];
#pragma unroll
    for (int it = 0; it < G::IT2; ++it) {
        const int run = tid + it * G::NT;
        if (G::NR2 % G::NT != 0 && run >= G::NR2) continue;
        const int c = run % G::BW, p0 = (run / G::BW) * kGfV2;
        const int ix = x0 - R + c, iy0 = y0 - R + p0;
        uint32_t s0[kGfV2], s1[kGfV2], s2[kGfV2], smx[kGfV2];
        float mmax[kGfV2], msum[kGfV2];
#ifdef VIP_GF_ISA_HOT
        if (true) {
#else
        if (ix >= 0 && ix <= W1 && iy0 >= H0 && iy0 + kGfV2 - 1 <= H1) {
#endif
            constexpr int NV = kGfV2 + K - 1;
            uint32_t hrb[NV], hg[NV], hmx[NV];
            // magnitudes are finite and >= +0: their bit patterns order like their values, so
            // the extremes are integer max3s (no NaN canonicalising of LDS loads)
            uint32_t rowmax[NV], mmaxb[kGfV2];
#pragma unroll
            for (int t = 0; t < NV; ++t) {
                hrb[t] = H[(p0 + t) * G::HWP + c];
                hg[t] = HG[(p0 + t) * G::HWP + c];
                hmx[t] = H[G::HPL + (p0 + t) * G::HWP + c];
            }
            if constexpr (PACKRB) {
                win_sum<kGfV2, K>(hrb, s0);
            } else {
                uint32_t hr_[NV], hb_[NV];
#pragma unroll
                for (int t = 0; t < NV; ++t) {
                    hr_[t] = hrb[t] & 0xffffu;
                    hb_[t] = hrb[t] >> 16;
                }
                win_sum<kGfV2, K>(hr_, s0);
                win_sum<kGfV2, K>(hb_, s2);
            }
            win_sum<kGfV2, K>(hg, s1);
            win_op<kGfV2, K>(hmx, smx, pk_max_u16);
#pragma unroll
            for (int t = 0; t < NV; ++t) {
                VIP_GF_PROGRESS(t * 4 / NV);
                const float* mrow = MR + (p0 + t) * G::MW + c;
                float m[K];
#pragma unroll
                for (int kx = 0; kx < K; ++kx) m[kx] = mrow[kx];
                uint32_t mx = __float_as_uint(m[0]);
#pragma unroll
                for (int kx = 1; kx < K; ++kx) {  // == the reference's max (no NaN)
                    const uint32_t b = __float_as_uint(m[kx]);
                    mx = mx > b ? mx : b;
                }
                rowmax[t] = mx;
                // window row t - j of output j, in the reference's row-major order
#pragma unroll
                for (int j = 0; j < kGfV2; ++j) {
                    if (t - j < 0 || t - j >= K) continue;
                    // the reference starts from 0.f; magnitudes are >= +0, so 0.f + m == m
                    msum[j] = t == j ? m[0] : msum[j] + m[0];
#pragma unroll
                    for (int kx = 1; kx < K; ++kx) msum[j] = msum[j] + m[kx];
                }
            }
            win_op<kGfV2, K>(rowmax, mmaxb, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
#pragma unroll
            for (int j = 0; j < kGfV2; ++j) mmax[j] = __uint_as_float(mmaxb[j]);
        } else {
            // a centre outside the image: the reference reads the stage values at the
            // clamped centre, whose window lies inside the pre-clamped regions
#pragma unroll
            for (int j = 0; j < kGfV2; ++j) {
                const int hrow = clampi(iy0 + j, H0, H1) - (y0 - 2 * R);  // H / MR row of the centre
                const int hcol = clampi(ix, 0, W1) - (x0 - R);            // H column; MR column hcol + R
                uint32_t a0 = 0, a1 = 0, a2 = 0, am = 0;
                float mm = 0.f, ms = 0.f;
                for (int ky = -R; ky <= R; ++ky) {
                    const int hi_ = (hrow + ky) * G::HWP + hcol;
                    const uint32_t rbv = H[hi_];
                    if constexpr (PACKRB) {
                        a0 += rbv;
                    } else {
                        a0 += rbv & 0xffffu;
                        a2 += rbv >> 16;
                    }
                    a1 += HG[hi_];
                    am = pk_max_u16(am, H[G::HPL + hi_]);
                    const float* mrow = MR + (hrow + ky) * G::MW + hcol;
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        mm = __builtin_fmaxf(mm, mrow[kx]);
                        ms = ms + mrow[kx];
                    }
                }
                s0[j] = a0;
                s1[j] = a1;
                s2[j] = a2;
                smx[j] = am;
                mmax[j] = mm;
                msum[j] = ms;
            }
        }
#pragma unroll
        for (int j = 0; j < kGfV2; ++j) {
            const uint32_t c0 = PACKRB ? (s0[j] & 0xffffu) : s0[j];
            const uint32_t c2 = PACKRB ? (s0[j] >> 16) : s2[j];
            res[it][j][0] = div_exact(c0, kk, rkk);
            res[it][j][1] = div_exact(s1[j], kk, rkk);
            res[it][j][2] = div_exact(c2, kk, rkk);
            const float imax = div_exact(smx[j] & 0xffffu, 3.f, kThird);
            const float imin = div_exact(1023u - (smx[j] >> 16), 3.f, kThird);
            const float num = (imax - imin) * mmax[j];
#ifdef VIP_GF_ABL_DIV  // timing ablation only (inexact): f32 divide instead of the double one
            res[it][j][3] = num / (msum[j] + 1e-9f);
#else
#ifndef VIP_GF_FAST_DIV
            res[it][j][3] = CPP ? num / (msum[j] + 1e-9f) : (float)((double)num / ((double)msum[j] + 1e-9));
#else
            res[it][j][3] = CPP ? num / (msum[j] + 1e-9f) : rtv_quotient((double)num, (double)msum[j] + 1e-9);
#endif
#endif
        }
    }
    VIP_GF_STAMP(4);
    __syncthreads();  // H and XR are consumed: BR/RR may overwrite them
#pragma unroll
    for (int it = 0; it < G::IT2; ++it) {
        const int run = tid + it * G::NT;
        if (G::NR2 % G::NT != 0 && run >= G::NR2) continue;
        const int c = run % G::BW, p0 = (run / G::BW) * kGfV2;
#pragma unroll
        for (int j = 0; j < kGfV2; ++j) {
            const int i = (p0 + j) * G::BW + c;
            BR[i] = res[it][j][0];
            BR[G::BPL + i] = res[it][j][1];
            BR[2 * G::BPL + i] = res[it][j][2];
            RR[i] = res[it][j][3];
        }
    }
    VIP_GF_STAMP(5);
    __syncthreads();

    // 4. guide: first strict argmin of rtv over the window (RR is pre-clamped, so the
    //    reference's clamped-coordinate scan is a direct row-major scan). A thread
    //    takes kGfRun vertically adjacent outputs: each window row's first argmin is
    //    found once and shared; scanning those rows in order with strict > then
    //    gives the row-major first argmin. Alpha blend per output.
#ifndef VIP_GF_FAST_DIV
    const float sigma_alpha = 1.f / (float)(5 * ksize);
#else
    const float sigma_alpha = recip_exact((float)(5 * ksize));  // == 1.f / (5 ksize), as rkk
#endif
    for (int run = tid; run < (G::TH / kGfRun) * G::TW; run += G::NT) {
        const int tx = run % G::TW, ty0 = (run / G::TW) * kGfRun;
        const int x = x0 + tx;
        if (x > W1 || y0 + ty0 >= gy1) continue;
#ifndef VIP_GF_ARGMIN_SCAN
        // rtv is finite and >= +0 (num >= 0, msum + 1e-9 > 0), so its bit patterns order
        // like its values: each row's minimum is an integer min3 (no NaN canonicalising),
        // its first position the lowest column holding that minimum -- the same position
        // as the reference's strict > scan. Every rtv is <= 255 < the scan's initial 1e10f
        // (FLT_MAX in the CPP profile), so that initial value never survives.
        uint32_t rv[kGfRun + 2 * R];
#ifndef VIP_GF_ARGMIN_LATE
        int ri[kGfRun + 2 * R];
#endif
#pragma unroll
        for (int t = 0; t < kGfRun + 2 * R; ++t) {  // window rows ty0-R .. ty0+kGfRun-1+R
            const float* row = RR + (ty0 + t) * G::BW + tx;
            uint32_t m[K];
#pragma unroll
            for (int kx = 0; kx < K; ++kx) m[kx] = __float_as_uint(row[kx]);
            uint32_t v = m[0];
#pragma unroll
            for (int kx = 1; kx < K; ++kx) v = v < m[kx] ? v : m[kx];
            rv[t] = v;
#ifndef VIP_GF_ARGMIN_LATE
            int c = K - 1;
#pragma unroll
            for (int kx = K - 2; kx >= 0; --kx) c = m[kx] == v ? kx : c;
            ri[t] = (ty0 + t) * G::BW + tx + c;
#endif
        }
#pragma unroll
        for (int j = 0; j < kGfRun; ++j) {
            VIP_GF_PROGRESS(j * 4 / kGfRun);
            const int y = y0 + ty0 + j;
            if (y >= gy1) break;
            uint32_t mb = rv[j];
#pragma unroll
            for (int ky = 1; ky < K; ++ky) mb = mb < rv[j + ky] ? mb : rv[j + ky];
#ifndef VIP_GF_ARGMIN_LATE
            int mi = ri[j + K - 1];
#pragma unroll
            for (int ky = K - 2; ky >= 0; --ky) mi = rv[j + ky] == mb ? ri[j + ky] : mi;
#else  // measurement knob: row minima only; the argmin's row, then its column, per output
            int roff = (j + K - 1) * G::BW;
#pragma unroll
            for (int ky = K - 2; ky >= 0; --ky) roff = rv[j + ky] == mb ? (j + ky) * G::BW : roff;
            const int rowi = ty0 * G::BW + tx + roff;
            uint32_t mm[K];
#pragma unroll
            for (int kx = 0; kx < K; ++kx) mm[kx] = __float_as_uint(RR[rowi + kx]);
            int c = K - 1;
#pragma unroll
            for (int kx = K - 2; kx >= 0; --kx) c = mm[kx] == mb ? kx : c;
            const int mi = rowi + c;
#endif
            const float rmin = __uint_as_float(mb);
#else  // the reference's scan: compare and select per position
        float rv[kGfRun + 2 * R];
        int ri[kGfRun + 2 * R];
#pragma unroll
        for (int t = 0; t < kGfRun + 2 * R; ++t) {  // window rows ty0-R .. ty0+kGfRun-1+R
            const float* row = RR + (ty0 + t) * G::BW + tx;
            float v = row[0];
            int c = 0;
#pragma unroll
            for (int kx = 1; kx < K; ++kx) {
                if (v > row[kx]) {
                    v = row[kx];
                    c = kx;
                }
            }
            rv[t] = v;
            ri[t] = (ty0 + t) * G::BW + tx + c;
        }
#pragma unroll
        for (int j = 0; j < kGfRun; ++j) {
            VIP_GF_PROGRESS(j * 4 / kGfRun);
            const int y = y0 + ty0 + j;
            if (y >= gy1) break;
            float rmin = CPP ? 3.402823466e+38f : 1e10f;
            int mi = 0;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                if (rmin > rv[j + ky]) {
                    rmin = rv[j + ky];
                    mi = ri[j + ky];
                }
            }
#endif
            const int ci = (ty0 + j + R) * G::BW + tx + R;
            const float arg = sigma_alpha * (RR[ci] - rmin);
#ifdef VIP_GF_ABL_EXP  // timing ablation only (inexact): hardware exp2
            const float e = __builtin_amdgcn_exp2f(arg * 1.44269504f);
#elif defined(VIP_GF_EXP_OCML)  // ocml's double exp
            const float e = (float)exp((double)arg);
#else
            // == (float)exp((double)arg) for every float arg in [0, 32) (microbench/div_check
            // on the GPU; microbench/exp_check against glibc, the oracle's exp)
            const float e = exp_tab_f32(arg, etab);
#endif
            // 2 / (1 + e) == 2 * RN(1 / (1 + e)) exactly (a power-of-two scale). e >= 1 and
            // arg <= 255 / (5 ksize) (rtv <= 255): 1 + e < 2^17 for ksize >= 5, < 2^37 at
            // ksize 2 (ksize 1: arg = 0). microbench/div_check verifies recip_exact for every
            // float in [1, 2^38)
            const float alpha = 2.f * recip_exact(1.f + e) - 1.f;
            const float beta = 1.f - alpha;
            uint32_t gw = 0;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float bm = BR[c * G::BPL + mi], bc = BR[c * G::BPL + ci];
                const float v = CPP ? (alpha * bm + beta * bc) + 0.5f : __builtin_fmaf(alpha, bm, beta * bc) + 0.5f;
                gw = pack_u8_clamped(v, c, gw);  // == clampi((int)v, 0, 255) << 8c
            }
            sink(ty0 + j, tx, gw);
        }
    }
}

// 5. guide tile -> HBM: 4 RGBX words -> 3 dwords per thread (byte stores at a ragged right
//    edge or an unaligned buffer)
template <class G>
__device__ __forceinline__ void store_guide_tile(const uint32_t* GT, uint8_t* __restrict__ guide, int width, int x0,
                                                 int y0, int gy1, int aligned, int tid) {
    const int W1 = width - 1;
    for (int q = tid; q < G::TH * (G::TW / 4); q += G::NT) {
        const int gr = q / (G::TW / 4), x = x0 + 4 * (q - gr * (G::TW / 4));
        const int y = y0 + gr;
        if (y >= gy1 || x > W1) continue;
        const uint4 w = *reinterpret_cast<const uint4*>(GT + gr * G::TW + (x - x0));
        uint8_t* row = guide + ((long long)y * width + x) * 3;
        if ((aligned & 2) && x + 3 <= W1) {
            uint32_t* d = reinterpret_cast<uint32_t*>(row);
            d[0] = w.x | (w.y << 24);
            d[1] = (w.y >> 8) | (w.z << 16);
            d[2] = (w.z >> 16) | (w.w << 8);
        } else {
            const uint32_t ws_[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (x + i > W1) break;
                row[3 * i] = (uint8_t)ws_[i];
                row[3 * i + 1] = (uint8_t)(ws_[i] >> 8);
                row[3 * i + 2] = (uint8_t)(ws_[i] >> 16);
            }
        }
    }
}

template <int R, bool CPP>
__global__ __launch_bounds__(GfGeom<R>::NT) __attribute__((amdgpu_waves_per_eu(gf_min_waves(R))))
void texture_guide_fused_kernel(const uint8_t* __restrict__ img,
                                                                   uint8_t* __restrict__ guide, int width, int lo,
                                                                   int hi, int gy0, int gy1, int ksize,
                                                                   int aligned) {
    using G = GfGeom<R>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int x0 = blockIdx.x * G::TW, y0 = gy0 + blockIdx.y * G::TH;
    const int tid = threadIdx.x;
    const int W1 = width - 1;
    VIP_GF_STAMP(0);
#ifdef VIP_GF_DIRECT_STORE
    // measurement knob: guide words straight to HBM -- a quad of lanes holds 4 horizontally
    // adjacent pixels (the guide runs are column-major in the lanes, TW % 4 == 0), lanes 0-2
    // of the quad store one dword each of the 12 bytes; byte stores at a ragged edge or an
    // unaligned buffer. No guide tile in LDS and no barrier after the guide phase; bit-exact
    // and 1 us slower per launch on top of VIP_GF_MR_SEP (profiles/r06_guide_barrier_cuts_ab.txt).
    static_assert(G::TW % 4 == 0, "whole quads per guide row");
    guide_tile<G, R, CPP>(lds, img, width, lo, hi, gy1, ksize, aligned, x0, y0, [&](int ty, int tx, uint32_t gw) {
        const uint32_t nx = (uint32_t)__builtin_amdgcn_mov_dpp((int)gw, 0xF9, 0xF, 0xF, false);  // quad_perm 1,2,3,3
        const int q = tx & 3, xq = x0 + tx - q;
        uint8_t* const orow = guide + ((long long)(y0 + ty) * width + xq) * 3;
        if ((aligned & 2) && xq + 3 <= W1) {
            if (q < 3) reinterpret_cast<uint32_t*>(orow)[q] = (gw >> (8 * q)) | (nx << (24 - 8 * q));
        } else {
            uint8_t* const o = orow + 3 * q;
            o[0] = (uint8_t)gw;
            o[1] = (uint8_t)(gw >> 8);
            o[2] = (uint8_t)(gw >> 16);
        }
    });
    (void)tid;
    VIP_GF_STAMP(6);
    VIP_GF_STAMP(7);
#else  // the guide tile through LDS, one barrier, then dword rows
    uint32_t* GT = lds + 4 * G::BPL;  // guide tile as RGBX words, after BR/RR
    guide_tile<G, R, CPP>(lds, img, width, lo, hi, gy1, ksize, aligned, x0, y0,
                          [&](int ty, int tx, uint32_t gw) { GT[ty * G::TW + tx] = gw; });
    VIP_GF_STAMP(6);
    __syncthreads();

    store_guide_tile<G>(GT, guide, width, x0, y0, gy1, aligned, tid);
    VIP_GF_STAMP(7);
#endif
}

template <int R, bool CPP>
static int launch_gf(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1, int ksize,
                     int aligned, hipStream_t stream) {
    using G = GfGeom<R>;
    constexpr int LDS = 4 * G::WORDS_ALL;
    static_assert(LDS <= kLdsBudget, "fused guide tile does not fit LDS");
    auto kern = texture_guide_fused_kernel<R, CPP>;
    static std::atomic<unsigned long long> attr_devs{0};
    if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), LDS, attr_devs)) return rc;
    note_launch(reinterpret_cast<const void*>(kern));
    if (gy1 <= gy0) return 0;
    dim3 grid((width + G::TW - 1) / G::TW, (gy1 - gy0 + G::TH - 1) / G::TH);
    launch(kern, grid, dim3(G::NT), LDS, stream, img, guide, width, lo, hi, gy0, gy1, ksize, aligned);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Streaming guide stage, R = 2 (ksize 4 and 5: C4) -- built, bit-exact, and SLOWER: 90.1
// against 65.0 us per 4K launch (profiles/r06_guide_stage_ab.txt), so it is a build knob
// (VIP_GF_STREAM), not the default. The rings cost 52 KiB per 512-thread workgroup, so only
// two workgroups share a CU at its 121 VGPRs (three at 80 VGPRs spill: 126.8 us); the guide
// and pass-2 phases then run on 2 of a SIMD's 4 waves, where the tiled stage runs each phase
// on all 8 -- the phases' LDS and f64 latency chains are no longer hidden. Same arithmetic
// as guide_tile, same bytes; a different schedule. One workgroup walks down a strip of GsTW output columns over
// a segment of rows, kGsV rows per step, and every phase of the stage is in flight in every
// step, each on its own row group (a software pipeline with one barrier per step):
//   A  image rows [Y0 + 5 + sV, +V): global loads issued at the top of step s, written to the
//      XR ring at its end (the loads fly under the step's compute)
//   B  rows [Y0 + 4 + (s-1)V, +V): gradient magnitudes (MR ring) and the horizontal K-window
//      aggregates of pass 1 (H ring), from XR rows stored by step s - 1
//   C  rows [Y0 + 2 + (s-2)V, +V): pass 2, box blur + mRTV (BR/RR rings), from H/MR rows of
//      step s - 1 (vertical windows of H, magnitude sums in the reference's row-major order)
//   D  rows [Y0 + (s-3)V, +V): the guide (first strict argmin, alpha blend) from BR/RR rows
//      of step s - 1, straight to HBM (a quad of lanes assembles 4 RGB pixels into 3 dwords)
// Each stage lags the one it reads by exactly the rows it needs (V + 1 rows for B, V + R for
// C and D), so one step of lag suffices and the rings hold 10 (XR) and 12 rows (the rest).
// The vertical apron is paid once per segment instead of once per tile: 1.03 blur positions
// and 1.06 gradients per output against the tiled stage's 1.16 and 1.33. The waves take
// roles: 0-1 the guide, 2-3 pass 2, 4-6 gradients and loads, 7 pass 1 -- two heavy and one
// or two light waves per SIMD, so no SIMD idles while a phase of another runs alone.
// Rings hold only rows in [lo, hi) (slot = row mod ring size); every reader clamps its row
// index, as the reference clamps its coordinates. Columns stay pre-clamped (XR holds the
// pixel at the clamped column, so MR, H and BR/RR hold the values at clamped centres).
// ---------------------------------------------------------------------------
namespace gs {
constexpr int R = 2, K = 2 * R + 1, V = 4;
constexpr int TW = 124, NT = 512;        // output columns per strip; 8 waves
constexpr int BW = TW + 2 * R;           // 128 blur / H columns: image x0 - R + c
constexpr int MW = TW + 4 * R;           // 132 magnitude columns: image x0 - 2R + c
constexpr int XL = 8;                    // XR column 0 = image x0 - XL (4-pixel aligned)
constexpr int XG = 35, XW = 4 * XG;      // 140 XR words per row: image x0 - 8 .. x0 + 131
constexpr int XRING = 10, RING = 12;     // ring rows
constexpr int O_XR = 0;
constexpr int O_MR = O_XR + XRING * XW;
constexpr int O_HRB = O_MR + RING * MW;  // R | B << 16 window sums
constexpr int O_HMX = O_HRB + RING * BW; // max s | (1023 - min s) << 16, s = r + g + b
constexpr int O_HG = O_HMX + RING * BW;  // G window sums, u16
constexpr int O_BR = O_HG + RING * BW / 2;
constexpr int O_RR = O_BR + 3 * RING * BW;
constexpr int O_ET = round_up(O_RR + RING * BW, 2);
constexpr int WORDS = O_ET + 128;        // + the exp table (64 doubles)
constexpr int LDS = 4 * WORDS;           // 52,384 bytes: three workgroups per CU
constexpr int NGRAD = V * MW;            // 528 gradients per step (waves 4-6, <= 3 each)
constexpr int NLOAD = V * XG;            // 140 four-pixel loads per step (waves 4-6)
static_assert(TW % 4 == 0 && TW <= 128 && BW == 128, "guide on waves 0-1, pass 2 on waves 2-3");
static_assert(V * (BW / 8) == 64, "pass 1 on wave 7: one run of 8 columns per lane");
static_assert(NGRAD <= 3 * 192 && NLOAD <= 192, "gradients and loads on waves 4-6");
static_assert(XW - XL >= TW + 2 * R + 2 && XW % 4 == 0, "XR covers the gradient and pass-1 reads");
static_assert(3 * LDS <= kLdsBudget, "three workgroups per CU");
constexpr int kMinSegRows = 16;          // rows per segment at least (the apron is ~10 rows)
}  // namespace gs

#ifdef VIP_GS_WAVES_PER_EU  // measurement knob: cap the VGPRs so more workgroups share a CU
#define VIP_GS_OCC __attribute__((amdgpu_waves_per_eu(VIP_GS_WAVES_PER_EU, VIP_GS_WAVES_PER_EU)))
#else
#define VIP_GS_OCC
#endif
template <bool CPP>
__global__ __launch_bounds__(gs::NT) VIP_GS_OCC void texture_guide_stream_kernel(const uint8_t* __restrict__ img,
                                                                      uint8_t* __restrict__ guide, int width, int lo,
                                                                      int hi, int gy0, int gy1, int seg_rows,
                                                                      int ksize, int aligned) {
    using namespace gs;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* const XR = lds + O_XR;
    float* const MR = reinterpret_cast<float*>(lds + O_MR);
    uint32_t* const HRB = lds + O_HRB;
    uint32_t* const HMX = lds + O_HMX;
    uint16_t* const HG = reinterpret_cast<uint16_t*>(lds + O_HG);
    float* const BR = reinterpret_cast<float*>(lds + O_BR);  // 3 planes of RING x BW
    float* const RR = reinterpret_cast<float*>(lds + O_RR);
    double* const etab = reinterpret_cast<double*>(lds + O_ET);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int x0 = blockIdx.x * TW, xr0 = x0 - XL;
    const int Y0 = gy0 + blockIdx.y * seg_rows;
    const int Y1 = Y0 + seg_rows < gy1 ? Y0 + seg_rows : gy1;
    if (Y0 >= Y1) return;  // whole workgroup
    const int W1 = width - 1, H1 = hi - 1;
    // rows each stage produces (the guide rows' reach, clamped to the valid rows)
    const int as = Y0 - 2 * R - 1 > lo ? Y0 - 2 * R - 1 : lo, ae = Y1 + 2 * R + 1 < hi ? Y1 + 2 * R + 1 : hi;
    const int bs = Y0 - 2 * R > lo ? Y0 - 2 * R : lo, be = Y1 + 2 * R < hi ? Y1 + 2 * R : hi;
    const int cs = Y0 - R > lo ? Y0 - R : lo, ce = Y1 + R < hi ? Y1 + R : hi;
    if (tid < 64) etab[tid] = kExp2Tab64[tid];  // first read by D at step 3, after barriers
    const float kk = (float)(ksize * ksize);
    const float rkk = 1.f / kk;
    constexpr float kThird = 0x1.555556p-2f;  // RN(1/3)
    const float sigma_alpha = 1.f / (float)(5 * ksize);
    const int ngroups = (Y1 - Y0 + V - 1) / V;

    for (int s = -3; s < ngroups + 3; ++s) {
        // ---- A: issue this step's image loads (waves 4-6) ----
        uint32_t raw0 = 0, raw1 = 0, raw2 = 0;
        int xr_at = -1;  // XR word the loaded group goes to
        if (wave >= 4 && wave < 7) {
            const int i = tid - 256;
            if (i < NLOAD) {
                const int rr = i / XG, gx = i - rr * XG;
                const int r = Y0 + 2 * R + 1 + s * V + rr;
                if (r >= as && r < ae) {
                    const uint8_t* row = img + (long long)r * width * 3;
                    const int x = xr0 + 4 * gx;
                    if ((aligned & 1) && x >= 0 && x + 3 <= W1) {
                        const uint32_t* w = reinterpret_cast<const uint32_t*>(row + 3 * x);
                        raw0 = w[0];
                        raw1 = w[1];
                        raw2 = w[2];
                    } else {
                        const uint32_t q0 = load_rgb(row, clampi(x, 0, W1)), q1 = load_rgb(row, clampi(x + 1, 0, W1));
                        const uint32_t q2 = load_rgb(row, clampi(x + 2, 0, W1)), q3 = load_rgb(row, clampi(x + 3, 0, W1));
                        raw0 = q0 | (q1 << 24);
                        raw1 = (q1 >> 8) | (q2 << 16);
                        raw2 = (q2 >> 16) | (q3 << 8);
                    }
                    xr_at = (r % XRING) * XW + 4 * gx;
                }
            }
        }

        if (wave < 2) {
            // ---- D: guide rows [g0, g0 + V) ----
            const int g0 = Y0 + (s - 3) * V;
            if (s >= 3) {
                const int tx = lane + 64 * wave;
                const int txr = tx < TW ? tx : TW - 1;  // lanes past the strip read in-strip values
                // window rows g0 - R .. g0 + V - 1 + R (clamped): each row's minimum and the
                // first column holding it (rtv >= +0 and finite: bit patterns order like values)
                uint32_t rv[V + 2 * R];
                int ri[V + 2 * R];
#pragma unroll
                for (int t = 0; t < V + 2 * R; ++t) {
                    const int row = clampi(g0 - R + t, lo, H1);
                    const int base = (row % RING) * BW + txr;
                    uint32_t m[K];
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) m[kx] = __float_as_uint(RR[base + kx]);
                    uint32_t v = m[0];
#pragma unroll
                    for (int kx = 1; kx < K; ++kx) v = v < m[kx] ? v : m[kx];
                    rv[t] = v;
                    int c = K - 1;
#pragma unroll
                    for (int kx = K - 2; kx >= 0; --kx) c = m[kx] == v ? kx : c;
                    ri[t] = base + c;
                }
                const int x = x0 + tx;
                const int q = lane & 3;
                // a quad of lanes = 4 pixels = 3 dwords (lanes 0-2 store one each); whole
                // quads are in or out of the strip (TW % 4 == 0)
                const bool dword_quad = (aligned & 2) && tx - q + 3 < TW && x - q + 3 <= W1;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const int g = g0 + j;
                    if (g >= Y1) break;
                    uint32_t mb = rv[j];
#pragma unroll
                    for (int ky = 1; ky < K; ++ky) mb = mb < rv[j + ky] ? mb : rv[j + ky];
                    int mi = ri[j + K - 1];
#pragma unroll
                    for (int ky = K - 2; ky >= 0; --ky) mi = rv[j + ky] == mb ? ri[j + ky] : mi;
                    const float rmin = __uint_as_float(mb);
                    const int ci = (g % RING) * BW + txr + R;
                    const float arg = sigma_alpha * (RR[ci] - rmin);
                    const float e = exp_tab_f32(arg, etab);  // == (float)exp((double)arg)
                    const float alpha = 2.f * recip_exact(1.f + e) - 1.f;
                    const float beta = 1.f - alpha;
                    uint32_t gw = 0;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float bm = BR[c * RING * BW + mi], bc = BR[c * RING * BW + ci];
                        const float v = CPP ? (alpha * bm + beta * bc) + 0.5f : __builtin_fmaf(alpha, bm, beta * bc) + 0.5f;
                        gw = pack_u8_clamped(v, c, gw);  // == clampi((int)v, 0, 255) << 8c
                    }
                    // the next lane's pixel (quad_perm [1, 2, 3, 3])
                    const uint32_t nx = (uint32_t)__builtin_amdgcn_mov_dpp((int)gw, 0xF9, 0xF, 0xF, false);
                    uint8_t* const orow = guide + ((long long)g * width + (x - q)) * 3;
                    if (dword_quad) {
                        if (q < 3)
                            reinterpret_cast<uint32_t*>(orow)[q] = (gw >> (8 * q)) | (nx << (24 - 8 * q));
                    } else if (tx < TW && x <= W1) {
                        uint8_t* const o = orow + 3 * q;
                        o[0] = (uint8_t)gw;
                        o[1] = (uint8_t)(gw >> 8);
                        o[2] = (uint8_t)(gw >> 16);
                    }
                }
            }
        } else if (wave < 4) {
            // ---- C: pass 2 at blur rows [p0, p0 + V), column bc ----
            const int p0 = Y0 + R + (s - 2) * V;
            if (p0 + V > cs && p0 < ce) {
                const int bc = tid - 128;
                // the blur centre's clamped column: its H column and its MR window's first column
                const int hcol = clampi(x0 - R + bc, 0, W1) - (x0 - R);
                constexpr int NV = V + K - 1;
                uint32_t hrb[NV], hg[NV], hmx[NV], rowmax[NV];
                int hro[NV];
#pragma unroll
                for (int t = 0; t < NV; ++t) {
                    hro[t] = clampi(p0 - R + t, lo, H1) % RING;
                    hrb[t] = HRB[hro[t] * BW + hcol];
                    hg[t] = HG[hro[t] * BW + hcol];
                    hmx[t] = HMX[hro[t] * BW + hcol];
                }
                uint32_t s0[V], s1[V], smx[V], mmaxb[V];
                float msum[V];
                win_sum<V, K>(hrb, s0);
                win_sum<V, K>(hg, s1);
                win_op<V, K>(hmx, smx, pk_max_u16);
#pragma unroll
                for (int t = 0; t < NV; ++t) {
                    const float* mrow = MR + hro[t] * MW + hcol;
                    float m[K];
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) m[kx] = mrow[kx];
                    uint32_t mx = __float_as_uint(m[0]);
#pragma unroll
                    for (int kx = 1; kx < K; ++kx) {  // == the reference's max (no NaN, >= +0)
                        const uint32_t b = __float_as_uint(m[kx]);
                        mx = mx > b ? mx : b;
                    }
                    rowmax[t] = mx;
#pragma unroll
                    for (int j = 0; j < V; ++j) {  // window row t - j of position j, row-major
                        if (t - j < 0 || t - j >= K) continue;
                        msum[j] = t == j ? m[0] : msum[j] + m[0];
#pragma unroll
                        for (int kx = 1; kx < K; ++kx) msum[j] = msum[j] + m[kx];
                    }
                }
                win_op<V, K>(rowmax, mmaxb, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const int p = p0 + j;
                    if (p < cs || p >= ce) continue;
                    const int o = (p % RING) * BW + bc;
                    BR[o] = div_exact(s0[j] & 0xffffu, kk, rkk);
                    BR[RING * BW + o] = div_exact(s1[j], kk, rkk);
                    BR[2 * RING * BW + o] = div_exact(s0[j] >> 16, kk, rkk);
                    const float imax = div_exact(smx[j] & 0xffffu, 3.f, kThird);
                    const float imin = div_exact(1023u - (smx[j] >> 16), 3.f, kThird);
                    const float num = (imax - imin) * __uint_as_float(mmaxb[j]);
                    RR[o] = CPP ? num / (msum[j] + 1e-9f) : (float)((double)num / ((double)msum[j] + 1e-9));
                }
            }
        } else {
            const int b0 = Y0 + 2 * R + (s - 1) * V;
            if (b0 + V > bs && b0 < be) {
                if (wave < 7) {
                    // ---- B: gradient magnitudes at rows [b0, b0 + V), MR columns ----
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const int i = tid - 256 + k * 192;
                        if (i >= NGRAD) break;
                        const int rr = i / MW, mc = i - rr * MW;
                        const int r = b0 + rr;
                        if (r < bs || r >= be) continue;
                        const int cx = clampi(x0 - 2 * R + mc, 0, W1) - xr0;
                        const uint32_t* rc = XR + (r % XRING) * XW + cx;
                        const uint32_t U = XR[((r - 1 > lo ? r - 1 : lo) % XRING) * XW + cx];
                        const uint32_t D = XR[((r + 1 < H1 ? r + 1 : H1) % XRING) * XW + cx];
                        const uint32_t L = rc[-1], Rt = rc[1];
                        const gf_s16x2 h02 = __builtin_bit_cast(gf_s16x2, Rt & 0x00ff00ffu) -
                                             __builtin_bit_cast(gf_s16x2, L & 0x00ff00ffu);
                        const gf_s16x2 v02 = __builtin_bit_cast(gf_s16x2, D & 0x00ff00ffu) -
                                             __builtin_bit_cast(gf_s16x2, U & 0x00ff00ffu);
                        const int h1 = (int)__builtin_amdgcn_ubfe(Rt, 8, 8) - (int)__builtin_amdgcn_ubfe(L, 8, 8);
                        const int v1 = (int)__builtin_amdgcn_ubfe(D, 8, 8) - (int)__builtin_amdgcn_ubfe(U, 8, 8);
                        const int ss = __builtin_amdgcn_sdot2(
                            h02, h02, __builtin_amdgcn_sdot2(v02, v02, h1 * h1 + v1 * v1, false), false);
                        MR[(r % RING) * MW + mc] = sqrt_int_exact((float)ss);  // == sqrtf
                    }
                } else {
                    // ---- B: pass 1, H at row b0 + lane / 16, columns 8 (lane % 16) .. +8 ----
                    const int r = b0 + (lane >> 4), hc0 = (lane & 15) * 8;
                    if (r >= bs && r < be) {
                        const uint32_t* xrow = XR + (r % XRING) * XW + hc0 + XL - 2 * R;
                        constexpr int NX = 8 + K - 1;
                        uint32_t rb[NX], gg[NX], mx[NX];
#pragma unroll
                        for (int t = 0; t < NX; ++t) {
                            const uint32_t p = xrow[t];
                            const uint32_t sb = __builtin_amdgcn_sad_u8(p, 0u, 0u);  // r + g + b
                            rb[t] = p & 0x00ff00ffu;
                            gg[t] = __builtin_amdgcn_ubfe(p, 8, 8);
                            mx[t] = ((sb ^ 1023u) << 16) | sb;  // max of lo = max s, of hi = 1023 - min s
                        }
                        uint32_t orb[8], og[8], omx[8];
                        win_sum<8, K>(rb, orb);
                        win_sum<8, K>(gg, og);
                        win_op<8, K>(mx, omx, pk_max_u16);
                        const int o = (r % RING) * BW + hc0;
                        *reinterpret_cast<uint4*>(HG + o) = make_uint4(og[0] | (og[1] << 16), og[2] | (og[3] << 16),
                                                                       og[4] | (og[5] << 16), og[6] | (og[7] << 16));
#pragma unroll
                        for (int j = 0; j < 8; j += 4) {
                            *reinterpret_cast<uint4*>(HRB + o + j) = make_uint4(orb[j], orb[j + 1], orb[j + 2], orb[j + 3]);
                            *reinterpret_cast<uint4*>(HMX + o + j) = make_uint4(omx[j], omx[j + 1], omx[j + 2], omx[j + 3]);
                        }
                    }
                }
            }
        }
        // ---- A: the loaded image group into the XR ring ----
        if (xr_at >= 0) *reinterpret_cast<uint4*>(XR + xr_at) = unpack_rgb4(raw0, raw1, raw2);
        __syncthreads();
    }
}

// Segments per strip: as many as fill the workgroup slots of the device in one round (the
// runtime's occupancy for this kernel: LDS and VGPRs), each at least kMinSegRows rows (the
// pipeline's apron is about ten rows).
template <bool CPP>
static int launch_gs(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1, int ksize,
                     int aligned, hipStream_t stream) {
    auto kern = texture_guide_stream_kernel<CPP>;
    static std::atomic<unsigned long long> attr_devs{0};
    if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), gs::LDS, attr_devs)) return rc;
    note_launch(reinterpret_cast<const void*>(kern));
    if (gy1 <= gy0) return 0;
    static std::atomic<int> per_cu{0};  // workgroups per CU (the same on every MI355X)
    int wg = per_cu.load(std::memory_order_relaxed);
    if (wg == 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&wg, reinterpret_cast<const void*>(kern), gs::NT, gs::LDS) !=
                hipSuccess ||
            wg < 1)
            wg = 1;
        per_cu.store(wg, std::memory_order_relaxed);
    }
    const int rows = gy1 - gy0;
    const int strips = (width + gs::TW - 1) / gs::TW;
    const int slots = wg * device_cus();
    int nseg = slots / strips;
    const int max_seg = (rows + gs::kMinSegRows - 1) / gs::kMinSegRows;
    nseg = nseg < 1 ? 1 : (nseg > max_seg ? max_seg : nseg);
    const int seg_rows = (rows + nseg - 1) / nseg;
    nseg = (rows + seg_rows - 1) / seg_rows;
    launch(kern, dim3(strips, nseg), dim3(gs::NT), gs::LDS, stream, img, guide, width, lo, hi, gy0, gy1, seg_rows,
           ksize, aligned);
    return (int)hipGetLastError();
}

template <bool CPP>
static int launch_gf_r(int ksize, const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1,
                       int aligned, hipStream_t s) {
#ifdef VIP_GF_STREAM  // measurement knob: the streaming stage at R = 2 (bit-exact, 1.39x slower)
    if (ksize / 2 == 2) return launch_gs<CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
#endif
#ifdef VIP_GF_ONLY_R2  // quick variant builds (scripts/build_texture_variant.sh): k = 4, 5 only
    if (ksize / 2 == 2) return launch_gf<2, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
    return VIP_ERR_UNSUPPORTED_KSIZE;
#endif
    switch (ksize / 2) {  // ksize 1..24 (kMaxKsizeTexture)
        case 1: return launch_gf<1, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 2: return launch_gf<2, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 3: return launch_gf<3, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 4: return launch_gf<4, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 5: return launch_gf<5, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 6: return launch_gf<6, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 7: return launch_gf<7, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 0: return launch_gf<0, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 8: return launch_gf<8, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 9: return launch_gf<9, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 10: return launch_gf<10, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 11: return launch_gf<11, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 12: return launch_gf<12, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        default: return VIP_ERR_UNSUPPORTED_KSIZE;
    }
}

int launch_texture_guide_fused_rows(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1,
                                    int ksize, bool cpp, hipStream_t stream) {
    // bit 0: image rows dword-aligned (dword tile loads); bit 1: guide rows (dword stores)
    const int aligned = (((uintptr_t)img % 4 == 0) && ((size_t)width * 3 % 4 == 0) ? 1 : 0) |
                        (((uintptr_t)guide % 4 == 0) && ((size_t)width * 3 % 4 == 0) ? 2 : 0);
    return cpp ? launch_gf_r<true>(ksize, img, guide, width, lo, hi, gy0, gy1, aligned, stream)
               : launch_gf_r<false>(ksize, img, guide, width, lo, hi, gy0, gy1, aligned, stream);
}

int launch_texture_guide_fused(const uint8_t* img, uint8_t* guide, int width, int height, int ksize, bool cpp,
                               hipStream_t stream) {
    return launch_texture_guide_fused_rows(img, guide, width, 0, height, 0, height, ksize, cpp, stream);
}

// ---------------------------------------------------------------------------
// One whole bilateral-texture iteration in one launch (guide + JBF fused
// in LDS), ksize 5 (C4) only: each workgroup owns a 128 x 64 tile of JBF outputs, the
// stencil kernel's tile (16 waves, 8 outputs per thread, JBF radius 4). It computes the
// guide over the tile (+) 4 -- 136 x 72 positions, in three 136 x 24 chunks through
// guide_tile -- straight into the JBF's guide plane, replaces every plane position
// outside the image by the guide at its clamped position (what the two-launch JBF reads
// through its clamped coordinates), loads the image plane (L2-hot: the guide just read
// it) and the 16-copy colour LUT into the chunks' dead scratch, and runs the JBF taps of
// bilateral_kernel. The guide never reaches HBM: 3 B/px read (+ halo) and 3 B/px
// written per iteration. The price is 1.2x the guide work (the 4-pixel JBF apron) and
// one workgroup per CU (127 KiB of LDS). Same arithmetic as the two launches, so the
// same bytes; selected per handle (vip_texture_set_mode).
// ---------------------------------------------------------------------------
constexpr int kFuR = 2, kFuJR = 4, kFuP = 8, kFuWaves = 16, kFuNT = kFuWaves * 64;
constexpr int kFuTH = kFuWaves * 4;            // 64 output rows
constexpr int kFuRows = kFuTH + 2 * kFuJR;     // 72 guide / image plane rows
constexpr int kFuChunk = 24;                   // guide rows per guide_tile call
constexpr int kFuCopies = 16;
using FuJG = Geom<kFuJR, kFuP>;                // TW 128, L 4, S 140
using FuGG = GfGeomT<kFuR, FuJG::TW + 2 * kFuJR, kFuChunk, kFuNT>;
constexpr int kFuPlane = kFuRows * FuJG::S;
constexpr int kFuLutWords = 768 * kFuCopies;
constexpr int kFuScratch = cmax(FuGG::WORDS_ALL, kFuPlane + kFuLutWords);
constexpr int kFuLds = 4 * (kFuPlane + kFuScratch);
static_assert(FuJG::L == kFuJR && FuGG::TW == FuJG::TW + 2 * FuJG::L, "guide chunk covers the plane columns");
static_assert(kFuRows % kFuChunk == 0 && FuJG::S >= FuGG::TW, "plane geometry");
static_assert(kFuLds <= kLdsBudget, "fused iteration does not fit LDS");

template <bool CPP>
__global__ __launch_bounds__(kFuNT) void texture_iteration_fused_kernel(const StencilArgs a, int ksize) {
    constexpr int R = kFuR, JR = kFuJR, P = kFuP, S = FuJG::S;
    constexpr bool FMA = !CPP;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* const gplane = lds;
    uint32_t* const scratch = lds + kFuPlane;
    uint32_t* const splane = scratch;
    uint32_t* const lut = scratch + kFuPlane;
    const int tid = threadIdx.x;
    const int tx0 = ((int)blockIdx.x % a.tiles_x) * FuJG::TW, ty0 = ((int)blockIdx.x / a.tiles_x) * kFuTH;
    const int W1 = a.width - 1, lo = a.row_lo, hi = a.row_hi;
    const int gx0 = tx0 - JR, gy0 = ty0 - JR;  // plane origin (image coordinates)
    const int aligned = a.aligned ? 1 : 0;

    // 1. guide over the plane, three chunks of rows; plane word (r, c) <-> (gx0 + c, gy0 + r)
#pragma unroll
    for (int c = 0; c < kFuRows / kFuChunk; ++c) {
        if (c) __syncthreads();  // the previous chunk is done with the scratch
        uint32_t* const prow = gplane + c * kFuChunk * S;
        guide_tile<FuGG, R, CPP, true>(scratch, a.src, a.width, lo, hi, hi, ksize, aligned, gx0, gy0 + c * kFuChunk,
                                 [&](int ty, int tx, uint32_t gw) { prow[ty * S + tx] = gw; });
    }
    __syncthreads();
    // 2. plane positions outside the image take the guide at their clamped position
    //    (reads in-image words, writes out-of-image words only: one pass, no hazard)
    if (gx0 < 0 || gy0 < lo || gx0 + FuGG::TW > W1 + 1 || gy0 + kFuRows > hi) {
        for (int q = tid; q < kFuRows * FuGG::TW; q += kFuNT) {
            const int r = q / FuGG::TW, cc = q - r * FuGG::TW;
            const int y = gy0 + r, x = gx0 + cc;
            const int cy = clampi(y, lo, hi - 1), cx = clampi(x, 0, W1);
            if (cy != y || cx != x) gplane[r * S + cc] = gplane[(cy - gy0) * S + (cx - gx0)];
        }
    }
    // 3. image plane (pre-clamped, as the stencil kernel's TilePrefetch loads it) and the
    //    colour LUT into the dead chunk scratch
    {
        TilePrefetch<JR, kFuRows, kFuNT, P> ps;
        LutStage<kFuNT, 768, kFuCopies> ls;
        ls.load(a.color);
        ps.issue(a.src, a.src_pitch, a, tx0, ty0);
        ls.store(lut);
        ps.commit(splane);
    }
    __syncthreads();

    // 4. JBF taps: bilateral_kernel's loop with two planes (src = image, guide = plane)
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = lane & 15;
    const int ty = wave * 4 + (lane >> 4);
    const uint32_t lane4 = (uint32_t)(lane & (kFuCopies - 1)) << 2;
    const char* const lut_bytes = reinterpret_cast<const char*>(lut);
    if (ty0 + wave * 4 >= a.out_rows) return;  // wave-uniform: rows past the frame
    uint32_t ctr[P];
    {
        const uint4* cp = reinterpret_cast<const uint4*>(gplane + (ty + JR) * S + tx * P + FuJG::L);
#pragma unroll
        for (int q = 0; q < P / 4; ++q) {
            const uint4 v = cp[q];
            ctr[4 * q + 0] = v.x; ctr[4 * q + 1] = v.y; ctr[4 * q + 2] = v.z; ctr[4 * q + 3] = v.w;
        }
    }
    f2 a01[P], a2k[P];
#pragma unroll
    for (int i = 0; i < P; ++i) a01[i] = a2k[i] = f2{0.f, 0.f};
    for_each_row<JR, true>([&](const int ky, auto hwc) {
        constexpr int HW = decltype(hwc)::value;
        const int aky = ky < 0 ? -ky : ky;
        set_progress_priority((ky + JR) * 4 / (2 * JR + 1));
        const int row_off = (ty + JR + ky) * S + tx * P;
        const float* const ws = a.ws + aky * kWsStride;
        constexpr int C0 = (FuJG::L - HW) / 4, C1 = (FuJG::L + P - 1 + HW) / 4;
        constexpr int NC = C1 - C0 + 1;
        float wsv[HW + 1];
#pragma unroll
        for (int k = 0; k <= HW; ++k) wsv[k] = ws[k];
        auto widx = [&](uint32_t g, f2, f2, int i, int) {
            const uint32_t d = __builtin_amdgcn_sad_u8(g, ctr[i], 0u);
            return (d << 6) | lane4;  // 16 copies: word d * 16 + copy
        };
        row_taps<HW, FuJG::L, C0, NC, FMA, false, P, true, decltype(widx)&>(gplane, splane, row_off, wsv, lut_bytes,
                                                                            widx, a01, a2k);
        fence_accumulators(a01, a2k);
    });
    uint32_t o[P];
    finish_outputs<P, true>(a01, a2k, o);
    store_px(a, ty0 + ty, tx0 + tx * P, o);
}

// One fused iteration of a whole frame (src -> dst, both dense pitch width*3; they must
// not alias). `a` carries the JBF handle's LUTs and the frame geometry.
int launch_texture_iteration_fused(const StencilArgs& a, int ksize, bool cpp, hipStream_t stream) {
    if (ksize != 2 * kFuR + 1) return VIP_ERR_UNSUPPORTED_KSIZE;
    auto kern = cpp ? texture_iteration_fused_kernel<true> : texture_iteration_fused_kernel<false>;
    static std::atomic<unsigned long long> attr_devs[2];
    if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), kFuLds, attr_devs[cpp ? 1 : 0]))
        return rc;
    note_launch(reinterpret_cast<const void*>(kern));
    StencilArgs args = a;
    args.tiles_x = (a.width + FuJG::TW - 1) / FuJG::TW;
    args.tiles_total = args.tiles_x * ((a.out_rows + kFuTH - 1) / kFuTH);
    if (args.tiles_total == 0) return 0;
    launch(kern, dim3(args.tiles_total), dim3(kFuNT), kFuLds, stream, args, ksize);
    return (int)hipGetLastError();
}

}  // namespace vip

#ifdef VIP_GF_STAMPS
extern "C" int vip_debug_read_gf_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vip::vip_gf_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
