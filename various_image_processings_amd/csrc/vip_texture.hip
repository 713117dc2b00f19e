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
    hipLaunchKernelGGL((gradient_kernel<T, CH, FMA>), grid, dim3(256), 0, stream, src, dst, width, height);
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
        hipLaunchKernelGGL(blur_rtv_kernel<true>, grid, dim3(256), lds, stream, img, mag, blurred, rtv, width, height,
                           ksize);
    else
        hipLaunchKernelGGL(blur_rtv_kernel<false>, grid, dim3(256), lds, stream, img, mag, blurred, rtv, width, height,
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
        hipLaunchKernelGGL(guide_kernel<true>, grid, dim3(256), lds, stream, blurred, rtv, guide, width, height, ksize);
    else
        hipLaunchKernelGGL(guide_kernel<false>, grid, dim3(256), lds, stream, blurred, rtv, guide, width, height, ksize);
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
//   XR : T (+) (2R+1)  image pixels as RGBX words (origin 4-px aligned)
//   MR : T (+) 2R      gradient magnitude
//   BR, RR : T (+) R   blurred RGB and rtv
// Bit-exact with the stage kernels: integer box sums (exact), intensity extremes
// from integer byte sums (x/3.f is monotonic), magnitude sum accumulated in the
// reference's row-major order, rtv divide in double (CUDA profile).
// ---------------------------------------------------------------------------
constexpr int kGfTW = 64, kGfTH = 16, kGfNT = 256, kGfRun = 4;

template <int R>
struct GfGeom {
    static constexpr int XL = round_up(2 * R + 1, 4);          // XR left apron (aligned)
    // widths padded so the runs of kGfRun positions that overhang the real
    // regions (their results are never read) stay inside their source rows
    static constexpr int XW = round_up(kGfTW + XL + 2 * R + 1 + 8, 4);
    static constexpr int XH = kGfTH + 4 * R + 2;
    static constexpr int MW = round_up(kGfTW + 4 * R + 4, kGfRun);
    static constexpr int MH = kGfTH + 4 * R;
    static constexpr int BW = round_up(kGfTW + 2 * R, kGfRun);
    static constexpr int BH = kGfTH + 2 * R;
    static constexpr int WORDS = XW * XH + MW * MH + 4 * BW * BH;
};

// Row bands: rows [lo, hi) of the (dense, width*3 pitch) buffers are the valid
// frame rows -- every stage clamps into them, as the reference clamps into
// [0, height) -- and guide rows [gy0, gy1) are produced (a row slab of a sharded
// frame; the whole frame is lo = gy0 = 0, hi = gy1 = height).
template <int R, bool CPP>
__global__ __launch_bounds__(kGfNT) void texture_guide_fused_kernel(const uint8_t* __restrict__ img,
                                                                   uint8_t* __restrict__ guide, int width, int lo,
                                                                   int hi, int gy0, int gy1, int ksize,
                                                                   int aligned) {
    using G = GfGeom<R>;
    constexpr int K = 2 * R + 1;  // window width; the reference divides by ksize^2 and
                                  // uses sigma_alpha = 1/(5 ksize) even when ksize is even
    constexpr bool PACKRB = K * K * 255 < 65536;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* XR = lds;
    float* MR = reinterpret_cast<float*>(XR + G::XW * G::XH);
    float* BR = MR + G::MW * G::MH;  // 3 planes of BW*BH
    float* RR = BR + 3 * G::BW * G::BH;
    const int x0 = blockIdx.x * kGfTW, y0 = gy0 + blockIdx.y * kGfTH;
    const int tid = threadIdx.x;
    // region origins (image coordinates)
    const int xr0 = x0 - G::XL, yr0 = y0 - 2 * R - 1;
    const int mr0x = x0 - 2 * R, mr0y = y0 - 2 * R;
    const int br0x = x0 - R, br0y = y0 - R;
    const int W1 = width - 1, H0 = lo, H1 = hi - 1;

    // 1. XR: 4-pixel groups, dword loads when interior and aligned, clamped bytes otherwise
    for (int g = tid; g < G::XH * (G::XW / 4); g += kGfNT) {
        const int ry = g / (G::XW / 4), gx = g - ry * (G::XW / 4);
        const uint8_t* row = img + (long long)clampi(yr0 + ry, H0, H1) * width * 3;
        const int x = xr0 + 4 * gx;
        uint4 q;
        if (aligned && x >= 0 && x + 3 <= W1) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(row + 3 * x);
            q = unpack_rgb4(w[0], w[1], w[2]);
        } else {
            q.x = load_rgb(row, clampi(x, 0, W1));
            q.y = load_rgb(row, clampi(x + 1, 0, W1));
            q.z = load_rgb(row, clampi(x + 2, 0, W1));
            q.w = load_rgb(row, clampi(x + 3, 0, W1));
        }
        *reinterpret_cast<uint4*>(XR + ry * G::XW + 4 * gx) = q;
    }
    __syncthreads();

    // 2. MR[q] = gradient at c = clamp(q); XR is pre-clamped, so c's neighbours
    //    are read directly (XR[c +- e] == X(clamp(c +- e)))
    for (int i = tid; i < G::MW * G::MH; i += kGfNT) {
        const int qy = i / G::MW, qx = i - qy * G::MW;
        const int cx = clampi(mr0x + qx, 0, W1) - xr0, cy = clampi(mr0y + qy, H0, H1) - yr0;
        const uint32_t* c = XR + cy * G::XW + cx;
        const uint32_t L = c[-1], Rt = c[1], U = c[-G::XW], D = c[G::XW];
        float dx = 0.f, dy = 0.f;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const int h = (int)((Rt >> (8 * ch)) & 0xffu) - (int)((L >> (8 * ch)) & 0xffu);
            const int v = (int)((D >> (8 * ch)) & 0xffu) - (int)((U >> (8 * ch)) & 0xffu);
            dx = dx + (float)(h * h);
            dy = dy + (float)(v * v);
        }
        MR[i] = __builtin_sqrtf(dx + dy);
    }
    __syncthreads();

    // 3. box blur + mRTV, kGfRun horizontally adjacent positions per thread
    const float kk = (float)(ksize * ksize);
    for (int run = tid; run < G::BH * (G::BW / kGfRun); run += kGfNT) {
        const int py = run / (G::BW / kGfRun), px0 = (run - py * (G::BW / kGfRun)) * kGfRun;
        const int iy = br0y + py, ix0 = br0x + px0;
        uint32_t s0[kGfRun], s1[kGfRun], smax[kGfRun], smin[kGfRun], s2[kGfRun];
        float mmax[kGfRun], msum[kGfRun];
#pragma unroll
        for (int j = 0; j < kGfRun; ++j) {
            s0[j] = s1[j] = s2[j] = smax[j] = 0u;
            smin[j] = 0xffffffffu;
            mmax[j] = msum[j] = 0.f;
        }
        if (iy >= H0 && iy <= H1 && ix0 >= 0 && ix0 + kGfRun - 1 <= W1) {
            // all centres inside the image: shared row segments
            for (int ky = -R; ky <= R; ++ky) {
                const uint32_t* xrow = XR + (iy + ky - yr0) * G::XW + (ix0 - R - xr0);
                const float* mrow = MR + (iy + ky - mr0y) * G::MW + (ix0 - R - mr0x);
                uint32_t xs[kGfRun + 2 * R];
                float ms[kGfRun + 2 * R];
#pragma unroll
                for (int t = 0; t < kGfRun + 2 * R; ++t) {
                    xs[t] = xrow[t];
                    ms[t] = mrow[t];
                }
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
#pragma unroll
                    for (int j = 0; j < kGfRun; ++j) {
                        const uint32_t p = xs[j + kx];
                        if constexpr (PACKRB) {
                            s0[j] += p & 0x00ff00ffu;  // R | B<<16 in 16-bit lanes
                        } else {
                            s0[j] += p & 0xffu;
                            s2[j] += __builtin_amdgcn_ubfe(p, 16, 8);
                        }
                        s1[j] += __builtin_amdgcn_ubfe(p, 8, 8);
                        const uint32_t sb = __builtin_amdgcn_sad_u8(p, 0u, 0u);
                        smax[j] = sb > smax[j] ? sb : smax[j];
                        smin[j] = sb < smin[j] ? sb : smin[j];
                        const float m = ms[j + kx];
                        mmax[j] = __builtin_fmaxf(mmax[j], m);  // == the reference's max for non-NaN
                        msum[j] = msum[j] + m;  // row-major order, as the reference
                    }
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < kGfRun; ++j) {
                const int cx = clampi(ix0 + j, 0, W1), cy = clampi(iy, H0, H1);
                for (int ky = -R; ky <= R; ++ky) {
                    const uint32_t* xrow = XR + (cy + ky - yr0) * G::XW + (cx - xr0);
                    const float* mrow = MR + (cy + ky - mr0y) * G::MW + (cx - mr0x);
#pragma unroll
                    for (int kx = -R; kx <= R; ++kx) {
                        const uint32_t p = xrow[kx];
                        if constexpr (PACKRB) {
                            s0[j] += p & 0x00ff00ffu;  // R | B<<16 in 16-bit lanes
                        } else {
                            s0[j] += p & 0xffu;
                            s2[j] += __builtin_amdgcn_ubfe(p, 16, 8);
                        }
                        s1[j] += __builtin_amdgcn_ubfe(p, 8, 8);
                        const uint32_t sb = __builtin_amdgcn_sad_u8(p, 0u, 0u);
                        smax[j] = sb > smax[j] ? sb : smax[j];
                        smin[j] = sb < smin[j] ? sb : smin[j];
                        const float m = mrow[kx];
                        mmax[j] = __builtin_fmaxf(mmax[j], m);
                        msum[j] = msum[j] + m;
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kGfRun; ++j) {
            const int i = py * G::BW + px0 + j;
            BR[i] = (float)(PACKRB ? (s0[j] & 0xffffu) : s0[j]) / kk;
            BR[G::BW * G::BH + i] = (float)s1[j] / kk;
            BR[2 * G::BW * G::BH + i] = (float)(PACKRB ? (s0[j] >> 16) : s2[j]) / kk;
            const float imax = (float)(int)smax[j] / 3.f, imin = (float)(int)smin[j] / 3.f;
            const float num = (imax - imin) * mmax[j];
            RR[i] = CPP ? num / (msum[j] + 1e-9f) : (float)((double)num / ((double)msum[j] + 1e-9));
        }
    }
    __syncthreads();

    // 4. guide: first strict argmin of rtv over the window (RR is pre-clamped, so the
    //    reference's clamped-coordinate scan is a direct row-major scan). A thread
    //    takes kGfRun vertically adjacent outputs: each window row's first argmin is
    //    found once and shared; scanning those rows in order with strict > then
    //    gives the row-major first argmin. Alpha blend per output.
    const float sigma_alpha = 1.f / (float)(5 * ksize);
    for (int run = tid; run < (kGfTH / kGfRun) * kGfTW; run += kGfNT) {
        const int tx = run % kGfTW, ty0 = (run / kGfTW) * kGfRun;
        const int x = x0 + tx;
        if (x > W1 || y0 + ty0 >= gy1) continue;
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
            const int ci = (ty0 + j + R) * G::BW + tx + R;
            const float arg = sigma_alpha * (RR[ci] - rmin);
            const float e = (float)exp((double)arg);
            const float alpha = 2.f / (1.f + e) - 1.f;
            const float beta = 1.f - alpha;
            uint8_t* g = guide + ((long long)y * width + x) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float bm = BR[c * G::BW * G::BH + mi], bc = BR[c * G::BW * G::BH + ci];
                const float v = CPP ? (alpha * bm + beta * bc) + 0.5f : __builtin_fmaf(alpha, bm, beta * bc) + 0.5f;
                g[c] = (uint8_t)clampi((int)v, 0, 255);
            }
        }
    }
}

template <int R, bool CPP>
static int launch_gf(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1, int ksize,
                     int aligned, hipStream_t stream) {
    constexpr int LDS = 4 * GfGeom<R>::WORDS;
    static_assert(LDS <= kLdsBudget, "fused guide tile does not fit LDS");
    auto kern = texture_guide_fused_kernel<R, CPP>;
    static bool attr_done = false;
    if (!attr_done) {
        VIP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
        attr_done = true;
    }
    if (gy1 <= gy0) return 0;
    dim3 grid((width + kGfTW - 1) / kGfTW, (gy1 - gy0 + kGfTH - 1) / kGfTH);
    hipLaunchKernelGGL(kern, grid, dim3(kGfNT), LDS, stream, img, guide, width, lo, hi, gy0, gy1, ksize, aligned);
    return (int)hipGetLastError();
}

template <bool CPP>
static int launch_gf_r(int ksize, const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1,
                       int aligned, hipStream_t s) {
    switch (ksize / 2) {
        case 1: return launch_gf<1, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 2: return launch_gf<2, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 3: return launch_gf<3, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 4: return launch_gf<4, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 5: return launch_gf<5, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 6: return launch_gf<6, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 7: return launch_gf<7, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        case 8: return launch_gf<8, CPP>(img, guide, width, lo, hi, gy0, gy1, ksize, aligned, s);
        default: return VIP_ERR_UNSUPPORTED_KSIZE;
    }
}

int launch_texture_guide_fused_rows(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1,
                                    int ksize, bool cpp, hipStream_t stream) {
    const int aligned = ((uintptr_t)img % 4 == 0) && ((size_t)width * 3 % 4 == 0);
    return cpp ? launch_gf_r<true>(ksize, img, guide, width, lo, hi, gy0, gy1, aligned, stream)
               : launch_gf_r<false>(ksize, img, guide, width, lo, hi, gy0, gy1, aligned, stream);
}

int launch_texture_guide_fused(const uint8_t* img, uint8_t* guide, int width, int height, int ksize, bool cpp,
                               hipStream_t stream) {
    return launch_texture_guide_fused_rows(img, guide, width, 0, height, 0, height, ksize, cpp, stream);
}

}  // namespace vip
