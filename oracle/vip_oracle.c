/*
 * vip_oracle.c — TEST INFRASTRUCTURE ONLY. Not part of the product.
 *
 * Plain-C CPU restatement of the reference bilateral-filter family
 * (yuyuyu-bot/various_image_processings). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / CPU baseline. The product path (various_image_processings_amd/)
 * never links or calls it.
 *
 * Parity status: the reference is unbuildable in this image (include/cpp needs
 * OpenCV core + ximgproc, src/ needs nvcc + thrust, test/ needs gtest), so
 * this restatement is "parity unpinned" against reference *execution*. What is
 * pinned: the input generator below is checked bit-for-bit against the
 * reference's own test/random_array.hpp compiled in place (oracle/Makefile,
 * tests/golden/random_array_*.bin). Every function cites the reference lines it
 * restates.
 *
 * Two numerics profiles, because the reference's own CPU and GPU paths differ:
 *   VIPO_CUDA (0): src/<filter>_impl.cu — float-coefficient LUTs built with expf on the
 *                  host, and `sum += p * w` contracted to fmaf (nvcc default
 *                  -fmad=true). This is what the HIP product reproduces by default.
 *   VIPO_CPP  (1): include/cpp/<filter>.hpp — double-coefficient LUTs
 *                  (bilateral_filter.hpp:15-16), separate multiply and add
 *                  (x86-64 baseline, no FMA), float epsilon in mRTV.
 *   VIPO_REF  (2): the reference TESTS' own CPU oracles (test/adaptive_bilateral_filter.cu:7-119,
 *                  test/bilateral_texture_filter.cu:8-113, test/gradient.cu:9-34): float-coefficient
 *                  LUTs as CUDA, separate multiply and add as CPP (host code, no FMA), float
 *                  epsilon / FLT_MAX seed / unfused blend and glibc expf in the texture stages, and
 *                  the gradient's f32 order sum_c h*h then sum_c v*v, unfused. The oracle's REF
 *                  outputs equal those oracles compiled from the reference (oracle/Makefile ->
 *                  oracle/_ref/libref_test_oracles.so) bit for bit on tests/golden/ref_oracles.npz.
 * Build with -ffp-contract=off so gcc never fuses what the reference does not.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { VIPO_CUDA = 0, VIPO_CPP = 1, VIPO_REF = 2 };

/* Numerics-sensitivity variants of the CUDA profile (tests/test_oracle.py,
 * scripts/numerics_sensitivity.py). Each bit replaces one code-generation choice
 * that no reference artifact pins with the alternative nvcc could also have made;
 * 0 (default) is the profile the HIP product reproduces bit for bit.
 *   SUMK_FMA : sumk += ws * wc contracted to fmaf(ws, wc, sumk)
 *              (src/bilateral_filter_impl.cu:84-89; the product also feeds the sums)
 *   BLEND_B  : guide blend contracted the other way, fmaf(1-a, Bc, a * Bm)
 *              (src/bilateral_texture_filter_impl.cu:168-176)
 *   BLEND_NO : guide blend not contracted, a * Bm + (1-a) * Bc
 *   EXP_UP / EXP_DOWN : the guide's exp one ulp above / below the correctly
 *              rounded value (CUDA's expf is accurate to 2 ulp, not correctly rounded) */
enum { VIPO_V_SUMK_FMA = 1, VIPO_V_BLEND_B = 2, VIPO_V_BLEND_NO = 4, VIPO_V_EXP_UP = 8, VIPO_V_EXP_DOWN = 16 };
static int g_variant = 0;
void vipo_set_variant(int flags) { g_variant = flags; }

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* float -> uint8 as static_cast<uint8_t>(v) does for v in [0,256); NaN (0/0 when
 * every weight underflows) maps to 0, which is what both x86 cvttss2si and the
 * AMD v_cvt_u32_f32 produce. */
static inline uint8_t f2u8(float v) {
    if (!(v >= 0.0f)) return 0;
    return (uint8_t)(int)v;
}

/* ------------------------------------------------------------------------- */
/* test/random_array.hpp:9-31 — std::mt19937(42); u8: gen() % max; f32:      */
/* max * float(gen()) / float(UINT32_MAX).                                    */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t mt[624]; int idx; } mt19937_t;

static void mt_seed(mt19937_t* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}

static uint32_t mt_next(mt19937_t* s) {
    if (s->idx >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            uint32_t v = s->mt[(i + 397) % 624] ^ (y >> 1);
            if (y & 1u) v ^= 0x9908b0dfu;
            s->mt[i] = v;
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

void vipo_random_u8(size_t len, int max, uint8_t* out) {
    mt19937_t s;
    mt_seed(&s, 42u);
    for (size_t i = 0; i < len; i++) out[i] = (uint8_t)(mt_next(&s) % (uint32_t)max);
}

void vipo_random_f32(size_t len, float max, float* out) {
    mt19937_t s;
    mt_seed(&s, 42u);
    const float denom = (float)4294967295u; /* numeric_limits<uint32_t>::max() -> float */
    for (size_t i = 0; i < len; i++) out[i] = max * (float)mt_next(&s) / denom;
}

/* ------------------------------------------------------------------------- */
/* LUTs                                                                       */
/*  CUDA: src/bilateral_filter_impl.cu:217-237 (float coeff, std::exp(float)) */
/*  CPP : include/cpp/bilateral_filter.hpp:13-36 (double coeff)               */
/* Out-of-circle taps (r2 > radius^2) are 0 in both.                          */
/* ------------------------------------------------------------------------- */
void vipo_space_lut(int ksize, float sigma_space, int profile, float* out) {
    const int radius = ksize / 2;
    const float two_s2 = 2 * sigma_space * sigma_space; /* evaluated in float in both */
    const float cf = -1.f / two_s2;
    const double cd = -1. / (double)two_s2;
    for (int ky = -radius; ky <= radius; ky++) {
        for (int kx = -radius; kx <= radius; kx++) {
            const int kidx = (ky + radius) * ksize + (kx + radius);
            const int r2 = kx * kx + ky * ky;
            if (r2 > radius * radius) { out[kidx] = 0.f; continue; }
            out[kidx] = profile == VIPO_CPP ? (float)exp((double)r2 * cd) : expf((float)r2 * cf);
        }
    }
}

void vipo_color_lut(int len, float sigma_color, int profile, float* out) {
    const float two_s2 = 2 * sigma_color * sigma_color;
    const float cf = -1.f / two_s2;
    const double cd = -1. / (double)two_s2;
    for (int i = 0; i < len; i++)
        out[i] = profile == VIPO_CPP ? (float)exp((double)(i * i) * cd) : expf((float)(i * i) * cf);
}

/* accumulate one tap: CUDA contracts `sum += p * w` into fmaf; CPP and REF do not. */
#define ACC(profile, sum, p, w) \
    ((profile) != VIPO_CUDA ? ((sum) + (float)(p) * (w)) : fmaf((float)(p), (w), (sum)))

/* ------------------------------------------------------------------------- */
/* Bilateral / joint bilateral.                                               */
/*  CUDA: src/bilateral_filter_impl.cu:7-96 (BF), :98-202 (JBF)               */
/*  CPP : include/cpp/bilateral_filter.hpp:41-124 (BF), :126-207 (JBF)        */
/* Row-major tap order, replicate border, L1 colour distance into a 768 LUT,  */
/* dst = u8(sum/sumk + 0.5f). guide == NULL -> plain bilateral.               */
/* `rows` = output rows starting at src row `row0`; rows clamp to [0,height). */
/* ------------------------------------------------------------------------- */
static void bilateral_rows(const uint8_t* src, const uint8_t* guide, uint8_t* dst, int width, int height,
                           int ksize, const float* space, const float* color, int profile, int row0, int rows) {
    const int radius = ksize / 2;
    const uint8_t* g = guide ? guide : src;
    for (int yy = 0; yy < rows; yy++) {
        const int y = row0 + yy;
        for (int x = 0; x < width; x++) {
            const uint8_t* c = g + ((size_t)y * width + x) * 3;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, sk = 0.f;
            for (int ky = -radius; ky <= radius; ky++) {
                const int yc = clampi(y + ky, 0, height - 1);
                for (int kx = -radius; kx <= radius; kx++) {
                    const int xc = clampi(x + kx, 0, width - 1);
                    const uint8_t* p = src + ((size_t)yc * width + xc) * 3;
                    const uint8_t* q = g + ((size_t)yc * width + xc) * 3;
                    const int d = abs((int)c[0] - (int)q[0]) + abs((int)c[1] - (int)q[1]) + abs((int)c[2] - (int)q[2]);
                    const float w = space[(ky + radius) * ksize + (kx + radius)] * color[d];
                    s0 = ACC(profile, s0, p[0], w);
                    s1 = ACC(profile, s1, p[1], w);
                    s2 = ACC(profile, s2, p[2], w);
                    if (profile == VIPO_CUDA && (g_variant & VIPO_V_SUMK_FMA))
                        sk = fmaf(space[(ky + radius) * ksize + (kx + radius)], color[d], sk);
                    else
                        sk = sk + w;
                }
            }
            uint8_t* o = dst + ((size_t)yy * width + x) * 3;
            o[0] = f2u8(s0 / sk + 0.5f);
            o[1] = f2u8(s1 / sk + 0.5f);
            o[2] = f2u8(s2 / sk + 0.5f);
        }
    }
}

void vipo_bilateral_rows(const uint8_t* src, const uint8_t* guide, uint8_t* dst, int width, int height, int ksize,
                         float sigma_space, float sigma_color, int profile, int row0, int rows) {
    float* space = (float*)malloc(sizeof(float) * ksize * ksize);
    float color[768];
    vipo_space_lut(ksize, sigma_space, profile, space);
    vipo_color_lut(768, sigma_color, profile, color);
    bilateral_rows(src, guide, dst, width, height, ksize, space, color, profile, row0, rows);
    free(space);
}

void vipo_bilateral(const uint8_t* src, const uint8_t* guide, uint8_t* dst, int width, int height, int ksize,
                    float sigma_space, float sigma_color, int profile) {
    vipo_bilateral_rows(src, guide, dst, width, height, ksize, sigma_space, sigma_color, profile, 0, height);
}

/* ------------------------------------------------------------------------- */
/* Adaptive bilateral.                                                        */
/*  CUDA: src/adaptive_bilateral_filter_impl.cu:7-115 (LUT of 512*3, :5)      */
/*  CPP : include/cpp/adaptive_bilateral_filter.hpp:13-104                    */
/* offset_c = ctr_c - boxsum_c / k^2 over the full k x k square (exact int    */
/* sum either way, float divide); d = |n0-c0-o0| + |n1-c1-o1| + |n2-c2-o2| in */
/* float, LUT index int(d) (truncation); weights use the circular space LUT.  */
/* ------------------------------------------------------------------------- */
void vipo_adaptive_rows(const uint8_t* src, uint8_t* dst, int width, int height, int ksize, float sigma_space,
                        float sigma_color, int profile, int row0, int rows) {
    const int radius = ksize / 2;
    float* space = (float*)malloc(sizeof(float) * ksize * ksize);
    float color[1536];
    vipo_space_lut(ksize, sigma_space, profile, space);
    vipo_color_lut(1536, sigma_color, profile, color);
    const float kk = (float)(ksize * ksize);
    for (int yy = 0; yy < rows; yy++) {
        const int y = row0 + yy;
        for (int x = 0; x < width; x++) {
            const uint8_t* c = src + ((size_t)y * width + x) * 3;
            int b0 = 0, b1 = 0, b2 = 0; /* exact integer box sums (== float sums, all < 2^24) */
            for (int ky = -radius; ky <= radius; ky++) {
                const int yc = clampi(y + ky, 0, height - 1);
                for (int kx = -radius; kx <= radius; kx++) {
                    const int xc = clampi(x + kx, 0, width - 1);
                    const uint8_t* p = src + ((size_t)yc * width + xc) * 3;
                    b0 += p[0]; b1 += p[1]; b2 += p[2];
                }
            }
            const float o0 = (float)c[0] - (float)b0 / kk;
            const float o1 = (float)c[1] - (float)b1 / kk;
            const float o2 = (float)c[2] - (float)b2 / kk;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, sk = 0.f;
            for (int ky = -radius; ky <= radius; ky++) {
                const int yc = clampi(y + ky, 0, height - 1);
                for (int kx = -radius; kx <= radius; kx++) {
                    const int xc = clampi(x + kx, 0, width - 1);
                    const uint8_t* p = src + ((size_t)yc * width + xc) * 3;
                    const float d0 = (float)((int)p[0] - (int)c[0]) - o0;
                    const float d1 = (float)((int)p[1] - (int)c[1]) - o1;
                    const float d2 = (float)((int)p[2] - (int)c[2]) - o2;
                    const float dist = fabsf(d0) + fabsf(d1) + fabsf(d2);
                    const float w = space[(ky + radius) * ksize + (kx + radius)] * color[(int)dist];
                    s0 = ACC(profile, s0, p[0], w);
                    s1 = ACC(profile, s1, p[1], w);
                    s2 = ACC(profile, s2, p[2], w);
                    if (profile == VIPO_CUDA && (g_variant & VIPO_V_SUMK_FMA))
                        sk = fmaf(space[(ky + radius) * ksize + (kx + radius)], color[(int)dist], sk);
                    else
                        sk = sk + w;
                }
            }
            uint8_t* o = dst + ((size_t)yy * width + x) * 3;
            o[0] = f2u8(s0 / sk + 0.5f);
            o[1] = f2u8(s1 / sk + 0.5f);
            o[2] = f2u8(s2 / sk + 0.5f);
        }
    }
    free(space);
}

void vipo_adaptive(const uint8_t* src, uint8_t* dst, int width, int height, int ksize, float sigma_space,
                   float sigma_color, int profile) {
    vipo_adaptive_rows(src, dst, width, height, ksize, sigma_space, sigma_color, profile, 0, height);
}

/* ------------------------------------------------------------------------- */
/* Gradient magnitude, central differences, replicate border.                 */
/*  CUDA: src/gradient_impl.cu:7-66 — del_x = sum_c (I[x+1]-I[x-1])^2,         */
/*        del_y likewise, sqrtf(del_x + del_y); for f32 the square-accumulate  */
/*        is contracted to fmaf; for u8 it is an exact int product.           */
/*  CPP : include/cpp/gradient.hpp:13-55 — sum_c (h*h + v*v), sqrt.           */
/* u8 results are identical in both profiles (exact integers < 2^24).         */
/* ------------------------------------------------------------------------- */
static void gradient_impl(const void* src, int is_f32, float* dst, int width, int height, int ch, int profile) {
    const uint8_t* s8 = (const uint8_t*)src;
    const float* sf = (const float*)src;
#define PIX(xx, yy, cc) (is_f32 ? sf[((size_t)(yy) * width + (xx)) * ch + (cc)] : (float)s8[((size_t)(yy) * width + (xx)) * ch + (cc)])
    for (int y = 0; y < height; y++) {
        const int ym = clampi(y - 1, 0, height - 1), yp = clampi(y + 1, 0, height - 1);
        for (int x = 0; x < width; x++) {
            const int xm = clampi(x - 1, 0, width - 1), xp = clampi(x + 1, 0, width - 1);
            float out;
            if (!is_f32) {
                float dx = 0.f, dy = 0.f;
                for (int c = 0; c < ch; c++) {
                    const int h = (int)s8[((size_t)y * width + xp) * ch + c] - (int)s8[((size_t)y * width + xm) * ch + c];
                    const int v = (int)s8[((size_t)yp * width + x) * ch + c] - (int)s8[((size_t)ym * width + x) * ch + c];
                    dx = dx + (float)(h * h);
                    dy = dy + (float)(v * v);
                }
                out = sqrtf(dx + dy);
            } else if (profile == VIPO_CPP) {  /* include/cpp/gradient.hpp */
                float sum = 0.f;
                for (int c = 0; c < ch; c++) {
                    const float h = PIX(xp, y, c) - PIX(xm, y, c);
                    const float v = PIX(x, yp, c) - PIX(x, ym, c);
                    sum += h * h + v * v;
                }
                out = sqrtf(sum);
            } else if (profile == VIPO_REF) {  /* test/gradient.cu:11-31: unfused, h then v */
                float dx = 0.f, dy = 0.f;
                for (int c = 0; c < ch; c++) {
                    const float h = PIX(xm, y, c) - PIX(xp, y, c);
                    dx = dx + h * h;
                }
                for (int c = 0; c < ch; c++) {
                    const float v = PIX(x, ym, c) - PIX(x, yp, c);
                    dy = dy + v * v;
                }
                out = sqrtf(dx + dy);
            } else {
                float dx = 0.f, dy = 0.f;
                for (int c = 0; c < ch; c++) {
                    const float h = PIX(xp, y, c) - PIX(xm, y, c);
                    dx = fmaf(h, h, dx);
                }
                for (int c = 0; c < ch; c++) {
                    const float v = PIX(x, yp, c) - PIX(x, ym, c);
                    dy = fmaf(v, v, dy);
                }
                out = sqrtf(dx + dy);
            }
            dst[(size_t)y * width + x] = out;
        }
    }
#undef PIX
}

void vipo_gradient_u8(const uint8_t* src, float* dst, int width, int height, int ch, int profile) {
    gradient_impl(src, 0, dst, width, height, ch, profile);
}

void vipo_gradient_f32(const float* src, float* dst, int width, int height, int ch, int profile) {
    gradient_impl(src, 1, dst, width, height, ch, profile);
}

/* ------------------------------------------------------------------------- */
/* Bilateral-texture stage 1: box blur + modified relative total variation.   */
/*  CUDA: src/bilateral_texture_filter_impl.cu:10-104 — epsilon is the double */
/*        1e-9 (:8), so the final divide happens in double.                   */
/*  CPP : include/cpp/bilateral_texture_filter.hpp:17-61 (float 1e-9f, :15).  */
/* ------------------------------------------------------------------------- */
void vipo_blur_rtv(const uint8_t* img, const float* mag, float* blurred, float* rtv, int width, int height, int ksize,
                   int profile) {
    const int radius = ksize / 2;
    const float kk = (float)(ksize * ksize);
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            float imax = 0.f, imin = 256.f, mmax = 0.f, msum = 0.f;
            for (int ky = -radius; ky <= radius; ky++) {
                const int yc = clampi(y + ky, 0, height - 1);
                for (int kx = -radius; kx <= radius; kx++) {
                    const int xc = clampi(x + kx, 0, width - 1);
                    const uint8_t* p = img + ((size_t)yc * width + xc) * 3;
                    s0 += (float)p[0]; s1 += (float)p[1]; s2 += (float)p[2];
                    const float inten = (float)(p[0] + p[1] + p[2]) / 3.f;
                    imax = imax < inten ? inten : imax;
                    imin = inten < imin ? inten : imin;
                    const float m = mag[(size_t)yc * width + xc];
                    mmax = mmax < m ? m : mmax;
                    msum += m;
                }
            }
            float* b = blurred + ((size_t)y * width + x) * 3;
            b[0] = s0 / kk; b[1] = s1 / kk; b[2] = s2 / kk;
            const float num = (imax - imin) * mmax;
            rtv[(size_t)y * width + x] = profile != VIPO_CUDA ? num / (msum + 1e-9f)
                                                             : (float)((double)num / ((double)msum + 1e-9));
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Bilateral-texture stage 2: guide image.                                    */
/*  CUDA: src/bilateral_texture_filter_impl.cu:106-177                        */
/*  CPP : include/cpp/bilateral_texture_filter.hpp:85-125                     */
/* First strict argmin of rtv in the k x k window (row-major, clamped coords);*/
/* alpha = 2/(1+exp(sigma_alpha*(rtv_c - rtv_min))) - 1, sigma_alpha=1/(5k); */
/* G = clamp(int(alpha*B[min] + (1-alpha)*B + 0.5f), 0, 255).                  */
/* exp: both the HIP kernel and this oracle evaluate it as (float)exp(double),*/
/* i.e. correctly rounded expf, so device and host agree bit for bit.         */
/* CUDA: alpha*Bm + (1-alpha)*Bc contracts to fmaf(alpha, Bm, (1-alpha)*Bc).  */
/* ------------------------------------------------------------------------- */
void vipo_guide(const float* blurred, const float* rtv, uint8_t* guide, int width, int height, int ksize,
                int profile) {
    const int radius = ksize / 2;
    const float sigma_alpha = 1.f / (float)(5 * ksize);
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            float rmin = profile != VIPO_CUDA ? 3.402823466e+38f : 1e10f;
            int mx = 0, my = 0;
            for (int ky = -radius; ky <= radius; ky++) {
                const int yc = clampi(y + ky, 0, height - 1);
                for (int kx = -radius; kx <= radius; kx++) {
                    const int xc = clampi(x + kx, 0, width - 1);
                    const float v = rtv[(size_t)yc * width + xc];
                    if (rmin > v) { rmin = v; mx = xc; my = yc; }
                }
            }
            const float arg = sigma_alpha * (rtv[(size_t)y * width + x] - rtv[(size_t)my * width + mx]);
            float e = profile == VIPO_REF ? expf(arg) : (float)exp((double)arg); /* REF: std::exp(float) */
            if (profile == VIPO_CUDA && (g_variant & VIPO_V_EXP_UP)) e = nextafterf(e, INFINITY);
            if (profile == VIPO_CUDA && (g_variant & VIPO_V_EXP_DOWN)) e = nextafterf(e, 0.f);
            const float alpha = 2.f / (1.f + e) - 1.f;
            const float beta = 1.f - alpha;
            const float* bm = blurred + ((size_t)my * width + mx) * 3;
            const float* bc = blurred + ((size_t)y * width + x) * 3;
            uint8_t* g = guide + ((size_t)y * width + x) * 3;
            for (int c = 0; c < 3; c++) {
                float v;
                if (profile != VIPO_CUDA || (g_variant & VIPO_V_BLEND_NO)) v = alpha * bm[c] + beta * bc[c] + 0.5f;
                else if (g_variant & VIPO_V_BLEND_B) v = fmaf(beta, bc[c], alpha * bm[c]) + 0.5f;
                else v = fmaf(alpha, bm[c], beta * bc[c]) + 0.5f;
                g[c] = (uint8_t)clampi((int)v, 0, 255);
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Bilateral texture filter, GPU semantics (replicate-border JBF).            */
/*  CUDA: src/bilateral_texture_filter_impl.cu:179-214 — JBF ksize 2k-1,      */
/*        sigma_space k-1, sigma_color sqrt(3) = 1.73205080757f (.cuh:31).    */
/*  CPP : include/cpp/bilateral_texture_filter.hpp:153-164 uses               */
/*        cv::ximgproc::jointBilateralFilter (reflect-101 border); the CPP     */
/*        profile here keeps the replicate border and only swaps numerics.    */
/* ------------------------------------------------------------------------- */
void vipo_texture(const uint8_t* src, uint8_t* dst, int width, int height, int ksize, int nitr, int profile) {
    const size_t n = (size_t)width * height;
    uint8_t* src_n = (uint8_t*)malloc(n * 3);
    float* mag = (float*)malloc(n * sizeof(float));
    float* blurred = (float*)malloc(n * 3 * sizeof(float));
    float* rtv = (float*)malloc(n * sizeof(float));
    uint8_t* guide = (uint8_t*)malloc(n * 3);
    memcpy(dst, src, n * 3);
    for (int it = 0; it < nitr; it++) {
        memcpy(src_n, dst, n * 3);
        vipo_gradient_u8(src_n, mag, width, height, 3, profile);
        vipo_blur_rtv(src_n, mag, blurred, rtv, width, height, ksize, profile);
        vipo_guide(blurred, rtv, guide, width, height, ksize, profile);
        vipo_bilateral(src_n, guide, dst, width, height, 2 * ksize - 1, (float)(ksize - 1), 1.73205080757f, profile);
    }
    free(src_n); free(mag); free(blurred); free(rtv); free(guide);
}
