// Runtime-radius bilateral / joint-bilateral / adaptive-bilateral kernel (gfx950).
//
// The templated kernels (vip_bilateral.hip, vip_adaptive.hip) are specialised per
// radius 1..15: every tile row is straight-line code with a compile-time disc
// half-width. The reference sizes its shared memory from ksize with no cap
// (src/bilateral_filter_impl.cu:252-254, 272-275; src/adaptive_bilateral_filter_impl.cu:
// 165-167), so under CUDA's 48 KB default it runs bilateral up to ksize 65, joint up to
// 47 and adaptive up to 63, and ksize 1 (radius 0) for all of them. Those radii (0 and
// 16..32) run here, with the radius a kernel argument:
//
//   * one 1024-thread workgroup per 64 x 64 output tile, 4 horizontally adjacent outputs
//     per thread; LDS = the tile plane(s) as RGBX words, (64 + 2R) rows x S words
//     (S = 64 or 128, so the 16-lane groups of a ds_read_b128 hit disjoint banks), then
//     the colour LUT with 32 interleaved copies (16 for the adaptive 1536-entry table
//     and the two-plane joint filter). At R = 32 that is exactly the CU's 160 KiB.
//   * per tile row ky the taps kx = -k4 .. k4' run in blocks of 4 (k4 = hw rounded up to
//     a multiple of 4, so every block's plane words are one aligned ds_read_b128): a
//     block needs 7 words for the thread's 4 outputs, the 4 of its own and the 4 of the
//     next block, each converted to floats once. The spatial weights come from a
//     zero-padded per-row table by scalar loads; a tap outside the disc (|kx| > hw) has
//     weight exactly 0, as in the reference's k x k loop -- fma(p, 0, s) == s and
//     sk + 0 == sk, so the padding leaves every sum bit-identical.
//   * per output the taps accumulate in row-major order (rows ascending, kx ascending),
//     in the reference's arithmetic (w = ws * wc, fma or mul+add by profile).
//   * adaptive: the k x k box sums (the window mean, src/adaptive_bilateral_filter_impl.cu:
//     79-93) are per-thread sliding row sums over the plane, exact integers; the mean is
//     the IEEE quotient by k^2 as in the reference.
#include "vip_stencil.hpp"

namespace vip {

constexpr int kRtP = 4;           // outputs per thread
constexpr int kRtTW = 16 * kRtP;  // tile width in pixels
constexpr int kRtWaves = 16;

// LDS words of one tile plane (+ a zeroed pad when the apron is narrower than the
// one-block over-read of the last row, i.e. only at R = 0)
__host__ __device__ constexpr int rt_plane_words(int R, int L, int S, int waves) {
    return (waves * 4 + 2 * R) * S + (L < 4 ? 8 : 0);
}
__host__ __device__ constexpr int rt_stride(int L) { return kRtTW + 2 * L <= 64 ? 64 : 128; }

// One 4-pixel group of image row sy starting at column x (clamped to the image), as
// RGBX words: three dword loads when interior and aligned, clamped bytes otherwise.
__device__ __forceinline__ uint4 load_group(const uint8_t* img, long long pitch, int sy, int x, int width,
                                            int aligned) {
    const uint8_t* row = img + (long long)sy * pitch;
    if (aligned && x >= 0 && x + 3 < width) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(row + 3 * x);
        return unpack_rgb4(w[0], w[1], w[2]);
    }
    uint4 r;
    r.x = load_rgb(row, clampi(x + 0, 0, width - 1));
    r.y = load_rgb(row, clampi(x + 1, 0, width - 1));
    r.z = load_rgb(row, clampi(x + 2, 0, width - 1));
    r.w = load_rgb(row, clampi(x + 3, 0, width - 1));
    return r;
}

// 4 consecutive plane words: guide words (colour distance) and source floats (sums)
template <bool JOINT>
struct RtWin {
    uint32_t g[4];
    float c0[4], c1[4], c2[4];
    __device__ __forceinline__ void load(const uint32_t* gplane, const uint32_t* splane, int off) {
        const uint4 v = *reinterpret_cast<const uint4*>(gplane + off);
        g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
        uint32_t s[4] = {v.x, v.y, v.z, v.w};
        if constexpr (JOINT) {
            const uint4 u = *reinterpret_cast<const uint4*>(splane + off);
            s[0] = u.x; s[1] = u.y; s[2] = u.z; s[3] = u.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            c0[k] = (float)(s[k] & 0xffu);
            c1[k] = (float)((s[k] >> 8) & 0xffu);
            c2[k] = (float)((s[k] >> 16) & 0xffu);
        }
    }
};

// The spatial table and the half-widths are read-only for the whole launch: read them
// through the constant address space so the uniform loads become scalar loads.
#define kconst __attribute__((address_space(4)))

template <int COPIES, bool JOINT, bool FMA, bool ADAPTIVE>
__global__ __launch_bounds__(kRtWaves * 64) void stencil_rt_kernel(const RtArgs a) {
    constexpr int P = kRtP, NT = kRtWaves * 64, TH = kRtWaves * 4;
    constexpr int NE = ADAPTIVE ? 1536 : 768;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int R = a.R, L = a.L, S = a.S;
    const int rows = TH + 2 * R;
    const int pw = rt_plane_words(R, L, S, kRtWaves);
    uint32_t* const gplane = lds;
    uint32_t* const splane = JOINT ? lds + pw : lds;
    uint32_t* const lut = lds + (JOINT ? 2 : 1) * pw;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = lane & 15;
    const int ty = wave * 4 + (lane >> 4);
    const int tile = blockIdx.x;
    const int tx0 = (tile % a.tiles_x) * kRtTW, ty0 = (tile / a.tiles_x) * TH;

    // colour LUT: word d*COPIES + c = color[d]
    {
        constexpr int SHIFT = COPIES == 32 ? 3 : 2;
        for (int q = tid; q < NE * COPIES / 4; q += NT) {
            const uint32_t v = __float_as_uint(a.color[q >> SHIFT]);
            *reinterpret_cast<uint4*>(lut + 4 * q) = make_uint4(v, v, v, v);
        }
    }
    // tile plane(s); columns [TW + 2L, S) and the pad are zeroed: the last tap block of
    // a row reads up to 4 words past its apron (weight 0), and those words must hold
    // RGBX data (byte 3 = 0) so that their LUT index stays inside the table
    {
        const int gpr = S / 4, valid = (kRtTW + 2 * L) / 4;
        for (int q = tid; q < rows * gpr; q += NT) {
            const int r = q / gpr, gc = q - r * gpr;
            uint4 gw = make_uint4(0u, 0u, 0u, 0u), sw = gw;
            if (gc < valid) {
                const int sy = clampi(ty0 + a.src_row0 - R + r, a.row_lo, a.row_hi - 1);
                const int x = tx0 - L + 4 * gc;
                gw = load_group(a.guide, a.guide_pitch, sy, x, a.width, a.aligned);
                if constexpr (JOINT) sw = load_group(a.src, a.src_pitch, sy, x, a.width, a.aligned);
            }
            *reinterpret_cast<uint4*>(gplane + r * S + 4 * gc) = gw;
            if constexpr (JOINT) *reinterpret_cast<uint4*>(splane + r * S + 4 * gc) = sw;
        }
        if (L < 4 && tid < 2) {
            *reinterpret_cast<uint4*>(gplane + rows * S + 4 * tid) = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (JOINT) *reinterpret_cast<uint4*>(splane + rows * S + 4 * tid) = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    __syncthreads();
    if (ty0 + wave * 4 >= a.out_rows) return;  // wave-uniform; no barrier follows

    const int xc = L + tx * P;  // plane column of the thread's output 0
    uint32_t ctr[P];
    {
        const uint4 v = *reinterpret_cast<const uint4*>(gplane + (ty + R) * S + xc);
        ctr[0] = v.x; ctr[1] = v.y; ctr[2] = v.z; ctr[3] = v.w;
    }
    const uint32_t lanec = (uint32_t)(lane & (COPIES - 1)) << 2;
    const char* const lut_bytes = reinterpret_cast<const char*>(lut);

    float c0f[P], c1f[P], c2f[P], o0[P], o1[P], o2[P];
    if constexpr (ADAPTIVE) {
        // exact integer k x k sums per output: sliding row sums (R|B packed in 16-bit
        // lanes, (2R+1) * 255 < 2^16) added into 32-bit totals row by row
        const int K = 2 * R + 1;
        uint32_t tr[P], tg[P], tb[P];
#pragma unroll
        for (int i = 0; i < P; ++i) tr[i] = tg[i] = tb[i] = 0u;
        for (int r = 0; r < K; ++r) {
            const uint32_t* base = gplane + (ty + r) * S + xc - R;
            uint32_t srb = 0u, sg = 0u;
            for (int c = 0; c < K; ++c) {
                const uint32_t p = base[c];
                srb += p & 0x00ff00ffu;
                sg += __builtin_amdgcn_ubfe(p, 8, 8);
            }
#pragma unroll
            for (int i = 0; i < P; ++i) {
                if (i > 0) {
                    const uint32_t pa = base[K - 1 + i], pd = base[i - 1];
                    srb = srb + (pa & 0x00ff00ffu) - (pd & 0x00ff00ffu);
                    sg = sg + __builtin_amdgcn_ubfe(pa, 8, 8) - __builtin_amdgcn_ubfe(pd, 8, 8);
                }
                tr[i] += srb & 0xffffu;
                tb[i] += srb >> 16;
                tg[i] += sg;
            }
        }
        // offset = centre - sum / (ksize * ksize) (src/adaptive_bilateral_filter_impl.cu:89-93)
        const float kk = (float)(K * K);
#pragma unroll
        for (int i = 0; i < P; ++i) {
            c0f[i] = (float)(ctr[i] & 0xffu);
            c1f[i] = (float)((ctr[i] >> 8) & 0xffu);
            c2f[i] = (float)((ctr[i] >> 16) & 0xffu);
            // keep (n - c) a float subtract (see vip_adaptive.hip set_offsets)
            __asm__("" : "+v"(c0f[i]), "+v"(c1f[i]), "+v"(c2f[i]));
            o0[i] = c0f[i] - (float)tr[i] / kk;
            o1[i] = c1f[i] - (float)tg[i] / kk;
            o2[i] = c2f[i] - (float)tb[i] / kk;
        }
    }

    f2 a01[P], a2k[P];  // {sum_b, sum_g}, {sum_r, sumk}
#pragma unroll
    for (int i = 0; i < P; ++i) a01[i] = a2k[i] = f2{0.f, 0.f};

    // 4 taps x 4 outputs: tap t of the block pairs output i with word t + i of cur|nxt
    auto block = [&](const RtWin<JOINT>& cur, const RtWin<JOINT>& nxt, const kconst float* wsb) {
        const float wsv[4] = {wsb[0], wsb[1], wsb[2], wsb[3]};  // uniform: one scalar load
        float wc[4][P];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const int j = t + i;
                uint32_t d;
                if constexpr (ADAPTIVE) {
                    const float n0 = j < 4 ? cur.c0[j & 3] : nxt.c0[j & 3];
                    const float n1 = j < 4 ? cur.c1[j & 3] : nxt.c1[j & 3];
                    const float n2 = j < 4 ? cur.c2[j & 3] : nxt.c2[j & 3];
                    const float d0 = (n0 - c0f[i]) - o0[i];
                    const float d1 = (n1 - c1f[i]) - o1[i];
                    const float d2 = (n2 - c2f[i]) - o2[i];
                    d = (uint32_t)((__builtin_fabsf(d0) + __builtin_fabsf(d1)) + __builtin_fabsf(d2));
                } else {
                    d = __builtin_amdgcn_sad_u8(j < 4 ? cur.g[j & 3] : nxt.g[j & 3], ctr[i], 0u);
                }
                wc[t][i] = *reinterpret_cast<const float*>(lut_bytes + ((d << (COPIES == 32 ? 7 : 6)) | lanec));
            }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const int j = t + i;
                const float n0 = j < 4 ? cur.c0[j & 3] : nxt.c0[j & 3];
                const float n1 = j < 4 ? cur.c1[j & 3] : nxt.c1[j & 3];
                const float n2 = j < 4 ? cur.c2[j & 3] : nxt.c2[j & 3];
                const float w = wc[t][i] * wsv[t];
                if constexpr (FMA) {
                    a01[i].x = __builtin_fmaf(n0, w, a01[i].x);
                    a01[i].y = __builtin_fmaf(n1, w, a01[i].y);
                    a2k[i].x = __builtin_fmaf(n2, w, a2k[i].x);
                } else {
                    a01[i].x = a01[i].x + n0 * w;
                    a01[i].y = a01[i].y + n1 * w;
                    a2k[i].x = a2k[i].x + n2 * w;
                }
                a2k[i].y = a2k[i].y + w;
            }
    };

    for (int ky = -R; ky <= R; ++ky) {
        const int aky = ky < 0 ? -ky : ky;
        set_progress_priority((ky + R) * 4 / (2 * R + 1));
        const int hw = ((const kconst int*)a.hw)[aky];
        const int k4 = (hw + 3) & ~3;
        const int nblk = ((hw + k4) >> 2) + 1;  // blocks cover kx = -k4 .. -k4 + 4 nblk - 1 >= hw
        const kconst float* const wsr =
            (const kconst float*)a.wsrow + (ky + R) * a.wst + (a.ra - k4);
        const int off = (ty + R + ky) * S + xc - k4;
        RtWin<JOINT> A, B;
        A.load(gplane, splane, off);
        int b = 0;
        for (; b + 2 <= nblk; b += 2) {  // two blocks per trip: the windows swap roles, no copies
            B.load(gplane, splane, off + 4 * (b + 1));
            block(A, B, wsr + 4 * b);
            A.load(gplane, splane, off + 4 * (b + 2));
            block(B, A, wsr + 4 * (b + 1));
        }
        if (b < nblk) {
            B.load(gplane, splane, off + 4 * (b + 1));
            block(A, B, wsr + 4 * b);
        }
    }

    uint32_t o[P];
    finish_outputs<P, false>(a01, a2k, o);
    store_px(a, ty0 + ty, tx0 + tx * P, o);
}

template <int COPIES, bool JOINT, bool FMA, bool ADAPTIVE>
static int launch_rt_c(const RtArgs& a, int lds, hipStream_t stream) {
    auto kern = stencil_rt_kernel<COPIES, JOINT, FMA, ADAPTIVE>;
    static std::atomic<unsigned long long> attr_devs{0};
    if (const int rc = ensure_dynamic_lds(reinterpret_cast<const void*>(kern), kLdsBudget, attr_devs)) return rc;
    note_launch(reinterpret_cast<const void*>(kern));
    const int tiles_y = (a.out_rows + kRtWaves * 4 - 1) / (kRtWaves * 4);
    const long long tiles = (long long)a.tiles_x * tiles_y;
    if (tiles == 0) return 0;
    if (tiles > 0x7fffffffLL) return VIP_ERR_INVALID_ARGUMENT;
    launch(kern, dim3((unsigned)tiles), dim3(kRtWaves * 64), lds, stream, a);
    return (int)hipGetLastError();
}

// LDS bytes of the runtime kernel for radius R with `copies` LUT copies, or 0 if it
// does not fit the CU.
static int rt_lds_bytes(int R, bool joint, bool adaptive, int copies) {
    const int L = round_up(R, 4);
    const int S = rt_stride(L);
    const long long bytes = 4LL * (joint ? 2 : 1) * rt_plane_words(R, L, S, kRtWaves) +
                            4LL * (adaptive ? 1536 : 768) * copies;
    return bytes <= kLdsBudget ? (int)bytes : 0;
}

template <bool FMA>
static int launch_rt(RtArgs a, bool joint, bool adaptive, hipStream_t stream) {
    if (a.R < 0 || a.R > kRtMaxRadius) return VIP_ERR_UNSUPPORTED_KSIZE;
    a.L = round_up(a.R, 4);
    a.S = rt_stride(a.L);
    a.tiles_x = (a.width + kRtTW - 1) / kRtTW;
    if (adaptive) {
        const int lds = rt_lds_bytes(a.R, false, true, 16);
        return lds ? launch_rt_c<16, false, FMA, true>(a, lds, stream) : VIP_ERR_UNSUPPORTED_KSIZE;
    }
    if (joint) {
        if (const int lds = rt_lds_bytes(a.R, true, false, 32)) return launch_rt_c<32, true, FMA, false>(a, lds, stream);
        const int lds = rt_lds_bytes(a.R, true, false, 16);
        return lds ? launch_rt_c<16, true, FMA, false>(a, lds, stream) : VIP_ERR_UNSUPPORTED_KSIZE;
    }
    const int lds = rt_lds_bytes(a.R, false, false, 32);
    return lds ? launch_rt_c<32, false, FMA, false>(a, lds, stream) : VIP_ERR_UNSUPPORTED_KSIZE;
}

int launch_stencil_rt(const RtArgs& a, bool joint, bool adaptive, bool fma, hipStream_t stream) {
    return fma ? launch_rt<true>(a, joint, adaptive, stream) : launch_rt<false>(a, joint, adaptive, stream);
}

int stencil_rt_max_radius(bool joint, bool adaptive) {
    for (int R = kRtMaxRadius; R >= 0; --R)
        if (rt_lds_bytes(R, joint, adaptive, joint ? 16 : (adaptive ? 16 : 32))) return R;
    return -1;
}

}  // namespace vip
