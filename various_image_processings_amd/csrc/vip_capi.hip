// extern "C" ABI of the MI355X bilateral-filter family (include/vip.h).
//
// Host-side responsibilities mirror the reference's Impl constructors
// (src/bilateral_filter_impl.cu:204-239, src/adaptive_bilateral_filter_impl.cu:117-152,
// src/bilateral_texture_filter_impl.cu:179-195): build the spatial and colour
// LUTs once per handle, own device scratch, validate arguments. Unlike the
// reference, run functions are asynchronous on the caller's stream and return a
// status instead of printing it.
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <cxxabi.h>
#include <dlfcn.h>
#include <new>
#include <string>
#include <vector>

#include "vip_stencil.hpp"

namespace vip {
int launch_bilateral_joint_fma(int radius, const StencilArgs& a, hipStream_t s);
int launch_bilateral_joint_mul(int radius, const StencilArgs& a, hipStream_t s);
int launch_bilateral_plain_fma(int radius, const StencilArgs& a, hipStream_t s);
int launch_bilateral_plain_mul(int radius, const StencilArgs& a, hipStream_t s);
int launch_adaptive_fma(int radius, const StencilArgs& a, hipStream_t s);
int launch_adaptive_mul(int radius, const StencilArgs& a, hipStream_t s);

static int launch_bilateral(int radius, bool joint, bool fma, const StencilArgs& a, hipStream_t s) {
    if (joint) return fma ? launch_bilateral_joint_fma(radius, a, s) : launch_bilateral_joint_mul(radius, a, s);
    return fma ? launch_bilateral_plain_fma(radius, a, s) : launch_bilateral_plain_mul(radius, a, s);
}
static int launch_adaptive(int radius, bool fma, const StencilArgs& a, hipStream_t s) {
    return fma ? launch_adaptive_fma(radius, a, s) : launch_adaptive_mul(radius, a, s);
}
int launch_gradient_u8(const uint8_t* src, float* dst, int width, int height, int ch, hipStream_t stream);
int launch_gradient_f32(const float* src, float* dst, int width, int height, int ch, bool fma, hipStream_t stream);
int launch_blur_rtv(const uint8_t* img, const float* mag, float* blurred, float* rtv, int width, int height,
                    int ksize, bool cpp, hipStream_t stream);
int launch_guide(const float* blurred, const float* rtv, uint8_t* guide, int width, int height, int ksize, bool cpp,
                 hipStream_t stream);
int launch_texture_guide_fused(const uint8_t* img, uint8_t* guide, int width, int height, int ksize, bool cpp,
                               hipStream_t stream);
int launch_texture_guide_fused_rows(const uint8_t* img, uint8_t* guide, int width, int lo, int hi, int gy0, int gy1,
                                    int ksize, bool cpp, hipStream_t stream);
int launch_texture_iteration_fused(const StencilArgs& a, int ksize, bool cpp, hipStream_t stream);

// LUT construction. CUDA profile: src/bilateral_filter_impl.cu:217-237 (float
// coefficient, std::exp(float) == expf). CPP profile: include/cpp/bilateral_filter.hpp:13-36
// (double coefficient, exp, stored as float). `2 * sigma * sigma` is a float
// expression in both.
static float space_weight(int r2, float sigma_space, int numerics) {
    const float two_s2 = 2 * sigma_space * sigma_space;
    const float cf = -1.f / two_s2;
    const double cd = -1. / (double)two_s2;
    return numerics == VIP_NUMERICS_CPP ? (float)std::exp((double)r2 * cd) : expf((float)r2 * cf);
}

// Quadrant table ws[|ky|][|kx|] of the templated kernels (radius <= kMaxRadius)
static void build_space_q(int radius, float sigma_space, int numerics, float* wsq /* kWsStride^2 */) {
    for (int i = 0; i < kWsStride * kWsStride; ++i) wsq[i] = 0.f;
    if (radius > kMaxRadius) return;  // the runtime-radius kernel reads its own table
    for (int ky = 0; ky <= radius; ++ky)
        for (int kx = 0; kx <= radius; ++kx) {
            const int r2 = kx * kx + ky * ky;
            if (r2 > radius * radius) continue;
            wsq[ky * kWsStride + kx] = space_weight(r2, sigma_space, numerics);
        }
}

// Tables of the runtime-radius kernel (vip_stencil_rt.hip), one device allocation:
// (2R+1) rows of wst floats, row ky + R holding ws(kx, ky) at kx + ra for kx in
// [-ra, ra + 8) (zero outside the disc), then the R+1 disc half-widths as ints.
struct RtTables {
    float* d = nullptr;
    int wst = 0, ra = 0;
};
static int upload_rt_tables(int radius, float sigma_space, int numerics, RtTables* t) {
    t->ra = round_up(radius, 4);
    t->wst = 2 * t->ra + 8;
    const int rows = 2 * radius + 1;
    const size_t nf = (size_t)rows * t->wst;
    float* host = (float*)calloc(nf + radius + 1, sizeof(float));
    if (!host) return (int)hipErrorOutOfMemory;
    int* hw = reinterpret_cast<int*>(host + nf);
    for (int ky = -radius; ky <= radius; ++ky) {
        const int h = isqrt_floor(radius * radius - ky * ky);
        if (ky >= 0) hw[ky] = h;
        for (int kx = -h; kx <= h; ++kx)
            host[(size_t)(ky + radius) * t->wst + kx + t->ra] = space_weight(kx * kx + ky * ky, sigma_space, numerics);
    }
    const size_t bytes = (nf + radius + 1) * sizeof(float);
    int rc = (int)hipMalloc(reinterpret_cast<void**>(&t->d), bytes);
    if (!rc) rc = (int)hipMemcpy(t->d, host, bytes, hipMemcpyHostToDevice);
    free(host);
    return rc;
}

static void build_color(int len, float sigma_color, int numerics, float* out) {
    const float two_s2 = 2 * sigma_color * sigma_color;
    const float cf = -1.f / two_s2;
    const double cd = -1. / (double)two_s2;
    for (int i = 0; i < len; ++i)
        out[i] = numerics == VIP_NUMERICS_CPP ? (float)std::exp((double)(i * i) * cd) : expf((float)(i * i) * cf);
}

// The largest ksize the reference runs for each filter: its kernels size dynamic
// shared memory from ksize with no cap, against CUDA's 48 KB default
// (src/bilateral_filter_impl.cu:252-254 and :272-275, src/adaptive_bilateral_filter_impl.cu:165-167;
// the texture filter's JBF is ksize 2k-1, src/bilateral_texture_filter_impl.cu:188).
// Even ksizes stay rejected: the reference sizes its tile for ksize - 1 halo columns but
// reads 2 * (ksize / 2), past the tile.
constexpr int kMaxKsizeBilateral = 65, kMaxKsizeJoint = 47, kMaxKsizeAdaptive = 63, kMaxKsizeTexture = 24;
static bool valid_ksize(int ksize, int max_ksize) { return ksize >= 1 && (ksize & 1) && ksize <= max_ksize; }

// vip_set_stencil_path: VIP_PATH_AUTO (templated kernels for radius 1..15, the
// runtime-radius kernel for 0 and 16..32) or VIP_PATH_RUNTIME (the runtime-radius
// kernel for every radius; a test and measurement knob). Process-wide.
static std::atomic<int> g_stencil_path{[] {
    const char* e = getenv("VIP_STENCIL_PATH");
    return e && atoi(e) == VIP_PATH_RUNTIME ? VIP_PATH_RUNTIME : VIP_PATH_AUTO;
}()};
static bool use_runtime_kernel(int radius) {
    return radius == 0 || radius > kMaxRadius || g_stencil_path.load(std::memory_order_relaxed) == VIP_PATH_RUNTIME;
}

// Returns the number of leading entries up to the last nonzero one in *nonzero.
static int upload_color(float** d_color, int len, float sigma_color, int numerics, int* nonzero) {
    float host[1536];
    build_color(len, sigma_color, numerics, host);
    int nz = len;
    while (nz > 0 && host[nz - 1] == 0.f) --nz;
    *nonzero = nz;
    VIP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(d_color), sizeof(float) * len));
    VIP_HIP_CHECK(hipMemcpy(*d_color, host, sizeof(float) * len, hipMemcpyHostToDevice));
    return 0;
}

static void fill_args(StencilArgs& a, int width, const uint8_t* src, size_t src_pitch, const uint8_t* guide,
                      size_t guide_pitch, uint8_t* dst, size_t dst_pitch, int out_rows, int src_row0, int row_lo,
                      int row_hi, const float* d_color, int lut_nonzero, const float* d_fold, const float* wsq) {
    a.src = src;
    a.guide = guide;
    a.dst = dst;
    a.src_pitch = (long long)src_pitch;
    a.guide_pitch = (long long)guide_pitch;
    a.dst_pitch = (long long)dst_pitch;
    a.width = width;
    a.out_rows = out_rows;
    a.src_row0 = src_row0;
    a.row_lo = row_lo;
    a.row_hi = row_hi;
    a.tiles_x = (width + kTW - 1) / kTW;
    const auto al4 = [](const void* p, size_t pitch) { return ((uintptr_t)p % 4 == 0) && (pitch % 4 == 0); };
    a.aligned = al4(src, src_pitch) && al4(guide, guide_pitch);
    a.dst_aligned = ((uintptr_t)dst % 8 == 0) && (dst_pitch % 8 == 0);
    a.color = d_color;
    a.lut_nonzero = lut_nonzero;
    a.fold = d_fold;
    a.inflight = 1;
    a.nframes = 1;
    a.tiles_frame = 0;
    a.free_cus = 0;
    a.tail_full = 0;  // set per launch (launch_*_ne: tiles_total, or plan_tail)
    a.tail_shift = 0;
    for (int f = 0; f < kMaxBatchFrames; ++f) {
        a.fsrc[f] = src;
        a.fdst[f] = dst;
    }
    std::memcpy(a.ws, wsq, sizeof(a.ws));
}

// Frames in flight on the current device, for the plain bilateral kernel's small-frame
// tiling: the distinct streams among the device's last 8 plain-bilateral launches, at most
// 4 (the hardware queues a process gets by default, GPU_MAX_HW_QUEUES). One stream counts
// 1. The count is of streams, not of launches outstanding: a caller that alternates two
// streams but waits for each frame before the next also counts 2 (and gets the throughput
// tiling, e.g. C1's 14.5 instead of 10.7 us for a lone 512 x 512 frame), and after a change
// of streams the ring keeps the old count for up to 8 launches. Such a caller fixes the
// count with vip_bilateral_set_frames_in_flight(1). (Checking each recorded stream with
// hipStreamQuery would cost host time per launch and could touch a destroyed stream.) The
// choice changes the tiling only, never the bytes.
static std::atomic<int> g_bil_inflight{0};  // vip_bilateral_set_frames_in_flight: 0 = counted
static int frames_in_flight(hipStream_t s) {
    constexpr int kDevs = 16, kRing = 8;
    static std::atomic<uintptr_t> recent[kDevs][kRing];
    static std::atomic<unsigned> pos[kDevs];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    dev &= kDevs - 1;
    recent[dev][pos[dev].fetch_add(1, std::memory_order_relaxed) % kRing].store((uintptr_t)s + 1,
                                                                                 std::memory_order_relaxed);
    uintptr_t seen[kRing];
    int n = 0;
    for (int i = 0; i < kRing; ++i) {
        const uintptr_t v = recent[dev][i].load(std::memory_order_relaxed);
        bool dup = v == 0;
        for (int j = 0; j < n && !dup; ++j) dup = seen[j] == v;
        if (!dup) seen[n++] = v;
    }
    const int forced = g_bil_inflight.load(std::memory_order_relaxed);
    if (forced) return forced;
    return n < 1 ? 1 : (n > 4 ? 4 : n);
}

// vip_bilateral_set_waves: one process-wide value, read by every bilateral launcher
static bool valid_waves(int w) { return w == 0 || w == 16 || w == 8 || w == 4; }
static std::atomic<int> g_bil_waves{[] {
    const char* e = getenv("VIP_BIL_WAVES");
    const int w = e ? atoi(e) : 0;
    return valid_waves(w) ? w : 0;
}()};
int bilateral_forced_waves() { return g_bil_waves.load(std::memory_order_relaxed); }
static std::atomic<int> g_bil_wide{[] {
    const char* e = getenv("VIP_BIL_WIDE");
    const int w = e ? atoi(e) : 0;
    return w >= 0 && w <= 2 ? w : 0;
}()};
int bilateral_forced_wide() { return g_bil_wide.load(std::memory_order_relaxed); }

}  // namespace vip

using namespace vip;

struct vip_bilateral_s {
    int width, height, ksize, radius, numerics, lut_nonzero;
    float* d_color;
    float* d_fold;  // joint kernel's folded tables (small sigma_color, radius <= kSatMaxR), or null
    RtTables rt;    // runtime-radius kernel tables
    float wsq[kWsStride * kWsStride];
};

struct vip_adaptive_s {
    int width, height, ksize, radius, numerics, lut_nonzero;
    float* d_color;
    RtTables rt;
    float wsq[kWsStride * kWsStride];
};

// The handle owns three u8x3 frames: the two ping-pong frames and the guide. The
// reference's Impl also holds f32 magnitude, blurred and rtv buffers
// (src/bilateral_texture_filter_impl.cu:189-194, 20 B/px); here the guide stage keeps
// them in LDS, and the stage entry points (vip_texture_blur_rtv / _guide) write the
// caller's buffers, so the handle holds none.
struct vip_texture_s {
    int width, height, ksize, nitr, numerics;
    int mode;  // VIP_TEXTURE_TWO_LAUNCH or VIP_TEXTURE_FUSED (vip_texture_set_mode)
    vip_bilateral_t jbf;
    uint8_t* d_ping[2];
    uint8_t* d_guide;
};

static RtArgs rt_args(const RtTables& t, int radius, int width, const uint8_t* src, size_t src_pitch,
                      const uint8_t* guide, size_t guide_pitch, uint8_t* dst, size_t dst_pitch, int out_rows,
                      int src_row0, int row_lo, int row_hi, const float* d_color) {
    RtArgs a{};
    a.src = src;
    a.guide = guide;
    a.dst = dst;
    a.src_pitch = (long long)src_pitch;
    a.guide_pitch = (long long)guide_pitch;
    a.dst_pitch = (long long)dst_pitch;
    a.width = width;
    a.out_rows = out_rows;
    a.src_row0 = src_row0;
    a.row_lo = row_lo;
    a.row_hi = row_hi;
    const auto al4 = [](const void* p, size_t pitch) { return ((uintptr_t)p % 4 == 0) && (pitch % 4 == 0); };
    a.aligned = al4(src, src_pitch) && al4(guide, guide_pitch);
    a.dst_aligned = ((uintptr_t)dst % 4 == 0) && (dst_pitch % 4 == 0);
    a.color = d_color;
    a.wsrow = t.d;
    a.hw = reinterpret_cast<const int*>(t.d + (size_t)(2 * radius + 1) * t.wst);
    a.R = radius;
    a.wst = t.wst;
    a.ra = t.ra;
    return a;
}

namespace {
thread_local const void* g_launched[16];  // distinct kernels launched since the last query
thread_local int g_nlaunched = 0;

// vip_kernel_timing_*: a per-thread pool of event pairs on one device, the kernel of each
// recorded launch, and how many of the `cap` slots are used
struct KernelTiming {
    std::vector<hipEvent_t> ev;  // 2 per slot: start, stop
    std::vector<const void*> kern;
    int device = -1, cap = 0, n = 0;
    bool on = false;
    ~KernelTiming() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
};
thread_local KernelTiming g_timing;

// The profiler's name of a kernel handle: the exported symbol's mangled name (dladdr; the
// runtime's lookup is the fallback), demangled, without the parameter list.
std::string kernel_name(const void* kern) {
    Dl_info info{};
    const char* mangled = dladdr(kern, &info) && info.dli_sname && info.dli_saddr == kern
                              ? info.dli_sname
                              : hipKernelNameRefByPtr(kern, nullptr);
    if (!mangled) return {};
    int st = 0;
    char* dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
    std::string name = st == 0 && dem ? dem : mangled;
    std::free(dem);
    const size_t paren = name.find('(');
    if (paren != std::string::npos) name.resize(paren);  // the profiler summaries' key: no parameter list
    return name;
}
}  // namespace

namespace vip {
void note_launch(const void* kern) {
    for (int i = 0; i < g_nlaunched; ++i)
        if (g_launched[i] == kern) return;
    if (g_nlaunched < 16) g_launched[g_nlaunched++] = kern;
}

LaunchEvents timing_events(const void* kern, hipStream_t stream) {
    KernelTiming& t = g_timing;
    if (!t.on || t.n >= t.cap) return {nullptr, nullptr};
    int dev = -1;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipGetDevice(&dev) != hipSuccess || dev != t.device || hipStreamIsCapturing(stream, &cap) != hipSuccess ||
        cap != hipStreamCaptureStatusNone)
        return {nullptr, nullptr};
    t.kern[t.n] = kern;
    const int i = t.n++;
    return {t.ev[2 * i], t.ev[2 * i + 1]};
}
}  // namespace vip

extern "C" {

int vip_launched_kernels(char* buf, size_t len) {
    std::string all;
    for (int i = 0; i < g_nlaunched; ++i) {
        const std::string name = kernel_name(g_launched[i]);
        if (!name.empty()) all += (all.empty() ? "" : "\n") + name;
    }
    if (buf && len) {
        g_nlaunched = 0;  // a size query (no buffer) keeps the list
        const size_t n = all.size() < len - 1 ? all.size() : len - 1;
        std::memcpy(buf, all.data(), n);
        buf[n] = 0;
    }
    return (int)all.size();
}

int vip_kernel_timing_begin(int capacity) {
    if (capacity < 1 || capacity > (1 << 16)) return VIP_ERR_INVALID_ARGUMENT;
    KernelTiming& t = g_timing;
    int dev = 0;
    VIP_HIP_CHECK(hipGetDevice(&dev));
    if (dev != t.device) {  // events belong to the device current at their creation
        for (hipEvent_t e : t.ev) (void)hipEventDestroy(e);
        t.ev.clear();
        t.device = dev;
    }
    while ((int)t.ev.size() < 2 * capacity) {
        hipEvent_t e = nullptr;
        VIP_HIP_CHECK(hipEventCreate(&e));
        t.ev.push_back(e);
    }
    t.kern.assign((size_t)capacity, nullptr);
    t.cap = capacity;
    t.n = 0;
    t.on = true;
    return 0;
}

int vip_kernel_timing_end(void) {
    g_timing.on = false;
    return g_timing.n;
}

int vip_kernel_timing_get(int index, float* ms, char* name, size_t len) {
    KernelTiming& t = g_timing;
    if (index < 0 || index >= t.n || t.on || !ms) return VIP_ERR_INVALID_ARGUMENT;
    VIP_HIP_CHECK(hipEventSynchronize(t.ev[2 * index + 1]));
    VIP_HIP_CHECK(hipEventElapsedTime(ms, t.ev[2 * index], t.ev[2 * index + 1]));
    if (name && len) {
        const std::string s = kernel_name(t.kern[index]);
        const size_t n = s.size() < len - 1 ? s.size() : len - 1;
        std::memcpy(name, s.data(), n);
        name[n] = 0;
    }
    return 0;
}

int vip_abi_version(void) { return VIP_ABI_VERSION; }
int vip_max_radius(void) { return kRtMaxRadius; }

int vip_max_ksize(int filter) {
    switch (filter) {
        case VIP_FILTER_BILATERAL: return kMaxKsizeBilateral;
        case VIP_FILTER_JOINT: return kMaxKsizeJoint;
        case VIP_FILTER_ADAPTIVE: return kMaxKsizeAdaptive;
        case VIP_FILTER_TEXTURE: return kMaxKsizeTexture;
        default: return VIP_ERR_INVALID_ARGUMENT;
    }
}

int vip_set_stencil_path(int path) {
    if (path != VIP_PATH_AUTO && path != VIP_PATH_RUNTIME) return VIP_ERR_INVALID_ARGUMENT;
    g_stencil_path.store(path, std::memory_order_relaxed);
    return 0;
}

int vip_bilateral_set_waves(int waves) {
    if (!valid_waves(waves)) return VIP_ERR_INVALID_ARGUMENT;
    g_bil_waves.store(waves, std::memory_order_relaxed);
    return 0;
}

int vip_bilateral_set_wide(int mode) {
    if (mode < 0 || mode > 2) return VIP_ERR_INVALID_ARGUMENT;
    g_bil_wide.store(mode, std::memory_order_relaxed);
    return 0;
}

int vip_bilateral_set_frames_in_flight(int n) {
    if (n < 0 || n > 4) return VIP_ERR_INVALID_ARGUMENT;
    g_bil_inflight.store(n, std::memory_order_relaxed);
    return 0;
}

const char* vip_error_string(int code) {
    switch (code) {
        case 0: return "success";
        case VIP_ERR_INVALID_ARGUMENT: return "invalid argument";
        case VIP_ERR_UNSUPPORTED_KSIZE:
            return "unsupported ksize (odd, 1..65 bilateral, 1..47 joint bilateral, 1..63 adaptive; texture 1..24)";
        case VIP_ERR_ALIASING: return "source and destination alias";
        default: return hipGetErrorString((hipError_t)code);
    }
}

int vip_malloc(void** d_ptr, size_t bytes) {
    if (!d_ptr) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipMalloc(d_ptr, bytes);
}
int vip_free(void* d_ptr) { return (int)hipFree(d_ptr); }
int vip_upload(void* d_dst, const void* h_src, size_t bytes) {
    return (int)hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice);
}
int vip_download(void* h_dst, const void* d_src, size_t bytes) {
    return (int)hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost);
}
int vip_device_synchronize(void) { return (int)hipDeviceSynchronize(); }
int vip_device_count(int* count) {
    if (!count) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipGetDeviceCount(count);
}
int vip_set_device(int device) { return (int)hipSetDevice(device); }
int vip_get_device(int* device) {
    if (!device) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipGetDevice(device);
}
int vip_stream_synchronize(void* stream) { return (int)hipStreamSynchronize((hipStream_t)stream); }
int vip_host_alloc(void** h_ptr, size_t bytes) {
    if (!h_ptr) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipHostMalloc(h_ptr, bytes, hipHostMallocDefault);
}
int vip_host_free(void* h_ptr) { return (int)hipHostFree(h_ptr); }
int vip_upload_async(void* d_dst, const void* h_src, size_t bytes, void* stream) {
    return (int)hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
}
int vip_download_async(void* h_dst, const void* d_src, size_t bytes, void* stream) {
    return (int)hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
}
int vip_stream_create(void** stream) {
    if (!stream) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipStreamCreateWithFlags(reinterpret_cast<hipStream_t*>(stream), hipStreamNonBlocking);
}
int vip_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }
int vip_event_create(void** event) {
    if (!event) return VIP_ERR_INVALID_ARGUMENT;
    return (int)hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(event), hipEventDisableTiming);
}
int vip_event_destroy(void* event) { return (int)hipEventDestroy((hipEvent_t)event); }
int vip_event_record(void* event, void* stream) { return (int)hipEventRecord((hipEvent_t)event, (hipStream_t)stream); }
int vip_stream_wait_event(void* stream, void* event) {
    return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
}
int vip_event_synchronize(void* event) { return (int)hipEventSynchronize((hipEvent_t)event); }

// ---------------------------------------------------------------- bilateral
// Folded joint-kernel tables: table t (the t-th distinct r^2 of the disc, ascending)
// entry d = RN(ws(r^2) * wc[d]) for d < kFoldEntries -- the product the kernel's unfolded
// taps form (one float multiply), so results are unchanged. The kernel reads them behind
// the saturating address (SatLut) when wc is zero from its DZ on.
static int upload_fold(vip_bilateral_s* h, float sigma_color) {
    const int R = h->radius;
    float wc[768];
    build_color(768, sigma_color, h->numerics, wc);
    float fold[(kSatMaxR * kSatMaxR + 1) * kFoldEntries];
    int ntab = 0;
    for (int v = 0; v <= R * R; ++v) {
        if (!is_disc_r2(R, v)) continue;
        float ws = 0.f;  // the spatial weight of any tap at squared distance v
        for (int y = 0; y <= R; ++y)
            for (int x = 0; x <= R; ++x)
                if (x * x + y * y == v) ws = h->wsq[y * kWsStride + x];
        for (int d = 0; d < kFoldEntries; ++d) fold[ntab * kFoldEntries + d] = wc[d] * ws;
        ++ntab;
    }
    VIP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->d_fold), sizeof(float) * kFoldEntries * ntab));
    VIP_HIP_CHECK(hipMemcpy(h->d_fold, fold, sizeof(float) * kFoldEntries * ntab, hipMemcpyHostToDevice));
    return 0;
}

int vip_bilateral_create(vip_bilateral_t* out, int width, int height, int ksize, float sigma_space, float sigma_color,
                         int numerics) {
    if (!out || width <= 0 || height <= 0) return VIP_ERR_INVALID_ARGUMENT;
    if (!valid_ksize(ksize, kMaxKsizeBilateral)) return VIP_ERR_UNSUPPORTED_KSIZE;
    auto* h = new (std::nothrow) vip_bilateral_s();
    if (!h) return (int)hipErrorOutOfMemory;
    h->width = width;
    h->height = height;
    h->ksize = ksize;
    h->radius = ksize / 2;
    h->numerics = numerics == VIP_NUMERICS_CPP ? VIP_NUMERICS_CPP : VIP_NUMERICS_CUDA;
    build_space_q(h->radius, sigma_space, h->numerics, h->wsq);
    int rc = upload_color(&h->d_color, 768, sigma_color, h->numerics, &h->lut_nonzero);
    if (!rc) rc = upload_rt_tables(h->radius, sigma_space, h->numerics, &h->rt);
    if (!rc && h->lut_nonzero < kFoldEntries && h->radius <= kSatMaxR) rc = upload_fold(h, sigma_color);
    if (rc) {
        vip_bilateral_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

int vip_bilateral_destroy(vip_bilateral_t h) {
    if (!h) return 0;
    if (h->d_fold) (void)hipFree(h->d_fold);
    if (h->rt.d) (void)hipFree(h->rt.d);
    const int rc = h->d_color ? (int)hipFree(h->d_color) : 0;
    delete h;
    return rc;
}

int vip_bilateral_run_rows(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, const uint8_t* d_guide,
                           size_t guide_pitch, uint8_t* d_dst, size_t dst_pitch, int out_rows, int src_row0,
                           int row_lo, int row_hi, void* stream) {
    // d_src (and d_guide) hold the handle's height rows: every read clamps into
    // [row_lo, row_hi), so that range must lie inside them
    if (!h || !d_src || !d_dst || out_rows < 0 || row_lo < 0 || row_hi > h->height || row_lo >= row_hi)
        return VIP_ERR_INVALID_ARGUMENT;
    if (d_dst == d_src || (d_guide && d_dst == d_guide)) return VIP_ERR_ALIASING;
    const bool joint = d_guide != nullptr;
    if (joint && h->ksize > kMaxKsizeJoint) return VIP_ERR_UNSUPPORTED_KSIZE;
    if (use_runtime_kernel(h->radius)) {
        const RtArgs r = rt_args(h->rt, h->radius, h->width, d_src, src_pitch, joint ? d_guide : d_src,
                                 joint ? guide_pitch : src_pitch, d_dst, dst_pitch, out_rows, src_row0, row_lo,
                                 row_hi, h->d_color);
        return launch_stencil_rt(r, joint, false, h->numerics == VIP_NUMERICS_CUDA, (hipStream_t)stream);
    }
    StencilArgs a;
    fill_args(a, h->width, d_src, src_pitch, joint ? d_guide : d_src, joint ? guide_pitch : src_pitch, d_dst,
              dst_pitch, out_rows, src_row0, row_lo, row_hi, h->d_color, h->lut_nonzero, joint ? h->d_fold : nullptr,
              h->wsq);
    if (!joint) a.inflight = frames_in_flight((hipStream_t)stream);
    return launch_bilateral(h->radius, joint, h->numerics == VIP_NUMERICS_CUDA, a, (hipStream_t)stream);
}

// Frames [f0, f0 + m) of a batch in one StencilArgs (m <= kMaxBatchFrames): frame 0's
// pointers in src/dst, every frame's in fsrc/fdst; dword tile loads / qword stores only
// when every frame allows them.
static void fill_batch(StencilArgs& a, int m, const uint8_t* const* srcs, size_t src_pitch, uint8_t* const* dsts,
                       size_t dst_pitch) {
    a.nframes = m;
    for (int f = 0; f < kMaxBatchFrames; ++f) {
        a.fsrc[f] = srcs[f < m ? f : 0];
        a.fdst[f] = dsts[f < m ? f : 0];
        a.aligned = a.aligned && (uintptr_t)a.fsrc[f] % 4 == 0 && src_pitch % 4 == 0;
        a.dst_aligned = a.dst_aligned && (uintptr_t)a.fdst[f] % 8 == 0 && dst_pitch % 8 == 0;
    }
}

// Batch arguments: every pointer set, no output that is also an input of the batch.
static int check_batch(int n, const uint8_t* const* srcs, uint8_t* const* dsts) {
    if (n < 0 || (n > 0 && (!srcs || !dsts))) return VIP_ERR_INVALID_ARGUMENT;
    for (int f = 0; f < n; ++f)
        if (!srcs[f] || !dsts[f]) return VIP_ERR_INVALID_ARGUMENT;
    for (int f = 0; f < n; ++f)
        for (int g = 0; g < n; ++g)
            if (dsts[f] == srcs[g]) return VIP_ERR_ALIASING;
    return 0;
}

int vip_bilateral_run_rows_batch(vip_bilateral_t h, int n, const uint8_t* const* d_srcs, size_t src_pitch,
                                 uint8_t* const* d_dsts, size_t dst_pitch, int out_rows, int src_row0, int row_lo,
                                 int row_hi, int free_cus, void* stream) {
    if (!h || out_rows < 0 || row_lo < 0 || row_hi > h->height || row_lo >= row_hi || free_cus < 0)
        return VIP_ERR_INVALID_ARGUMENT;
    if (const int rc = check_batch(n, d_srcs, d_dsts)) return rc;
    const hipStream_t s = (hipStream_t)stream;
    if (use_runtime_kernel(h->radius) || h->radius > kBatchMaxRadius) {  // no multi-frame form: frame by frame
        for (int f = 0; f < n; ++f)
            if (const int rc = vip_bilateral_run_rows(h, d_srcs[f], src_pitch, nullptr, 0, d_dsts[f], dst_pitch,
                                                      out_rows, src_row0, row_lo, row_hi, stream))
                return rc;
        return 0;
    }
    for (int f0 = 0; f0 < n; f0 += kMaxBatchFrames) {
        const int m = n - f0 < kMaxBatchFrames ? n - f0 : kMaxBatchFrames;
        StencilArgs a;
        fill_args(a, h->width, d_srcs[f0], src_pitch, d_srcs[f0], src_pitch, d_dsts[f0], dst_pitch, out_rows,
                  src_row0, row_lo, row_hi, h->d_color, h->lut_nonzero, nullptr, h->wsq);
        fill_batch(a, m, d_srcs + f0, src_pitch, d_dsts + f0, dst_pitch);
        a.inflight = frames_in_flight(s);
        a.free_cus = free_cus;
        if (const int rc = launch_bilateral(h->radius, false, h->numerics == VIP_NUMERICS_CUDA, a, s)) return rc;
    }
    return 0;
}

int vip_bilateral_run(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                      void* stream) {
    if (!h) return VIP_ERR_INVALID_ARGUMENT;
    return vip_bilateral_run_rows(h, d_src, src_pitch, nullptr, 0, d_dst, dst_pitch, h->height, 0, 0, h->height,
                                  stream);
}

int vip_joint_bilateral_run(vip_bilateral_t h, const uint8_t* d_src, size_t src_pitch, const uint8_t* d_guide,
                            size_t guide_pitch, uint8_t* d_dst, size_t dst_pitch, void* stream) {
    if (!h || !d_guide) return VIP_ERR_INVALID_ARGUMENT;
    return vip_bilateral_run_rows(h, d_src, src_pitch, d_guide, guide_pitch, d_dst, dst_pitch, h->height, 0, 0,
                                  h->height, stream);
}

// ---------------------------------------------------------------- adaptive
int vip_adaptive_create(vip_adaptive_t* out, int width, int height, int ksize, float sigma_space, float sigma_color,
                        int numerics) {
    if (!out || width <= 0 || height <= 0) return VIP_ERR_INVALID_ARGUMENT;
    if (!valid_ksize(ksize, kMaxKsizeAdaptive)) return VIP_ERR_UNSUPPORTED_KSIZE;
    auto* h = new (std::nothrow) vip_adaptive_s();
    if (!h) return (int)hipErrorOutOfMemory;
    h->width = width;
    h->height = height;
    h->ksize = ksize;
    h->radius = ksize / 2;
    h->numerics = numerics == VIP_NUMERICS_CPP ? VIP_NUMERICS_CPP : VIP_NUMERICS_CUDA;
    build_space_q(h->radius, sigma_space, h->numerics, h->wsq);
    // the reference's table is 512*3 long (src/adaptive_bilateral_filter_impl.cu:5)
    int rc = upload_color(&h->d_color, 1536, sigma_color, h->numerics, &h->lut_nonzero);
    if (!rc) rc = upload_rt_tables(h->radius, sigma_space, h->numerics, &h->rt);
    if (rc) {
        vip_adaptive_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

int vip_adaptive_destroy(vip_adaptive_t h) {
    if (!h) return 0;
    if (h->rt.d) (void)hipFree(h->rt.d);
    const int rc = h->d_color ? (int)hipFree(h->d_color) : 0;
    delete h;
    return rc;
}

int vip_adaptive_run_rows(vip_adaptive_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                          int out_rows, int src_row0, int row_lo, int row_hi, void* stream) {
    if (!h || !d_src || !d_dst || out_rows < 0 || row_lo < 0 || row_hi > h->height || row_lo >= row_hi)
        return VIP_ERR_INVALID_ARGUMENT;
    if (d_dst == d_src) return VIP_ERR_ALIASING;
    if (use_runtime_kernel(h->radius)) {
        const RtArgs r = rt_args(h->rt, h->radius, h->width, d_src, src_pitch, d_src, src_pitch, d_dst, dst_pitch,
                                 out_rows, src_row0, row_lo, row_hi, h->d_color);
        return launch_stencil_rt(r, false, true, h->numerics == VIP_NUMERICS_CUDA, (hipStream_t)stream);
    }
    StencilArgs a;
    fill_args(a, h->width, d_src, src_pitch, d_src, src_pitch, d_dst, dst_pitch, out_rows, src_row0, row_lo, row_hi,
              h->d_color, h->lut_nonzero, nullptr, h->wsq);
    return launch_adaptive(h->radius, h->numerics == VIP_NUMERICS_CUDA, a, (hipStream_t)stream);
}

int vip_adaptive_run_rows_batch(vip_adaptive_t h, int n, const uint8_t* const* d_srcs, size_t src_pitch,
                                uint8_t* const* d_dsts, size_t dst_pitch, int out_rows, int src_row0, int row_lo,
                                int row_hi, int free_cus, void* stream) {
    if (!h || out_rows < 0 || row_lo < 0 || row_hi > h->height || row_lo >= row_hi || free_cus < 0)
        return VIP_ERR_INVALID_ARGUMENT;
    if (const int rc = check_batch(n, d_srcs, d_dsts)) return rc;
    const hipStream_t s = (hipStream_t)stream;
    if (use_runtime_kernel(h->radius) || h->radius > kBatchMaxRadius) {  // no multi-frame form: frame by frame
        for (int f = 0; f < n; ++f)
            if (const int rc = vip_adaptive_run_rows(h, d_srcs[f], src_pitch, d_dsts[f], dst_pitch, out_rows, src_row0,
                                                     row_lo, row_hi, stream))
                return rc;
        return 0;
    }
    for (int f0 = 0; f0 < n; f0 += kMaxBatchFrames) {
        const int m = n - f0 < kMaxBatchFrames ? n - f0 : kMaxBatchFrames;
        StencilArgs a;
        fill_args(a, h->width, d_srcs[f0], src_pitch, d_srcs[f0], src_pitch, d_dsts[f0], dst_pitch, out_rows,
                  src_row0, row_lo, row_hi, h->d_color, h->lut_nonzero, nullptr, h->wsq);
        fill_batch(a, m, d_srcs + f0, src_pitch, d_dsts + f0, dst_pitch);
        a.free_cus = free_cus;
        if (const int rc = launch_adaptive(h->radius, h->numerics == VIP_NUMERICS_CUDA, a, s)) return rc;
    }
    return 0;
}

int vip_adaptive_run(vip_adaptive_t h, const uint8_t* d_src, size_t src_pitch, uint8_t* d_dst, size_t dst_pitch,
                     void* stream) {
    if (!h) return VIP_ERR_INVALID_ARGUMENT;
    return vip_adaptive_run_rows(h, d_src, src_pitch, d_dst, dst_pitch, h->height, 0, 0, h->height, stream);
}

// ---------------------------------------------------------------- gradient
int vip_gradient_u8(const uint8_t* d_src, float* d_dst, int width, int height, int src_ch, int numerics,
                    void* stream) {
    (void)numerics;  // u8 arithmetic is exact in both profiles
    if (!d_src || !d_dst || width <= 0 || height <= 0) return VIP_ERR_INVALID_ARGUMENT;
    return launch_gradient_u8(d_src, d_dst, width, height, src_ch, (hipStream_t)stream);
}

int vip_gradient_f32(const float* d_src, float* d_dst, int width, int height, int src_ch, int numerics,
                     void* stream) {
    if (!d_src || !d_dst || width <= 0 || height <= 0) return VIP_ERR_INVALID_ARGUMENT;
    return launch_gradient_f32(d_src, d_dst, width, height, src_ch, numerics != VIP_NUMERICS_CPP,
                               (hipStream_t)stream);
}

// ---------------------------------------------------------------- texture
int vip_texture_destroy(vip_texture_t h) {
    if (!h) return 0;
    vip_bilateral_destroy(h->jbf);
    (void)hipFree(h->d_ping[0]);
    (void)hipFree(h->d_ping[1]);
    (void)hipFree(h->d_guide);
    delete h;
    return 0;
}

int vip_texture_create(vip_texture_t* out, int width, int height, int ksize, int nitr, int numerics) {
    if (!out || width <= 0 || height <= 0 || nitr < 0) return VIP_ERR_INVALID_ARGUMENT;
    // any ksize 1..24 (even too); the embedded JBF has ksize 2k-1 <= 47
    // (src/bilateral_texture_filter_impl.cu:188)
    if (ksize < 1 || ksize > kMaxKsizeTexture) return VIP_ERR_UNSUPPORTED_KSIZE;
    auto* h = new (std::nothrow) vip_texture_s();
    if (!h) return (int)hipErrorOutOfMemory;
    h->width = width;
    h->height = height;
    h->ksize = ksize;
    h->nitr = nitr;
    h->numerics = numerics == VIP_NUMERICS_CPP ? VIP_NUMERICS_CPP : VIP_NUMERICS_CUDA;
    const size_t frame = vip_texture_scratch_bytes(width, height) / 3;
    int rc = vip_bilateral_create(&h->jbf, width, height, 2 * ksize - 1, (float)(ksize - 1), 1.73205080757f,
                                  h->numerics);
    if (!rc) rc = (int)hipMalloc(reinterpret_cast<void**>(&h->d_ping[0]), frame);
    if (!rc) rc = (int)hipMalloc(reinterpret_cast<void**>(&h->d_ping[1]), frame);
    if (!rc) rc = (int)hipMalloc(reinterpret_cast<void**>(&h->d_guide), frame);
    if (rc) {
        vip_texture_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

size_t vip_texture_scratch_bytes(int width, int height) {
    if (width <= 0 || height <= 0) return 0;
    return 3 * ((size_t)width * height * 3);  // two ping-pong frames + the guide, u8x3 each
}

int vip_texture_set_mode(vip_texture_t h, int mode) {
    if (!h || (mode != VIP_TEXTURE_TWO_LAUNCH && mode != VIP_TEXTURE_FUSED)) return VIP_ERR_INVALID_ARGUMENT;
    if (mode == VIP_TEXTURE_FUSED && h->ksize != 5) return VIP_ERR_UNSUPPORTED_KSIZE;
    h->mode = mode;
    return 0;
}

int vip_texture_blur_rtv(vip_texture_t h, const uint8_t* d_image, const float* d_magnitude, float* d_blurred,
                         float* d_rtv, void* stream) {
    if (!h || !d_image || !d_magnitude || !d_blurred || !d_rtv) return VIP_ERR_INVALID_ARGUMENT;
    return launch_blur_rtv(d_image, d_magnitude, d_blurred, d_rtv, h->width, h->height, h->ksize,
                           h->numerics == VIP_NUMERICS_CPP, (hipStream_t)stream);
}

int vip_texture_guide(vip_texture_t h, const float* d_blurred, const float* d_rtv, uint8_t* d_guide, void* stream) {
    if (!h || !d_blurred || !d_rtv || !d_guide) return VIP_ERR_INVALID_ARGUMENT;
    return launch_guide(d_blurred, d_rtv, d_guide, h->width, h->height, h->ksize, h->numerics == VIP_NUMERICS_CPP,
                        (hipStream_t)stream);
}

static int texture_run(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, void* stream, void* const* events) {
    if (!h || !d_src || !d_dst) return VIP_ERR_INVALID_ARGUMENT;
    const hipStream_t s = (hipStream_t)stream;
    const size_t bytes = (size_t)h->width * h->height * 3;
    const size_t pitch = (size_t)h->width * 3;
    if (h->nitr == 0) {
        if (events) VIP_HIP_CHECK(hipEventRecord((hipEvent_t)events[0], s));
        if (d_src != d_dst) VIP_HIP_CHECK(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, s));
        return 0;
    }
    const uint8_t* cur = d_src;
    if (d_src == d_dst) {  // the last JBF must not write the frame it reads
        VIP_HIP_CHECK(hipMemcpyAsync(h->d_ping[1], d_src, bytes, hipMemcpyDeviceToDevice, s));
        cur = h->d_ping[1];
    }
    for (int it = 0; it < h->nitr; ++it) {
        uint8_t* next = (it == h->nitr - 1) ? d_dst : (cur == h->d_ping[0] ? h->d_ping[1] : h->d_ping[0]);
        // gradient -> blur/mRTV -> guide fused in LDS (one launch), then the JBF
        if (events) VIP_HIP_CHECK(hipEventRecord((hipEvent_t)events[2 * it], s));
        int rc;
        if (h->mode == VIP_TEXTURE_FUSED) {  // guide + JBF in one launch, the guide stays in LDS
            const vip_bilateral_s* j = h->jbf;
            StencilArgs a;
            fill_args(a, h->width, cur, pitch, cur, pitch, next, pitch, h->height, 0, 0, h->height, j->d_color,
                      j->lut_nonzero, nullptr, j->wsq);
            rc = launch_texture_iteration_fused(a, h->ksize, h->numerics == VIP_NUMERICS_CPP, s);
            if (!rc && events) rc = (int)hipEventRecord((hipEvent_t)events[2 * it + 1], s);
        } else {
            rc = launch_texture_guide_fused(cur, h->d_guide, h->width, h->height, h->ksize,
                                            h->numerics == VIP_NUMERICS_CPP, s);
            if (!rc && events) rc = (int)hipEventRecord((hipEvent_t)events[2 * it + 1], s);
            if (!rc) rc = vip_joint_bilateral_run(h->jbf, cur, pitch, h->d_guide, pitch, next, pitch, stream);
        }
        if (rc) return rc;
        cur = next;
    }
    if (events) VIP_HIP_CHECK(hipEventRecord((hipEvent_t)events[2 * h->nitr], s));
    return 0;
}

// Impl::execute (src/bilateral_texture_filter_impl.cu:199-214) without the
// nitr + 2 device-to-device copies: iteration i reads X_i and writes X_{i+1},
// X_0 = d_src, X_nitr = d_dst, intermediates alternate between two scratch frames.
// Each iteration is two launches: the fused guide stage and the joint bilateral.
int vip_texture_run(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, void* stream) {
    return texture_run(h, d_src, d_dst, stream, nullptr);
}

int vip_texture_run_timed(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, void* stream, void* const* events) {
    if (!events) return VIP_ERR_INVALID_ARGUMENT;
    return texture_run(h, d_src, d_dst, stream, events);
}

int vip_texture_halo_rows(int ksize) {
    if (ksize < 1) return VIP_ERR_INVALID_ARGUMENT;
    // JBF radius (2k-1)/2 = k-1 on the guide, whose stages reach gradient 1 + blur/mRTV
    // k/2 + argmin k/2 rows further into the image
    return (ksize - 1) + 2 * (ksize / 2) + 1;
}

// One iteration on a row slab (multi-GPU texture filter): guide rows
// [out_row0 - (k-1), out_row0 + out_rows + (k-1)) clipped to the valid rows, then
// the JBF of the output rows. Stage reads clamp into [row_lo, row_hi), so at a
// frame edge the result is the reference's; elsewhere the caller supplies
// vip_texture_halo_rows(k) valid rows around the output rows.
int vip_texture_iterate_rows(vip_texture_t h, const uint8_t* d_src, uint8_t* d_dst, size_t dst_pitch, int out_row0,
                             int out_rows, int row_lo, int row_hi, void* stream) {
    if (!h || !d_src || !d_dst || out_rows < 0 || row_lo < 0 || row_hi > h->height || row_lo >= row_hi ||
        out_row0 < row_lo || out_row0 + out_rows > row_hi)
        return VIP_ERR_INVALID_ARGUMENT;
    if (out_rows == 0) return 0;
    const size_t pitch = (size_t)h->width * 3;
    const uint8_t* dst_end = d_dst + (size_t)(out_rows - 1) * dst_pitch + pitch;
    const uint8_t* src_end = d_src + (size_t)h->height * pitch;
    if (d_dst < src_end && dst_end > d_src) return VIP_ERR_ALIASING;
    const int rj = h->ksize - 1;
    const int g0 = out_row0 - rj > row_lo ? out_row0 - rj : row_lo;
    const int g1 = out_row0 + out_rows + rj < row_hi ? out_row0 + out_rows + rj : row_hi;
    const hipStream_t s = (hipStream_t)stream;
    int rc = launch_texture_guide_fused_rows(d_src, h->d_guide, h->width, row_lo, row_hi, g0, g1, h->ksize,
                                             h->numerics == VIP_NUMERICS_CPP, s);
    if (!rc) rc = vip_bilateral_run_rows(h->jbf, d_src, pitch, h->d_guide, pitch, d_dst, dst_pitch, out_rows,
                                         out_row0, row_lo, row_hi, stream);
    return rc;
}

}  // extern "C"
