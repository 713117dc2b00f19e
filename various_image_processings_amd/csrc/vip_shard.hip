// Row-sharded frames with an RCCL halo exchange (include/vip_shard.h), host code.
//
// No reference counterpart (the reference is single-GPU): the
// north_star's row-tiled configuration as a native C entry point. One shard = one rank's
// slab of the frame plus the filter handle (vip.h row-band form) that filters it, a
// communication stream and two events. A run overlaps the halo exchange (RCCL
// ncclSend/ncclRecv with the two row neighbours, in one group; or device copies for the
// LOCAL transport) with the interior rows, whose windows stay inside the own rows, and
// filters the two r-row edge bands once the halos are in.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "vip_shard.h"

namespace {

thread_local std::string g_last_error;

int comm_fail(ncclResult_t r, const char* what) {
    g_last_error = std::string(what) + ": " + ncclGetErrorString(r);
    return VIP_ERR_COMM;
}

#define VIP_HIP_TRY(expr)                                 \
    do {                                                  \
        const hipError_t e_ = (expr);                     \
        if (e_ != hipSuccess) return (int)e_;             \
    } while (0)

// Polls a non-blocking communicator until its pending operation (initialisation or
// the enqueue of a group) completes, fails, or the deadline passes.
int wait_comm(ncclComm_t c, int timeout_ms, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(c, &st);
        if (r != ncclSuccess) return comm_fail(r, what);
        if (st == ncclSuccess) return 0;
        if (st != ncclInProgress) return comm_fail(st, what);
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
        if (ms.count() > timeout_ms) {
            g_last_error = std::string(what) + ": not complete after " + std::to_string(timeout_ms) + " ms";
            return VIP_ERR_COMM_TIMEOUT;
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

int default_timeout(int t) { return t > 0 ? t : 180000; }

// Communicator initialisation, bounded: RCCL's init blocks in its bootstrap until every
// rank has joined (measured: ncclCommInitRankConfig with blocking = 0 does not return
// either while a rank is missing), and ncclCommAbort / ncclCommDestroy on such a
// communicator join the blocked thread. So the init runs on a helper thread that owns its
// result; the caller waits up to timeout_ms and otherwise returns VIP_ERR_COMM_TIMEOUT,
// leaving the helper detached (the communicator is never handed out, the process keeps the
// stuck thread until it exits).
struct InitJob {
    std::vector<ncclComm_t> comms;
    std::atomic<int> status{0};
    std::atomic<bool> done{false};
    std::string error;
};

template <class F>
int bounded_init(const std::shared_ptr<InitJob>& job, F&& body, int timeout_ms, std::vector<ncclComm_t>* out) {
    std::thread([job, body]() mutable {
        job->status = body(*job);
        job->done = true;
    }).detach();
    const auto t0 = std::chrono::steady_clock::now();
    while (!job->done.load()) {
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
        if (ms.count() > timeout_ms) {
            g_last_error = "communicator initialisation: not complete after " + std::to_string(timeout_ms) +
                           " ms (a rank did not join)";
            return VIP_ERR_COMM_TIMEOUT;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (job->status != 0) {
        g_last_error = job->error;
        return job->status;
    }
    *out = job->comms;
    return 0;
}

}  // namespace

struct vip_shard_s {
    int kind, width, frame_height, ksize, numerics;
    int nranks, rank, transport, device, timeout_ms;
    int row_begin, own, r;
    vip_bilateral_t bil = nullptr;
    vip_adaptive_t ada = nullptr;
    vip_texture_t tex = nullptr;           // VIP_FILTER_TEXTURE: nitr iterations, ghost zone
    int nitr = 0, step = 0;                // iterations; rows one iteration reaches (halo = nitr * step)
    uint8_t* scratch[2] = {nullptr, nullptr};  // texture: ping-pong slabs between iterations
    hipStream_t comm = nullptr;  // halo exchange stream
    hipEvent_t ev_in = nullptr;  // own rows written (on the caller's stream)
    hipEvent_t ev_x = nullptr;   // halos received (on comm)
    ncclComm_t nccl = nullptr;   // VIP_SHARD_RCCL
    int peer_up = -1, peer_down = -1;  // communicator ranks of the row neighbours (loopback: 0, itself)
    int split = 0;               // 1: interior rows under the exchange, then the edge bands
    int frames_launch = 0;       // vip_shard_set_frames_launch: a batch's frames in one launch
    int free_cus = 0;            // ... leaving this many CUs to concurrent work
    // graph mode (vip_shard_set_graph): one captured hipGraph per (slab, out, pitch, stream)
    struct Graph {
        uint8_t* slab;
        uint8_t* out;
        size_t pitch;
        hipStream_t stream;
        hipGraphExec_t exec;
        hipEvent_t done;  // shard-owned, recorded after every replay: freed without the caller's stream
    };
    int graph = 0;
    bool warm = false;           // one direct exchange done: RCCL connects peers lazily, a capture cannot
    std::vector<Graph> graphs;
    bool above() const { return rank > 0 && r > 0; }
    bool below() const { return rank < nranks - 1 && r > 0; }
    int slab_rows() const { return own + 2 * r; }
    size_t pitch() const { return (size_t)width * 3; }
};

extern "C" int vip_shard_destroy(vip_shard_t h);

namespace {

// What every rank's shard filters (the create functions' arguments).
struct FilterSpec {
    int kind, ksize;
    float sigma_space, sigma_color;  // bilateral, adaptive
    int nitr;                        // texture
    int numerics;
};

// Filter handle, stream and events of a shard on the current device (geometry set).
int init_shard(vip_shard_s* h, const FilterSpec& f) {
    VIP_HIP_TRY(hipGetDevice(&h->device));
    int rc = 0;
    if (h->kind == VIP_FILTER_TEXTURE) {
        rc = vip_texture_create(&h->tex, h->width, h->slab_rows(), h->ksize, h->nitr, h->numerics);
        for (int i = 0; i < 2 && !rc && h->nitr > 1; ++i)
            rc = (int)hipMalloc(reinterpret_cast<void**>(&h->scratch[i]), (size_t)h->slab_rows() * h->pitch());
    } else if (h->kind == VIP_FILTER_ADAPTIVE) {
        rc = vip_adaptive_create(&h->ada, h->width, h->slab_rows(), h->ksize, f.sigma_space, f.sigma_color,
                                 h->numerics);
    } else {
        rc = vip_bilateral_create(&h->bil, h->width, h->slab_rows(), h->ksize, f.sigma_space, f.sigma_color,
                                  h->numerics);
    }
    if (rc) return rc;
    VIP_HIP_TRY(hipStreamCreateWithFlags(&h->comm, hipStreamNonBlocking));
    VIP_HIP_TRY(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    VIP_HIP_TRY(hipEventCreateWithFlags(&h->ev_x, hipEventDisableTiming));
    return 0;
}

// Geometry shared by every rank (sharded.py SlabGeometry); VIP_ERR_INVALID_ARGUMENT when
// the thinnest shard cannot cover a halo (checked identically on every rank, before any
// communication, so no rank is left waiting in an exchange the others never join).
// The texture filter's halo is nitr iterations deep (sharded.py ShardedTexture): one
// exchange per frame, then iteration t filters the own rows plus (nitr - 1 - t) * step
// rows on each side, so the last iteration's own rows are exact.
int new_shard(vip_shard_s** out, const FilterSpec& f, int width, int frame_height, int nranks, int rank,
              int transport, int timeout_ms) {
    if (!out || width <= 0 || frame_height <= 0 || nranks <= 0 || rank < 0 || rank >= nranks)
        return VIP_ERR_INVALID_ARGUMENT;
    int r = 0, step = 0;
    if (f.kind == VIP_FILTER_TEXTURE) {
        if (f.ksize < 1) return VIP_ERR_UNSUPPORTED_KSIZE;  // the texture handle checks the upper limit
        if (f.nitr < 0) return VIP_ERR_INVALID_ARGUMENT;
        step = vip_texture_halo_rows(f.ksize);
        r = f.nitr * step;
    } else if (f.kind == VIP_FILTER_BILATERAL || f.kind == VIP_FILTER_ADAPTIVE) {
        if (f.ksize < 1 || !(f.ksize & 1)) return VIP_ERR_UNSUPPORTED_KSIZE;
        r = f.ksize / 2;
    } else {
        return VIP_ERR_INVALID_ARGUMENT;
    }
    if (nranks > 1 && frame_height / nranks < r) return VIP_ERR_INVALID_ARGUMENT;
    auto* h = new (std::nothrow) vip_shard_s();
    if (!h) return (int)hipErrorOutOfMemory;
    h->kind = f.kind;
    h->width = width;
    h->frame_height = frame_height;
    h->ksize = f.ksize;
    h->numerics = f.numerics;
    h->nitr = f.nitr;
    h->step = step;
    h->nranks = nranks;
    h->rank = rank;
    h->transport = transport;
    h->timeout_ms = default_timeout(timeout_ms);
    vip_shard_rows(frame_height, nranks, rank, &h->row_begin, &h->own);
    h->r = r;
    h->peer_up = rank - 1;
    h->peer_down = rank + 1;
    *out = h;
    return 0;
}

// Rows the shard's filter may read: the halos where a neighbour supplies them, else the
// own rows (the reference's replicate border at the frame's top and bottom).
void clamp_range(const vip_shard_s* h, int* lo, int* hi) {
    *lo = h->above() ? 0 : h->r;
    *hi = h->below() ? h->slab_rows() : h->r + h->own;
}

// Texture: all own rows, nitr iterations with a shrinking ghost zone (the halos must be in).
int texture_rows(const vip_shard_s* h, uint8_t* slab, uint8_t* out, size_t out_pitch, hipStream_t s) {
    int lo, hi;
    clamp_range(h, &lo, &hi);
    if (h->nitr == 0)  // the reference's execute with nitr = 0 returns the source
        return (int)hipMemcpy2DAsync(out, out_pitch, slab + (size_t)h->r * h->pitch(), h->pitch(), h->pitch(),
                                     h->own, hipMemcpyDeviceToDevice, s);
    const uint8_t* a = slab;
    for (int t = 0; t < h->nitr; ++t) {
        if (t == h->nitr - 1)
            return vip_texture_iterate_rows(h->tex, a, out, out_pitch, h->r, h->own, lo, hi, s);
        const int m = (h->nitr - 1 - t) * h->step;
        const int r0 = h->r - m > lo ? h->r - m : lo, r1 = h->r + h->own + m < hi ? h->r + h->own + m : hi;
        uint8_t* b = h->scratch[t % 2];
        if (const int rc = vip_texture_iterate_rows(h->tex, a, b + (size_t)r0 * h->pitch(), h->pitch(), r0, r1 - r0,
                                                    lo, hi, s))
            return rc;
        a = b;
    }
    return 0;
}

// Own rows [row0, row0 + n) of the slab -> the same rows of out.
int filter_rows(const vip_shard_s* h, uint8_t* slab, uint8_t* out, size_t out_pitch, int row0, int n,
                hipStream_t s) {
    if (n <= 0) return 0;
    if (h->kind == VIP_FILTER_TEXTURE) return texture_rows(h, slab, out, out_pitch, s);  // row0 = 0, n = own
    int lo, hi;
    clamp_range(h, &lo, &hi);
    uint8_t* o = out + (size_t)row0 * out_pitch;
    if (h->kind == VIP_FILTER_ADAPTIVE)
        return vip_adaptive_run_rows(h->ada, slab, h->pitch(), o, out_pitch, n, h->r + row0, lo, hi, s);
    return vip_bilateral_run_rows(h->bil, slab, h->pitch(), nullptr, 0, o, out_pitch, n, h->r + row0, lo, hi, s);
}

// Every own row of n frames: one launch per frame, or (vip_shard_set_frames_launch, plain
// and adaptive filters) one launch per 6 frames (vip_*_run_rows_batch: the launch prologue
// and tail once per launch).
int filter_frames(const vip_shard_s* h, int n, uint8_t* const* slabs, uint8_t* const* outs, size_t out_pitch,
                  hipStream_t s) {
    if (h->kind == VIP_FILTER_TEXTURE || n == 1 || !h->frames_launch) {
        for (int f = 0; f < n; ++f)
            if (const int rc = filter_rows(h, slabs[f], outs[f], out_pitch, 0, h->own, s)) return rc;
        return 0;
    }
    int lo, hi;
    clamp_range(h, &lo, &hi);
    const uint8_t* const* srcs = const_cast<const uint8_t* const*>(slabs);
    if (h->kind == VIP_FILTER_ADAPTIVE)
        return vip_adaptive_run_rows_batch(h->ada, n, srcs, h->pitch(), outs, out_pitch, h->own, h->r, lo, hi,
                                           h->free_cus, s);
    return vip_bilateral_run_rows_batch(h->bil, n, srcs, h->pitch(), outs, out_pitch, h->own, h->r, lo, hi,
                                        h->free_cus, s);
}

// Interior rows [r, own - r) read only own rows; the edge bands need the halos.
int interior(const vip_shard_s* h, uint8_t* slab, uint8_t* out, size_t out_pitch, hipStream_t s) {
    return filter_rows(h, slab, out, out_pitch, h->r, h->own - 2 * h->r, s);
}
int edges(const vip_shard_s* h, uint8_t* slab, uint8_t* out, size_t out_pitch, hipStream_t s) {
    const int top = h->r < h->own ? h->r : h->own;
    const int b0 = h->own - h->r > top ? h->own - h->r : top;
    int rc = filter_rows(h, slab, out, out_pitch, 0, top, s);
    if (!rc) rc = filter_rows(h, slab, out, out_pitch, b0, h->own - b0, s);
    return rc;
}

// This shard's sends and receives (inside the caller's ncclGroupStart/End).
int enqueue_p2p(const vip_shard_s* h, uint8_t* slab) {
    const size_t bytes = (size_t)h->r * h->pitch();
    ncclResult_t e = ncclSuccess;
    if (h->above()) {
        if ((e = ncclSend(slab + (size_t)h->r * h->pitch(), bytes, ncclUint8, h->peer_up, h->nccl, h->comm)))
            return comm_fail(e, "ncclSend (up)");
        if ((e = ncclRecv(slab, bytes, ncclUint8, h->peer_up, h->nccl, h->comm))) return comm_fail(e, "ncclRecv (up)");
    }
    if (h->below()) {
        if ((e = ncclSend(slab + (size_t)h->own * h->pitch(), bytes, ncclUint8, h->peer_down, h->nccl, h->comm)))
            return comm_fail(e, "ncclSend (down)");
        if ((e = ncclRecv(slab + (size_t)(h->r + h->own) * h->pitch(), bytes, ncclUint8, h->peer_down, h->nccl,
                          h->comm)))
            return comm_fail(e, "ncclRecv (down)");
    }
    return 0;
}

int group_end(vip_shard_s* const* hs, int n) {
    const ncclResult_t e = ncclGroupEnd();
    if (e == ncclSuccess) return 0;  // enqueued (blocking communicators)
    if (e != ncclInProgress) return comm_fail(e, "ncclGroupEnd");
    for (int i = 0; i < n; ++i)
        if (const int rc = wait_comm(hs[i]->nccl, hs[i]->timeout_ms, "halo exchange")) return rc;
    return 0;
}

// Record `ev` on `s` when the caller asked for timing events.
int mark(void* const* events, int k, hipStream_t s) {
    return events ? (int)hipEventRecord((hipEvent_t)events[k], s) : 0;
}

struct DeviceGuard {  // restores the caller's current device
    int dev = -1;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// A replay may still be in flight: wait on the shard's own event for it, never on the
// caller's stream (which vip_shard.h does not require to outlive the shard).
void free_graph(vip_shard_s::Graph& g) {
    if (g.done) {
        (void)hipEventSynchronize(g.done);
        (void)hipEventDestroy(g.done);
    }
    (void)hipGraphExecDestroy(g.exec);
}

void free_graphs(vip_shard_s* h) {
    for (auto& g : h->graphs) free_graph(g);
    h->graphs.clear();
}

// RCCL builds whose capture of a ncclSend/ncclRecv group was verified: 2.27.7 (the image's
// /opt/rocm/lib/librccl.so; tests/cpp/shard_graph_test). torch's bundled 2.26.6 crashes
// on the first capture in every capture mode (profiles/r04_graph_capture.txt), and inside a
// torch process this library's RCCL symbols bind to that copy.
constexpr int kGraphMinRcclVersion = 22707;

int rccl_version() {
    int v = 0;
    return ncclGetVersion(&v) == ncclSuccess ? v : 0;
}

constexpr size_t kMaxGraphs = 64;  // captured (slab, out, stream) combinations kept per shard

// Capture mode of graph mode: thread-local by default; VIP_SHARD_CAPTURE_MODE=1 global,
// 2 relaxed (a measurement knob for RCCL builds that treat the modes differently).
hipStreamCaptureMode capture_mode() {
    static const hipStreamCaptureMode m = [] {
        const char* e = std::getenv("VIP_SHARD_CAPTURE_MODE");
        const int v = e ? std::atoi(e) : 0;
        return v == 1 ? hipStreamCaptureModeGlobal : v == 2 ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeThreadLocal;
    }();
    return m;
}

}  // namespace

extern "C" {

int vip_shard_rows(int frame_height, int nranks, int rank, int* row_begin, int* own_rows) {
    if (frame_height < 0 || nranks <= 0 || rank < 0 || rank >= nranks || !row_begin || !own_rows)
        return VIP_ERR_INVALID_ARGUMENT;
    const int base = frame_height / nranks, rem = frame_height % nranks;
    *row_begin = rank * base + (rank < rem ? rank : rem);
    *own_rows = base + (rank < rem ? 1 : 0);
    return 0;
}

int vip_shard_unique_id(void* id) {
    if (!id) return VIP_ERR_INVALID_ARGUMENT;
    static_assert(sizeof(ncclUniqueId) == VIP_SHARD_ID_BYTES, "id size");
    ncclUniqueId u;
    if (const ncclResult_t e = ncclGetUniqueId(&u)) return comm_fail(e, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

const char* vip_shard_last_error(void) { return g_last_error.c_str(); }

// This shard's communicator: rank comm_rank of comm_n over the id (bounded, see InitJob).
static int init_comm(vip_shard_s* h, const ncclUniqueId& u, int comm_n, int comm_rank) {
    const int dev = h->device;
    auto job = std::make_shared<InitJob>();
    std::vector<ncclComm_t> comms;
    const int rc = bounded_init(
        job,
        [u, comm_n, comm_rank, dev](InitJob& j) {
            j.comms.assign(1, nullptr);
            if (hipSetDevice(dev) != hipSuccess) return (int)hipErrorInvalidDevice;
            const ncclResult_t e = ncclCommInitRank(&j.comms[0], comm_n, u, comm_rank);
            if (e != ncclSuccess) {
                j.error = std::string("ncclCommInitRank: ") + ncclGetErrorString(e);
                return (int)VIP_ERR_COMM;
            }
            return 0;
        },
        h->timeout_ms, &comms);
    if (!rc) h->nccl = comms[0];
    return rc;
}

static int create_rank(vip_shard_t* out, const FilterSpec& f, int width, int frame_height, int nranks, int rank,
                       const void* id, int timeout_ms) {
    if (!out || !id) return VIP_ERR_INVALID_ARGUMENT;
    vip_shard_s* h = nullptr;
    int rc = new_shard(&h, f, width, frame_height, nranks, rank, VIP_SHARD_RCCL, timeout_ms);
    if (rc) return rc;
    rc = init_shard(h, f);
    if (!rc) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        rc = init_comm(h, u, nranks, rank);
    }
    if (rc) {
        vip_shard_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

static int create_group(vip_shard_t* out, int n, int transport, const int* devices, const FilterSpec& f, int width,
                        int frame_height, int timeout_ms) {
    if (!out || n <= 0 || (transport != VIP_SHARD_RCCL && transport != VIP_SHARD_LOCAL)) return VIP_ERR_INVALID_ARGUMENT;
    if (transport == VIP_SHARD_RCCL && !devices) return VIP_ERR_INVALID_ARGUMENT;
    DeviceGuard guard;
    for (int i = 0; i < n; ++i) out[i] = nullptr;
    int rc = 0;
    for (int i = 0; i < n && !rc; ++i) {
        rc = new_shard(&out[i], f, width, frame_height, n, i, transport, timeout_ms);
        if (!rc && transport == VIP_SHARD_RCCL) rc = (int)hipSetDevice(devices[i]);
        if (!rc) rc = init_shard(out[i], f);
    }
    if (!rc && transport == VIP_SHARD_RCCL) {
        // one communicator per device, initialised in one group (ncclCommInitAll's pattern)
        ncclUniqueId u;
        if (const ncclResult_t e = ncclGetUniqueId(&u)) rc = comm_fail(e, "ncclGetUniqueId");
        std::vector<int> devs(devices, devices + n);
        auto job = std::make_shared<InitJob>();
        std::vector<ncclComm_t> comms;
        if (!rc)
            rc = bounded_init(
                job,
                [u, n, devs](InitJob& j) {
                    j.comms.assign(n, nullptr);
                    ncclResult_t e = ncclGroupStart();
                    for (int i = 0; i < n && e == ncclSuccess; ++i) {
                        if (hipSetDevice(devs[i]) != hipSuccess) return (int)hipErrorInvalidDevice;
                        e = ncclCommInitRank(&j.comms[i], n, u, i);
                    }
                    const ncclResult_t e2 = ncclGroupEnd();
                    if (e == ncclSuccess) e = e2;
                    if (e != ncclSuccess) {
                        j.error = std::string("ncclCommInitRank (group): ") + ncclGetErrorString(e);
                        return (int)VIP_ERR_COMM;
                    }
                    return 0;
                },
                out[0]->timeout_ms, &comms);
        for (int i = 0; i < n && !rc; ++i) out[i]->nccl = comms[i];
    }
    if (rc) {
        for (int i = 0; i < n; ++i) {
            vip_shard_destroy(out[i]);
            out[i] = nullptr;
        }
    }
    return rc;
}

int vip_shard_create(vip_shard_t* out, int kind, int width, int frame_height, int ksize, float sigma_space,
                     float sigma_color, int numerics, int nranks, int rank, const void* id, int timeout_ms) {
    if (kind != VIP_FILTER_BILATERAL && kind != VIP_FILTER_ADAPTIVE) return VIP_ERR_INVALID_ARGUMENT;
    return create_rank(out, FilterSpec{kind, ksize, sigma_space, sigma_color, 0, numerics}, width, frame_height,
                       nranks, rank, id, timeout_ms);
}

int vip_shard_create_texture(vip_shard_t* out, int width, int frame_height, int ksize, int nitr, int numerics,
                             int nranks, int rank, const void* id, int timeout_ms) {
    return create_rank(out, FilterSpec{VIP_FILTER_TEXTURE, ksize, 0.f, 0.f, nitr, numerics}, width, frame_height,
                       nranks, rank, id, timeout_ms);
}

int vip_shard_create_group(vip_shard_t* out, int n, int transport, const int* devices, int kind, int width,
                           int frame_height, int ksize, float sigma_space, float sigma_color, int numerics,
                           int timeout_ms) {
    if (kind != VIP_FILTER_BILATERAL && kind != VIP_FILTER_ADAPTIVE) return VIP_ERR_INVALID_ARGUMENT;
    return create_group(out, n, transport, devices, FilterSpec{kind, ksize, sigma_space, sigma_color, 0, numerics},
                        width, frame_height, timeout_ms);
}

int vip_shard_create_group_texture(vip_shard_t* out, int n, int transport, const int* devices, int width,
                                   int frame_height, int ksize, int nitr, int numerics, int timeout_ms) {
    return create_group(out, n, transport, devices, FilterSpec{VIP_FILTER_TEXTURE, ksize, 0.f, 0.f, nitr, numerics},
                        width, frame_height, timeout_ms);
}

int vip_shard_create_loopback(vip_shard_t* out, int kind, int width, int frame_height, int ksize, float sigma_space,
                              float sigma_color, int nitr, int numerics, int nranks, int rank, int timeout_ms) {
    if (!out) return VIP_ERR_INVALID_ARGUMENT;
    if (kind != VIP_FILTER_BILATERAL && kind != VIP_FILTER_ADAPTIVE && kind != VIP_FILTER_TEXTURE)
        return VIP_ERR_INVALID_ARGUMENT;
    const FilterSpec f{kind, ksize, sigma_space, sigma_color, kind == VIP_FILTER_TEXTURE ? nitr : 0, numerics};
    vip_shard_s* h = nullptr;
    int rc = new_shard(&h, f, width, frame_height, nranks, rank, VIP_SHARD_RCCL, timeout_ms);
    if (rc) return rc;
    rc = init_shard(h, f);
    if (!rc) {
        ncclUniqueId u;
        if (const ncclResult_t e = ncclGetUniqueId(&u)) rc = comm_fail(e, "ncclGetUniqueId");
        if (!rc) rc = init_comm(h, u, 1, 0);
    }
    if (rc) {
        vip_shard_destroy(h);
        return rc;
    }
    h->peer_up = h->peer_down = 0;  // both neighbours are this rank of the one-rank communicator
    *out = h;
    return 0;
}

int vip_shard_set_split(vip_shard_t h, int split) {
    if (!h || (split != 0 && split != 1)) return VIP_ERR_INVALID_ARGUMENT;
    if (split && h->kind == VIP_FILTER_TEXTURE) return VIP_ERR_INVALID_ARGUMENT;  // every iteration needs the halos
    if (split != h->split) {
        DeviceGuard guard;
        (void)hipSetDevice(h->device);
        free_graphs(h);  // the captured sequences follow the old split
    }
    h->split = split;
    return 0;
}

int vip_shard_set_frames_launch(vip_shard_t h, int on, int free_cus) {
    if (!h || (on != 0 && on != 1) || free_cus < 0) return VIP_ERR_INVALID_ARGUMENT;
    h->frames_launch = h->kind == VIP_FILTER_TEXTURE ? 0 : on;
    h->free_cus = free_cus;
    return 0;
}

int vip_shard_set_graph(vip_shard_t h, int on) {
    if (!h || (on != 0 && on != 1)) return VIP_ERR_INVALID_ARGUMENT;
    if (h->transport != VIP_SHARD_RCCL) return VIP_ERR_INVALID_ARGUMENT;
    if (on && rccl_version() < kGraphMinRcclVersion) {
        g_last_error = "graph mode needs RCCL >= 2.27.7 (the RCCL bound in this process is " +
                       std::to_string(rccl_version()) + "; older builds crash capturing a send/recv group)";
        return VIP_ERR_UNSUPPORTED;
    }
    if (!on) {
        DeviceGuard guard;
        (void)hipSetDevice(h->device);
        free_graphs(h);
    }
    h->graph = on;
    return 0;
}

int vip_shard_rccl_version(int* version) {
    if (!version) return VIP_ERR_INVALID_ARGUMENT;
    *version = rccl_version();
    return 0;
}

int vip_shard_comm_info(vip_shard_t h, int* count, int* user_rank, int* device) {
    if (!h || !count || !user_rank || !device || h->transport != VIP_SHARD_RCCL || !h->nccl)
        return VIP_ERR_INVALID_ARGUMENT;
    ncclResult_t e = ncclCommCount(h->nccl, count);
    if (e != ncclSuccess) return comm_fail(e, "ncclCommCount");
    if ((e = ncclCommUserRank(h->nccl, user_rank)) != ncclSuccess) return comm_fail(e, "ncclCommUserRank");
    if ((e = ncclCommCuDevice(h->nccl, device)) != ncclSuccess) return comm_fail(e, "ncclCommCuDevice");
    return 0;
}

int vip_shard_pci_bus_id(vip_shard_t h, char* bus_id, int len) {
    if (!h || !bus_id || len < 13) return VIP_ERR_INVALID_ARGUMENT;  // "0000:00:00.0" + NUL
    return (int)hipDeviceGetPCIBusId(bus_id, len, h->device);
}

int vip_shard_graph_count(vip_shard_t h, int* count) {
    if (!h || !count) return VIP_ERR_INVALID_ARGUMENT;
    *count = (int)h->graphs.size();
    return 0;
}

int vip_shard_geometry(vip_shard_t h, int* row_begin, int* own_rows, int* halo_rows) {
    if (!h || !row_begin || !own_rows || !halo_rows) return VIP_ERR_INVALID_ARGUMENT;
    *row_begin = h->row_begin;
    *own_rows = h->own;
    *halo_rows = h->r;
    return 0;
}

static int check_run(vip_shard_t h, uint8_t* slab, uint8_t* out, size_t out_pitch) {
    if (!h || !slab || !out || out_pitch < h->pitch() || h->transport != VIP_SHARD_RCCL || !h->nccl)
        return VIP_ERR_INVALID_ARGUMENT;
    return 0;
}

// One frame's work enqueued on `s` (and the communication stream), device already set.
static int enqueue_run(vip_shard_t h, uint8_t* slab, uint8_t* out, size_t out_pitch, hipStream_t s,
                       void* const* events) {
    int rc = mark(events, 0, s);
    if (!rc && !h->above() && !h->below()) {  // no neighbours: one launch over the own rows
        rc = mark(events, 1, s);
        if (!rc) rc = filter_rows(h, slab, out, out_pitch, 0, h->own, s);
        if (!rc) rc = mark(events, 2, s);
        if (!rc) rc = mark(events, 3, s);
        return rc;
    }
    // exchange first on the communication stream (its kernel is dispatched ahead of the
    // interior launch), then the interior on the caller's stream, then the edges after
    // the halos
    if (!rc) rc = (int)hipEventRecord(h->ev_in, s);
    if (!rc) rc = (int)hipStreamWaitEvent(h->comm, h->ev_in, 0);
    if (!rc) {
        if (const ncclResult_t e = ncclGroupStart()) rc = comm_fail(e, "ncclGroupStart");
        if (!rc) rc = enqueue_p2p(h, slab);
        const int rc2 = group_end(&h, 1);
        if (!rc) rc = rc2;
    }
    if (!rc) rc = mark(events, 1, h->comm);
    if (!rc) rc = (int)hipEventRecord(h->ev_x, h->comm);
    if (!h->split) {  // one launch over the own rows once the halos are in
        if (!rc) rc = (int)hipStreamWaitEvent(s, h->ev_x, 0);
        if (!rc) rc = mark(events, 2, s);  // halos in, on the filter stream
        if (!rc) rc = filter_rows(h, slab, out, out_pitch, 0, h->own, s);
        if (!rc) rc = mark(events, 3, s);
        return rc;
    }
    if (!rc) rc = interior(h, slab, out, out_pitch, s);
    if (!rc) rc = mark(events, 2, s);
    if (!rc) rc = (int)hipStreamWaitEvent(s, h->ev_x, 0);
    if (!rc) rc = edges(h, slab, out, out_pitch, s);
    if (!rc) rc = mark(events, 3, s);
    return rc;
}

int vip_shard_run_batch(vip_shard_t h, int n, uint8_t* const* d_slabs, uint8_t* const* d_outs, size_t out_pitch,
                        void* stream) {
    if (!h || n <= 0 || !d_slabs || !d_outs || out_pitch < h->pitch() || h->transport != VIP_SHARD_RCCL || !h->nccl)
        return VIP_ERR_INVALID_ARGUMENT;
    for (int f = 0; f < n; ++f)
        if (!d_slabs[f] || !d_outs[f]) return VIP_ERR_INVALID_ARGUMENT;
    DeviceGuard guard;
    const hipStream_t s = (hipStream_t)stream;
    VIP_HIP_TRY(hipSetDevice(h->device));
    if (!h->above() && !h->below())  // no neighbours: the launches only
        return filter_frames(h, n, d_slabs, d_outs, out_pitch, s);
    // every frame's own rows written -> one group with all the halos on the communication stream
    VIP_HIP_TRY(hipEventRecord(h->ev_in, s));
    VIP_HIP_TRY(hipStreamWaitEvent(h->comm, h->ev_in, 0));
    int rc = 0;
    if (const ncclResult_t e = ncclGroupStart()) return comm_fail(e, "ncclGroupStart");
    for (int f = 0; f < n && !rc; ++f) rc = enqueue_p2p(h, d_slabs[f]);
    const int rc2 = group_end(&h, 1);
    if (rc || rc2) return rc ? rc : rc2;
    h->warm = true;
    VIP_HIP_TRY(hipEventRecord(h->ev_x, h->comm));
    if (!h->split) {
        VIP_HIP_TRY(hipStreamWaitEvent(s, h->ev_x, 0));
        return filter_frames(h, n, d_slabs, d_outs, out_pitch, s);
    }
    for (int f = 0; f < n; ++f)  // interiors under the exchange, then every frame's edge bands
        if ((rc = interior(h, d_slabs[f], d_outs[f], out_pitch, s))) return rc;
    VIP_HIP_TRY(hipStreamWaitEvent(s, h->ev_x, 0));
    for (int f = 0; f < n; ++f)
        if ((rc = edges(h, d_slabs[f], d_outs[f], out_pitch, s))) return rc;
    return 0;
}

// Graph mode: the frame's whole sequence (own rows written -> exchange on the
// communication stream -> filter launches) captured once per (slab, out, pitch, stream)
// into a hipGraph and replayed with one hipGraphLaunch: a few us of host time per frame
// instead of an RCCL group's 16-30 us (profiles/r03_rccl_enqueue.txt). Each shard has its
// own communicator, so the graphs of shards on different streams never run one
// communicator's kernels concurrently.
static int run_graph(vip_shard_t h, uint8_t* slab, uint8_t* out, size_t out_pitch, hipStream_t s) {
    for (const auto& g : h->graphs)
        if (g.slab == slab && g.out == out && g.pitch == out_pitch && g.stream == s) {
            VIP_HIP_TRY(hipGraphLaunch(g.exec, s));
            return (int)hipEventRecord(g.done, s);
        }
    if (h->graphs.size() >= kMaxGraphs) {  // the oldest graph may still be in flight: free_graph waits
        free_graph(h->graphs.front());
        h->graphs.erase(h->graphs.begin());
    }
    // nothing is enqueued yet: if the stream cannot capture, run this frame directly
    if (hipStreamBeginCapture(s, capture_mode()) != hipSuccess) {
        (void)hipGetLastError();
        return enqueue_run(h, slab, out, out_pitch, s, nullptr);
    }
    const int rc = enqueue_run(h, slab, out, out_pitch, s, nullptr);
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &graph);
    hipGraphExec_t exec = nullptr;
    hipError_t ei = hipErrorUnknown;
    // VIP_SHARD_TEST_FAIL_CAPTURE=1: treat every capture as failed (the recovery path's test,
    // tests/cpp/shard_graph_test --fail-capture)
    static const bool fail_capture = [] {
        const char* v = std::getenv("VIP_SHARD_TEST_FAIL_CAPTURE");
        return v && v[0] == '1';
    }();
    if (!rc && e == hipSuccess && !fail_capture) ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    hipEvent_t done = nullptr;
    if (ei == hipSuccess) ei = hipEventCreateWithFlags(&done, hipEventDisableTiming);
    if (ei != hipSuccess) {
        // The capture failed, so this rank's sends and receives for the frame never ran,
        // while the peers ran (or replay) their half of the exchange: run the frame directly
        // now so every rank still performs it, and leave graph mode for this shard (a
        // second capture would fail the same way).
        if (exec) (void)hipGraphExecDestroy(exec);
        (void)hipGetLastError();
        fprintf(stderr, "vip_shard: graph capture failed (run %d, end capture %d, instantiate %d): graph mode off, "
                        "running the frame directly\n", rc, (int)e, (int)ei);
        h->graph = 0;
        free_graphs(h);
        return enqueue_run(h, slab, out, out_pitch, s, nullptr);
    }
    h->graphs.push_back({slab, out, out_pitch, s, exec, done});
    VIP_HIP_TRY(hipGraphLaunch(exec, s));
    return (int)hipEventRecord(done, s);
}

int vip_shard_run(vip_shard_t h, uint8_t* d_slab, uint8_t* d_out, size_t out_pitch, void* stream) {
    if (const int rc = check_run(h, d_slab, d_out, out_pitch)) return rc;
    DeviceGuard guard;
    VIP_HIP_TRY(hipSetDevice(h->device));
    const hipStream_t s = (hipStream_t)stream;
    // the null stream cannot be captured; the first exchange connects the peers directly
    if (h->graph && h->warm && s != nullptr) return run_graph(h, d_slab, d_out, out_pitch, s);
    const int rc = enqueue_run(h, d_slab, d_out, out_pitch, s, nullptr);
    if (!rc) h->warm = true;
    return rc;
}

int vip_shard_run_timed(vip_shard_t h, uint8_t* d_slab, uint8_t* d_out, size_t out_pitch, void* stream,
                        void* const* events) {
    if (!events) return VIP_ERR_INVALID_ARGUMENT;
    if (const int rc = check_run(h, d_slab, d_out, out_pitch)) return rc;
    DeviceGuard guard;
    VIP_HIP_TRY(hipSetDevice(h->device));
    const int rc = enqueue_run(h, d_slab, d_out, out_pitch, (hipStream_t)stream, events);
    if (!rc) h->warm = true;
    return rc;
}

int vip_shard_run_group(vip_shard_t* hs, int n, uint8_t* const* slabs, uint8_t* const* outs, size_t out_pitch,
                        void* const* streams) {
    if (!hs || n <= 0 || !slabs || !outs || !streams) return VIP_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; ++i)
        if (!hs[i] || hs[i]->nranks != n || hs[i]->rank != i || hs[i]->transport != hs[0]->transport ||
            !slabs[i] || !outs[i] || out_pitch < hs[i]->pitch())
            return VIP_ERR_INVALID_ARGUMENT;
    DeviceGuard guard;
    const bool rccl = hs[0]->transport == VIP_SHARD_RCCL;
    auto st = [&](int i) { return (hipStream_t)streams[i]; };
    // own rows written -> the exchange may read them
    for (int i = 0; i < n; ++i) {
        VIP_HIP_TRY(hipSetDevice(hs[i]->device));
        VIP_HIP_TRY(hipEventRecord(hs[i]->ev_in, st(i)));
    }
    if (n > 1 && hs[0]->r > 0) {
        if (rccl) {
            for (int i = 0; i < n; ++i) {
                VIP_HIP_TRY(hipSetDevice(hs[i]->device));
                VIP_HIP_TRY(hipStreamWaitEvent(hs[i]->comm, hs[i]->ev_in, 0));
            }
            if (const ncclResult_t e = ncclGroupStart()) return comm_fail(e, "ncclGroupStart");
            int rc = 0;
            for (int i = 0; i < n && !rc; ++i) {
                rc = (int)hipSetDevice(hs[i]->device);
                if (!rc) rc = enqueue_p2p(hs[i], slabs[i]);
            }
            const int rc2 = group_end(hs, n);
            if (rc || rc2) return rc ? rc : rc2;
            for (int i = 0; i < n; ++i) {
                VIP_HIP_TRY(hipSetDevice(hs[i]->device));
                VIP_HIP_TRY(hipEventRecord(hs[i]->ev_x, hs[i]->comm));
            }
        } else {
            // LOCAL: every slab on one device; shard 0's stream carries all the copies
            const hipStream_t c = hs[0]->comm;
            for (int i = 0; i < n; ++i) VIP_HIP_TRY(hipStreamWaitEvent(c, hs[i]->ev_in, 0));
            for (int i = 0; i < n; ++i) {
                const vip_shard_s* h = hs[i];
                const size_t bytes = (size_t)h->r * h->pitch();
                if (i > 0)  // own top rows -> the halo below of shard i - 1
                    VIP_HIP_TRY(hipMemcpyAsync(slabs[i - 1] + (size_t)(hs[i - 1]->r + hs[i - 1]->own) * h->pitch(),
                                               slabs[i] + (size_t)h->r * h->pitch(), bytes, hipMemcpyDeviceToDevice, c));
                if (i < n - 1)  // own bottom rows -> the halo above of shard i + 1
                    VIP_HIP_TRY(hipMemcpyAsync(slabs[i + 1], slabs[i] + (size_t)h->own * h->pitch(), bytes,
                                               hipMemcpyDeviceToDevice, c));
            }
            VIP_HIP_TRY(hipEventRecord(hs[0]->ev_x, c));  // shard 0's event covers the group
        }
        for (int i = 0; i < n; ++i) {
            VIP_HIP_TRY(hipSetDevice(hs[i]->device));
            const hipEvent_t x = rccl ? hs[i]->ev_x : hs[0]->ev_x;
            if (!hs[i]->split) {
                VIP_HIP_TRY(hipStreamWaitEvent(st(i), x, 0));
                if (const int rc = filter_rows(hs[i], slabs[i], outs[i], out_pitch, 0, hs[i]->own, st(i))) return rc;
                continue;
            }
            if (const int rc = interior(hs[i], slabs[i], outs[i], out_pitch, st(i))) return rc;
            VIP_HIP_TRY(hipStreamWaitEvent(st(i), x, 0));
            if (const int rc = edges(hs[i], slabs[i], outs[i], out_pitch, st(i))) return rc;
        }
        return 0;
    }
    for (int i = 0; i < n; ++i) {  // one shard or no halo: nothing to exchange
        VIP_HIP_TRY(hipSetDevice(hs[i]->device));
        if (const int rc = filter_rows(hs[i], slabs[i], outs[i], out_pitch, 0, hs[i]->own, st(i))) return rc;
    }
    return 0;
}

int vip_shard_destroy(vip_shard_t h) {
    if (!h) return 0;
    DeviceGuard guard;
    (void)hipSetDevice(h->device);
    free_graphs(h);
    if (h->nccl) {  // only complete communicators are stored (bounded_init)
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(h->nccl, &st) == ncclSuccess && st == ncclSuccess)
            (void)ncclCommDestroy(h->nccl);
        else
            (void)ncclCommAbort(h->nccl);  // an initialisation that timed out or failed
    }
    if (h->bil) vip_bilateral_destroy(h->bil);
    if (h->ada) vip_adaptive_destroy(h->ada);
    if (h->tex) vip_texture_destroy(h->tex);
    for (uint8_t* p : h->scratch)
        if (p) (void)hipFree(p);
    if (h->comm) (void)hipStreamDestroy(h->comm);
    if (h->ev_in) (void)hipEventDestroy(h->ev_in);
    if (h->ev_x) (void)hipEventDestroy(h->ev_x);
    delete h;
    return 0;
}

}  // extern "C"
