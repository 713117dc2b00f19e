// Host-frame pipeline over the drop-in C++ API: frames arrive in
// page-locked host memory, are uploaded, filtered and downloaded on NS streams so
// the H2D copy of frame f+1, the kernel of frame f and the D2H copy of frame f-1
// overlap (copy engines run beside the compute queue). Reports the PCIe-inclusive
// frame rate next to the kernel-only and copy-only rates.
// usage: vip_host_pipeline [width height] [frames] [ksize] [streams]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cuda/bilateral_filter.hpp"
#include "cuda/device_image.hpp"
#include "vip.h"

#define CHECK(expr)                                                                              \
    do {                                                                                         \
        const int rc_ = (expr);                                                                  \
        if (rc_) {                                                                               \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #expr, vip_error_string(rc_)); \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

int main(int argc, char** argv) {
    const int width = argc > 2 ? std::atoi(argv[1]) : 3840;
    const int height = argc > 2 ? std::atoi(argv[2]) : 2160;
    const int frames = argc > 3 ? std::atoi(argv[3]) : 60;
    const int ksize = argc > 4 ? std::atoi(argv[4]) : 15;
    const int ns = argc > 5 ? std::atoi(argv[5]) : 3;
    const size_t bytes = (size_t)width * height * 3;

    std::vector<std::uint8_t*> h_in(ns), h_out(ns);
    std::vector<void*> streams(ns);
    std::vector<DeviceImage<std::uint8_t>> d_src, d_dst;
    std::mt19937 gen(42);
    for (int s = 0; s < ns; ++s) {
        CHECK(vip_host_alloc(reinterpret_cast<void**>(&h_in[s]), bytes));
        CHECK(vip_host_alloc(reinterpret_cast<void**>(&h_out[s]), bytes));
        for (size_t i = 0; i < bytes; ++i) h_in[s][i] = (std::uint8_t)(gen() % 255);
        CHECK(vip_stream_create(&streams[s]));
        d_src.emplace_back(width, height, 3);
        d_dst.emplace_back(width, height, 3);
    }
    CudaBilateralFilter filter(width, height, ksize);

    // warm-up: every slot once
    for (int s = 0; s < ns; ++s) {
        d_src[s].upload_async(h_in[s], streams[s]);
        filter.bilateral_filter(d_src[s].get(), d_dst[s].get(), streams[s]);
        d_dst[s].download_async(h_out[s], streams[s]);
    }
    CHECK(vip_device_synchronize());

    // kernel only (frames resident in HBM)
    auto t0 = clk::now();
    for (int f = 0; f < frames; ++f) filter.bilateral_filter(d_src[f % ns].get(), d_dst[f % ns].get(), streams[0]);
    CHECK(vip_stream_synchronize(streams[0]));
    const double kernel_ms = ms_since(t0) / frames;

    // copies only, H2D and D2H on separate streams
    t0 = clk::now();
    for (int f = 0; f < frames; ++f) d_src[f % ns].upload_async(h_in[f % ns], streams[0]);
    CHECK(vip_stream_synchronize(streams[0]));
    const double h2d_ms = ms_since(t0) / frames;
    t0 = clk::now();
    for (int f = 0; f < frames; ++f) d_dst[f % ns].download_async(h_out[f % ns], streams[0]);
    CHECK(vip_stream_synchronize(streams[0]));
    const double d2h_ms = ms_since(t0) / frames;

    // both directions at once, H2D on stream 0 and D2H on stream 1 (can they overlap?)
    double both_ms = 0.0;
    if (ns >= 2) {
        t0 = clk::now();
        for (int f = 0; f < frames; ++f) {
            d_src[f % ns].upload_async(h_in[f % ns], streams[0]);
            d_dst[f % ns].download_async(h_out[f % ns], streams[1]);
        }
        CHECK(vip_device_synchronize());
        both_ms = ms_since(t0) / frames;
    }

    // pipelined host frames: slot f % ns; reusing a slot waits for its previous frame
    t0 = clk::now();
    for (int f = 0; f < frames; ++f) {
        const int s = f % ns;
        if (f >= ns) CHECK(vip_stream_synchronize(streams[s]));  // h_out[s] of frame f-ns is ready here
        d_src[s].upload_async(h_in[s], streams[s]);
        filter.bilateral_filter(d_src[s].get(), d_dst[s].get(), streams[s]);
        d_dst[s].download_async(h_out[s], streams[s]);
    }
    CHECK(vip_device_synchronize());
    const double pipe_ms = ms_since(t0) / frames;

    // split pipeline: uploads on one stream, filters on another, downloads on a third,
    // ordered by events; slot s = f % ns is reused once frame f-ns has left it
    // (filter of f waits for the upload of f and the download of f-ns; upload of f
    // waits for the filter of f-ns, which read d_src[s])
    void *su = nullptr, *sc = nullptr, *sd = nullptr;
    CHECK(vip_stream_create(&su));
    CHECK(vip_stream_create(&sc));
    CHECK(vip_stream_create(&sd));
    std::vector<void*> ev_up(ns), ev_flt(ns), ev_down(ns);
    for (int s = 0; s < ns; ++s) {
        CHECK(vip_event_create(&ev_up[s]));
        CHECK(vip_event_create(&ev_flt[s]));
        CHECK(vip_event_create(&ev_down[s]));
    }
    t0 = clk::now();
    for (int f = 0; f < frames; ++f) {
        const int s = f % ns;
        if (f >= ns) CHECK(vip_stream_wait_event(su, ev_flt[s]));
        d_src[s].upload_async(h_in[s], su);
        CHECK(vip_event_record(ev_up[s], su));
        CHECK(vip_stream_wait_event(sc, ev_up[s]));
        if (f >= ns) CHECK(vip_stream_wait_event(sc, ev_down[s]));
        filter.bilateral_filter(d_src[s].get(), d_dst[s].get(), sc);
        CHECK(vip_event_record(ev_flt[s], sc));
        CHECK(vip_stream_wait_event(sd, ev_flt[s]));
        d_dst[s].download_async(h_out[s], sd);
        CHECK(vip_event_record(ev_down[s], sd));
    }
    CHECK(vip_device_synchronize());
    const double split_ms = ms_since(t0) / frames;
    // the last ns frames' outputs against the kernel-only results of the same inputs
    std::vector<std::uint8_t> check(bytes);
    bool split_ok = true;
    for (int s = 0; s < ns; ++s) {
        filter.bilateral_filter(d_src[s].get(), d_dst[s].get(), streams[0]);
        d_dst[s].download_async(check.data(), streams[0]);
        CHECK(vip_stream_synchronize(streams[0]));
        split_ok = split_ok && std::memcmp(check.data(), h_out[s], bytes) == 0;
    }
    for (int s = 0; s < ns; ++s) {
        vip_event_destroy(ev_up[s]);
        vip_event_destroy(ev_flt[s]);
        vip_event_destroy(ev_down[s]);
    }
    vip_stream_destroy(su);
    vip_stream_destroy(sc);
    vip_stream_destroy(sd);

    const double mpx = (double)width * height / 1e6;
    std::printf("frame %dx%d RGB8 (%.1f MB), ksize %d, %d frames, %d streams\n", width, height, bytes / 1e6, ksize,
                frames, ns);
    std::printf("%-34s : %8.3f ms/frame  %9.1f Mpx/s\n", "kernel only (HBM resident)", kernel_ms, mpx / kernel_ms * 1e3);
    std::printf("%-34s : %8.3f ms/frame  %9.1f GB/s\n", "H2D pinned", h2d_ms, bytes / h2d_ms / 1e6);
    std::printf("%-34s : %8.3f ms/frame  %9.1f GB/s\n", "D2H pinned", d2h_ms, bytes / d2h_ms / 1e6);
    if (ns >= 2)
        std::printf("%-34s : %8.3f ms/frame  %9.1f GB/s\n", "H2D || D2H (two streams)", both_ms,
                    2.0 * bytes / both_ms / 1e6);
    std::printf("%-34s : %8.3f ms/frame  %9.1f Mpx/s\n", "host frames, H2D+filter+D2H piped", pipe_ms,
                mpx / pipe_ms * 1e3);
    std::printf("%-34s : %8.3f ms/frame  %9.1f Mpx/s  (outputs %s)\n", "host frames, split up/filter/down", split_ms,
                mpx / split_ms * 1e3, split_ok ? "match" : "MISMATCH");

    for (int s = 0; s < ns; ++s) {
        vip_host_free(h_in[s]);
        vip_host_free(h_out[s]);
        vip_stream_destroy(streams[s]);
    }
    return split_ok ? 0 : 1;
}
