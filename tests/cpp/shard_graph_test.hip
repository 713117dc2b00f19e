// Graph mode of the native shard (include/vip_shard.h vip_shard_set_graph) from C++, on ONE
// GPU, outside any torch process (this links the system RCCL): loopback shards
// (vip_shard_create_loopback: the row neighbours are the shard itself over a one-rank
// communicator, so the real ncclSend/ncclRecv group runs), one shard per stream, two frames
// in flight. Every replayed frame must equal the direct run of the same frame; then host
// enqueue time and device time per frame are measured for the direct and the graph form.
//
// usage: shard_graph_test [width own_rows ksize ngeo] [--texture NITR] [--split]
// exit 0 and "graph frames equal the direct frames" on success.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "vip.h"
#include "vip_shard.h"

#define CHECK(x)                                                                                 \
    do {                                                                                         \
        const int rc_ = (int)(x);                                                                \
        if (rc_) {                                                                               \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,            \
                         rc_ >= VIP_ERR_COMM ? vip_shard_last_error() : vip_error_string(rc_));   \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

static void on_segv(int sig) {
    void* bt[64];
    const int n = backtrace(bt, 64);
    std::fprintf(stderr, "signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(bt, n, 2);
    _exit(128 + sig);
}

int main(int argc, char** argv) {
    signal(SIGSEGV, on_segv);
    signal(SIGABRT, on_segv);
    int nitr = -1, split = 0, fail_capture = 0;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--texture") && i + 1 < argc) nitr = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--split")) split = 1;
        else if (!std::strcmp(argv[i], "--fail-capture")) fail_capture = 1;
        else pos.push_back(argv[i]);
    }
    // --fail-capture: every capture fails (the library's test knob); each frame must still run
    // directly, with its exchange, and graph mode must switch itself off
    if (fail_capture) setenv("VIP_SHARD_TEST_FAIL_CAPTURE", "1", 1);
    int rccl = 0;
    CHECK(vip_shard_rccl_version(&rccl));
    std::printf("RCCL %d\n", rccl);
    const int width = pos.size() >= 4 ? std::atoi(pos[0].c_str()) : 3840;
    const int own = pos.size() >= 4 ? std::atoi(pos[1].c_str()) : 270;
    const int ksize = pos.size() >= 4 ? std::atoi(pos[2].c_str()) : 15;
    const int ngeo = pos.size() >= 4 ? std::atoi(pos[3].c_str()) : 8;
    const bool texture = nitr >= 0;
    const int kind = texture ? VIP_FILTER_TEXTURE : VIP_FILTER_BILATERAL;
    const int S = 2, F = 6;  // streams (one shard each), frames (buffer f on stream f % S)
    vip_shard_t sh[S];
    for (int i = 0; i < S; ++i)
        CHECK(vip_shard_create_loopback(&sh[i], kind, width, own * ngeo, ksize, 10.f, 30.f, texture ? nitr : 0, 0,
                                        ngeo, ngeo / 2, 60000));
    int b0, own_rows, r;
    CHECK(vip_shard_geometry(sh[0], &b0, &own_rows, &r));
    if (own_rows != own) {
        std::fprintf(stderr, "own rows %d != %d\n", own_rows, own);
        return 1;
    }
    for (int i = 0; i < S; ++i)
        if (!texture) CHECK(vip_shard_set_split(sh[i], split));
    const size_t pitch = (size_t)width * 3, slab_bytes = (size_t)(own + 2 * r) * pitch, out_bytes = (size_t)own * pitch;
    hipStream_t st[S];
    for (int i = 0; i < S; ++i) CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    std::vector<uint8_t*> slab(F), out(F), ref(F);
    std::mt19937 gen(42);
    std::vector<uint8_t> host(slab_bytes);
    for (int f = 0; f < F; ++f) {
        CHECK(hipMalloc(&slab[f], slab_bytes));
        CHECK(hipMalloc(&out[f], out_bytes));
        CHECK(hipMalloc(&ref[f], out_bytes));
        for (auto& v : host) v = (uint8_t)(gen() % 255);
        CHECK(hipMemcpy(slab[f], host.data(), slab_bytes, hipMemcpyHostToDevice));
    }
    auto round = [&](std::vector<uint8_t*>& dst) -> int {
        for (int f = 0; f < F; ++f) {
            const int rc = vip_shard_run(sh[f % S], slab[f], dst[f], pitch, st[f % S]);
            if (rc) return rc;
        }
        return 0;
    };
    CHECK(round(ref));  // direct
    CHECK(hipDeviceSynchronize());
    for (int i = 0; i < S; ++i) CHECK(vip_shard_set_graph(sh[i], 1));
    std::vector<uint8_t> a(out_bytes), b(out_bytes);
    for (int rnd = 0; rnd < 3; ++rnd) {  // round 0 captures, then replays
        for (int f = 0; f < F; ++f) CHECK(hipMemset(out[f], 3, out_bytes));
        CHECK(hipDeviceSynchronize());
        CHECK(round(out));
        CHECK(hipDeviceSynchronize());
        for (int f = 0; f < F; ++f) {
            CHECK(hipMemcpy(a.data(), out[f], out_bytes, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(b.data(), ref[f], out_bytes, hipMemcpyDeviceToHost));
            if (std::memcmp(a.data(), b.data(), out_bytes)) {
                std::fprintf(stderr, "round %d frame %d differs from the direct run\n", rnd, f);
                return 1;
            }
        }
    }
    int ng = 0;
    CHECK(vip_shard_graph_count(sh[0], &ng));
    std::printf("graph frames equal the direct frames (%d graphs on shard 0)\n", ng);
    if (fail_capture) {
        if (ng != 0) {
            std::fprintf(stderr, "a failed capture left %d graphs\n", ng);
            return 1;
        }
        std::printf("failed captures fell back to direct frames, graph mode off\n");
    }
    // the caller's streams need not outlive the shard: destroy one, then drop the graphs
    if (!fail_capture && ng > 0) {
        CHECK(hipDeviceSynchronize());
        for (int i = 0; i < S; ++i) CHECK(hipStreamDestroy(st[i]));
        for (int i = 0; i < S; ++i) CHECK(vip_shard_set_graph(sh[i], 0));
        for (int i = 0; i < S; ++i) CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        std::printf("graphs dropped after their streams were destroyed\n");
    }
    // host enqueue and device time per frame, direct vs graph (frames in flight on S streams)
    for (int graph = 0; graph < 2; ++graph) {
        for (int i = 0; i < S; ++i) CHECK(vip_shard_set_graph(sh[i], graph));
        for (int w = 0; w < 5; ++w) CHECK(round(out));
        CHECK(hipDeviceSynchronize());
        const int rounds = 200;
        const auto t0 = std::chrono::steady_clock::now();
        double host_us = 0;
        for (int k = 0; k < rounds; ++k) {
            const auto h0 = std::chrono::steady_clock::now();
            CHECK(round(out));
            host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
        }
        CHECK(hipDeviceSynchronize());
        const double wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%-6s %dx%d slab (r=%d, %s%s): host enqueue %.2f us per frame, wall %.2f us per frame\n",
                    graph ? "graph" : "direct", width, own, r, texture ? "texture" : "bilateral",
                    split ? ", split" : "", host_us / (rounds * F), wall_us / (rounds * F));
    }
    for (int i = 0; i < S; ++i) CHECK(vip_shard_destroy(sh[i]));
    return 0;
}
