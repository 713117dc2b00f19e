// Row-sharded frame driver over the native sharding C ABI (include/vip_shard.h): the
// north_star's configuration 5 -- bilateral r=15 on a 16384x16384 RGB8 frame, row-tiled
// over every visible GPU with the r-row halos exchanged by RCCL ncclSend/ncclRecv -- from
// C++, in one process (one RCCL communicator per device, ncclCommInitAll's pattern).
// The reference has no multi-device code; this is what a C++ caller of
// vip_bilateral_run_rows would otherwise write by hand.
//
// usage: vip_shard_frame [width height ksize] [steps] [--local N] [--adaptive | --texture NITR]
//   default 16384 16384 31, 10 timed steps; --local N: N shards on device 0 (halos by
//   device copies), the same code path on a single GPU; --texture NITR: the bilateral
//   texture filter with k = ksize (one nitr-deep halo exchange per frame).
// The frame is mt19937(42) % 255 per byte (test/random_array.hpp's generator); each
// device gets its own rows, the sharded output is gathered and compared byte for byte
// with one whole-frame launch on device 0. Prints Mpixels/s over the timed steps (host
// clock around vip_shard_run_group + a device sync per device).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "vip.h"
#include "vip_shard.h"

#define CHECK(x)                                                                                 \
    do {                                                                                         \
        const int rc_ = (x);                                                                     \
        if (rc_) {                                                                               \
            std::fprintf(stderr, "%s:%d %s -> %d (%s%s%s)\n", __FILE__, __LINE__, #x, rc_,        \
                         vip_error_string(rc_), rc_ >= VIP_ERR_COMM ? ": " : "",                 \
                         rc_ >= VIP_ERR_COMM ? vip_shard_last_error() : "");                      \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

int main(int argc, char** argv) {
    int local = 0, nitr = -1;
    bool adaptive = false;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--local") && i + 1 < argc) local = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--adaptive")) adaptive = true;
        else if (!std::strcmp(argv[i], "--texture") && i + 1 < argc) nitr = std::atoi(argv[++i]);
        else pos.push_back(argv[i]);
    }
    const int width = pos.size() >= 3 ? std::atoi(pos[0].c_str()) : 16384;
    const int height = pos.size() >= 3 ? std::atoi(pos[1].c_str()) : 16384;
    const int ksize = pos.size() >= 3 ? std::atoi(pos[2].c_str()) : 31;
    const int steps = pos.size() >= 4 ? std::atoi(pos[3].c_str()) : (pos.size() == 1 ? std::atoi(pos[0].c_str()) : 10);
    const bool texture = nitr >= 0;
    const int kind = texture ? VIP_FILTER_TEXTURE : adaptive ? VIP_FILTER_ADAPTIVE : VIP_FILTER_BILATERAL;
    int ndev = 0;
    CHECK(vip_device_count(&ndev));
    const int n = local > 0 ? local : ndev;
    const int transport = local > 0 ? VIP_SHARD_LOCAL : VIP_SHARD_RCCL;
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = local > 0 ? 0 : i;
    std::printf("frame %dx%d ksize %d %s, %d shard(s) on %s\n", width, height, ksize,
                texture ? "texture" : adaptive ? "adaptive" : "bilateral", n,
                local > 0 ? "device 0 (LOCAL transport)" : "one GPU each (RCCL)");

    const size_t pitch = (size_t)width * 3;
    std::vector<uint8_t> frame(pitch * height);
    std::mt19937 gen(42);
    for (auto& b : frame) b = (uint8_t)(gen() % 255);

    CHECK(vip_set_device(devs[0]));
    std::vector<vip_shard_t> hs(n);
    if (texture)
        CHECK(vip_shard_create_group_texture(hs.data(), n, transport, devs.data(), width, height, ksize, nitr,
                                             VIP_NUMERICS_CUDA, 120000));
    else
        CHECK(vip_shard_create_group(hs.data(), n, transport, devs.data(), kind, width, height, ksize, 10.f, 30.f,
                                     VIP_NUMERICS_CUDA, 120000));
    std::vector<uint8_t*> slabs(n), outs(n);
    std::vector<void*> streams(n);
    std::vector<int> own(n), begin(n);
    for (int i = 0; i < n; ++i) {
        int r = 0;
        CHECK(vip_shard_geometry(hs[i], &begin[i], &own[i], &r));
        CHECK(vip_set_device(devs[i]));
        CHECK(vip_malloc(reinterpret_cast<void**>(&slabs[i]), pitch * (own[i] + 2 * r)));
        CHECK(vip_malloc(reinterpret_cast<void**>(&outs[i]), pitch * own[i]));
        CHECK(vip_stream_create(&streams[i]));
        CHECK(vip_upload(slabs[i] + pitch * r, frame.data() + pitch * begin[i], pitch * own[i]));  // own rows only
    }
    auto sync_all = [&]() {
        for (int i = 0; i < n; ++i) {
            if (vip_set_device(devs[i]) || vip_stream_synchronize(streams[i])) return 1;
        }
        return 0;
    };
    CHECK(vip_shard_run_group(hs.data(), n, slabs.data(), outs.data(), pitch, streams.data()));  // warm-up
    CHECK(sync_all());
    const auto t0 = std::chrono::steady_clock::now();
    for (int s = 0; s < steps; ++s)
        CHECK(vip_shard_run_group(hs.data(), n, slabs.data(), outs.data(), pitch, streams.data()));
    CHECK(sync_all());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / steps;
    std::vector<uint8_t> got(pitch * height);
    for (int i = 0; i < n; ++i) {
        CHECK(vip_set_device(devs[i]));
        CHECK(vip_download(got.data() + pitch * begin[i], outs[i], pitch * own[i]));
    }
    // reference: one launch over the whole frame on device 0
    CHECK(vip_set_device(devs[0]));
    uint8_t *d_src = nullptr, *d_dst = nullptr;
    CHECK(vip_malloc(reinterpret_cast<void**>(&d_src), frame.size()));
    CHECK(vip_malloc(reinterpret_cast<void**>(&d_dst), frame.size()));
    CHECK(vip_upload(d_src, frame.data(), frame.size()));
    if (texture) {
        vip_texture_t t = nullptr;
        CHECK(vip_texture_create(&t, width, height, ksize, nitr, VIP_NUMERICS_CUDA));
        CHECK(vip_texture_run(t, d_src, d_dst, nullptr));
        CHECK(vip_device_synchronize());
        vip_texture_destroy(t);
    } else if (adaptive) {
        vip_adaptive_t a = nullptr;
        CHECK(vip_adaptive_create(&a, width, height, ksize, 10.f, 30.f, VIP_NUMERICS_CUDA));
        CHECK(vip_adaptive_run(a, d_src, pitch, d_dst, pitch, nullptr));
        CHECK(vip_device_synchronize());
        vip_adaptive_destroy(a);
    } else {
        vip_bilateral_t b = nullptr;
        CHECK(vip_bilateral_create(&b, width, height, ksize, 10.f, 30.f, VIP_NUMERICS_CUDA));
        CHECK(vip_bilateral_run(b, d_src, pitch, d_dst, pitch, nullptr));
        CHECK(vip_device_synchronize());
        vip_bilateral_destroy(b);
    }
    std::vector<uint8_t> want(frame.size());
    CHECK(vip_download(want.data(), d_dst, want.size()));
    size_t diff = 0;
    for (size_t j = 0; j < want.size(); ++j) diff += got[j] != want[j];
    std::printf("sharded step %.3f ms, %.1f Mpixels/s over %d step(s); %s one-launch output (%zu differing bytes)\n",
                ms, (double)width * height / (ms * 1e3), steps, diff ? "DIFFERS from the" : "equals the", diff);
    for (int i = 0; i < n; ++i) {
        vip_set_device(devs[i]);
        vip_free(slabs[i]);
        vip_free(outs[i]);
        vip_stream_destroy(streams[i]);
        vip_shard_destroy(hs[i]);
    }
    vip_set_device(devs[0]);
    vip_free(d_src);
    vip_free(d_dst);
    return diff ? 2 : 0;
}
