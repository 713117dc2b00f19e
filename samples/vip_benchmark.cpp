// Timing driver over the drop-in C++ API (include/cuda/*.hpp), the MI355X
// counterpart of the reference's sample/benchmark/main.cpp:20-213 without toml11
// or OpenCV: a random RGB8 frame (values in [lo, hi), like cv::randu(100,120)),
// one discarded warm-up call, then the mean of N blocking calls per filter.
// usage: vip_benchmark [width height] [execute_times] [ksize] [texture_ksize nitr] [--dump DIR]
// The input is 100 + (mt19937(42)() % 20) per byte (test/random_array.hpp's generator
// with max 20, shifted into the narrow [100, 120) range of the reference's benchmark),
// so the oracle can recompute it. Each filter's output is downloaded into its own
// buffer and checksummed (FNV-1a 64); --dump writes input.bin and <filter>.bin to DIR
// (tests/test_gpu_dropin.py compares them with the oracle).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "cuda/adaptive_bilateral_filter.hpp"
#include "cuda/bilateral_filter.hpp"
#include "cuda/bilateral_texture_filter.hpp"
#include "cuda/device_image.hpp"
#include "cuda/gradient.hpp"

template <class F>
static double measure_ms(int times, F&& fn) {
    double sum = 0.0;
    for (int i = 0; i <= times; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        fn();
        const auto t1 = std::chrono::steady_clock::now();
        if (i) sum += std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    return sum / times;
}

static unsigned long long fnv1a(const std::vector<std::uint8_t>& v) {
    unsigned long long h = 1469598103934665603ull;
    for (auto b : v) h = (h ^ b) * 1099511628211ull;
    return h;
}

static void dump(const std::string& dir, const char* name, const std::vector<std::uint8_t>& v) {
    if (dir.empty()) return;
    const std::string path = dir + "/" + name + ".bin";
    if (FILE* f = std::fopen(path.c_str(), "wb")) {
        std::fwrite(v.data(), 1, v.size(), f);
        std::fclose(f);
    }
}

int main(int argc, char** argv) {
    std::string dump_dir;
    if (argc > 2 && std::strcmp(argv[argc - 2], "--dump") == 0) {
        dump_dir = argv[argc - 1];
        argc -= 2;
    }
    const int width = argc > 2 ? std::atoi(argv[1]) : 100;
    const int height = argc > 2 ? std::atoi(argv[2]) : 100;
    const int times = argc > 3 ? std::atoi(argv[3]) : 10;
    const int ksize = argc > 4 ? std::atoi(argv[4]) : 9;
    const int tk = argc > 5 ? std::atoi(argv[5]) : 9;
    const int nitr = argc > 6 ? std::atoi(argv[6]) : 3;

    std::vector<std::uint8_t> host((size_t)width * height * 3);
    std::mt19937 gen(42);
    for (auto& v : host) v = (std::uint8_t)(100 + gen() % 20);
    dump(dump_dir, "input", host);

    DeviceImage<std::uint8_t> d_src(width, height, 3), d_dst(width, height, 3);
    DeviceImage<float> d_mag(width, height);
    d_src.upload(host.data());

    std::printf("Parameters\n\twidth %d height %d execute times %d ksize %d texture ksize %d nitr %d\n\n", width,
                height, times, ksize, tk, nitr);
    const auto report = [](const char* name, double ms) { std::printf("%-40s : %10.6f [msec]\n", name, ms); };

    std::vector<float> mag_host((size_t)width * height);  // scratch: the input frame stays in d_src
    report("gradient [hip]", measure_ms(times, [&] {
               cuda_gradient(d_src.get(), d_mag.get(), width, height, 3);
               d_mag.download(mag_host.data());  // the reference's call does not sync; a D2H does
           }));
    std::vector<std::uint8_t> out(host.size());
    const auto finish = [&](const char* name) {  // the input frame stays untouched in d_src
        d_dst.download(out.data());
        std::printf("checksum %-26s %016llx\n", name, fnv1a(out));
        dump(dump_dir, name, out);
    };
    CudaBilateralFilter bf(width, height, ksize);
    report("bilateral filter [hip]", measure_ms(times, [&] { bf.bilateral_filter(d_src.get(), d_dst.get()); }));
    finish("bilateral");
    CudaAdaptiveBilateralFilter abf(width, height, ksize);
    report("adaptive bilateral filter [hip]", measure_ms(times, [&] { abf.execute(d_src.get(), d_dst.get()); }));
    finish("adaptive");
    CudaBilateralTextureFilter btf(width, height, tk, nitr);
    report("bilateral texture filter [hip]", measure_ms(times, [&] { btf.execute(d_src.get(), d_dst.get()); }));
    finish("texture");
    return 0;
}
