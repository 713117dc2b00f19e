// Timing driver over the drop-in C++ API (include/cuda/*.hpp), the MI355X
// counterpart of the reference's sample/benchmark/main.cpp:20-213 without toml11
// or OpenCV: a random RGB8 frame (values in [lo, hi), like cv::randu(100,120)),
// one discarded warm-up call, then the mean of N blocking calls per filter.
// usage: vip_benchmark [width height] [execute_times] [ksize] [texture_ksize nitr]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
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

int main(int argc, char** argv) {
    const int width = argc > 2 ? std::atoi(argv[1]) : 100;
    const int height = argc > 2 ? std::atoi(argv[2]) : 100;
    const int times = argc > 3 ? std::atoi(argv[3]) : 10;
    const int ksize = argc > 4 ? std::atoi(argv[4]) : 9;
    const int tk = argc > 5 ? std::atoi(argv[5]) : 9;
    const int nitr = argc > 6 ? std::atoi(argv[6]) : 3;

    std::vector<std::uint8_t> host((size_t)width * height * 3);
    std::mt19937 gen(42);
    std::uniform_int_distribution<int> dist(100, 119);
    for (auto& v : host) v = (std::uint8_t)dist(gen);

    DeviceImage<std::uint8_t> d_src(width, height, 3), d_dst(width, height, 3);
    DeviceImage<float> d_mag(width, height);
    d_src.upload(host.data());

    std::printf("Parameters\n\twidth %d height %d execute times %d ksize %d texture ksize %d nitr %d\n\n", width,
                height, times, ksize, tk, nitr);
    const auto report = [](const char* name, double ms) { std::printf("%-40s : %10.6f [msec]\n", name, ms); };

    report("gradient [hip]", measure_ms(times, [&] {
               cuda_gradient(d_src.get(), d_mag.get(), width, height, 3);
               d_dst.download(host.data());  // the reference's call does not sync; a D2H does
           }));
    d_src.upload(host.data());
    CudaBilateralFilter bf(width, height, ksize);
    report("bilateral filter [hip]", measure_ms(times, [&] { bf.bilateral_filter(d_src.get(), d_dst.get()); }));
    CudaAdaptiveBilateralFilter abf(width, height, ksize);
    report("adaptive bilateral filter [hip]", measure_ms(times, [&] { abf.execute(d_src.get(), d_dst.get()); }));
    CudaBilateralTextureFilter btf(width, height, tk, nitr);
    report("bilateral texture filter [hip]", measure_ms(times, [&] { btf.execute(d_src.get(), d_dst.get()); }));
    d_dst.download(host.data());
    unsigned long long checksum = 0;
    for (auto v : host) checksum = checksum * 131 + v;
    std::printf("checksum %llu\n", checksum);
    return 0;
}
