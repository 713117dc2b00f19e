// Per-filter image driver over the drop-in C++ API (include/cuda/*.hpp): the MI355X
// counterpart of the reference's sample/{bilateral_filter, adaptive_bilateral_filter,
// bilateral_texture_filter, gradient}/main.cpp, with the same positional parameters and
// defaults, and without OpenCV or a display: the image is read as cv::imread(...,
// IMREAD_COLOR) would (vip_image_io.hpp: PNG / PPM / PGM -> BGR), uploaded into a
// DeviceImage, filtered by the public blocking call, downloaded and written to a file.
//
//   vip_filter bilateral IN OUT [ksize=9] [sigma_space=10] [sigma_color=30]
//                                       (sample/bilateral_filter/main.cpp:14-17)
//   vip_filter joint     IN GUIDE OUT [ksize=9] [sigma_space=10] [sigma_color=30]
//                                       (CudaBilateralFilter::joint_bilateral_filter)
//   vip_filter adaptive  IN OUT [ksize=9] [sigma_space=10] [sigma_color=30]
//                                       (sample/adaptive_bilateral_filter/main.cpp:15-18)
//   vip_filter texture   IN OUT [ksize=9] [nitr=3]
//                                       (sample/bilateral_texture_filter/main.cpp:15-17)
//   vip_filter gradient  IN OUT         (sample/gradient/main.cpp:23-40; OUT is the
//                                       magnitude scaled to 0..255 by its maximum as the
//                                       sample's convert_to_u8 displays it, or the raw
//                                       float32 magnitudes when OUT ends in .f32)
//   vip_filter convert   IN OUT         (no GPU: re-encode an image, e.g. PNG -> PPM)
//
// Options (anywhere): --repeat N  time N more blocking calls after the first and print
// the mean in ms. The output extension picks the format (.png, .ppm, .pgm). Exit
// status 0 on success, 1 on a usage / file error, 2 on a filter error.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cuda/adaptive_bilateral_filter.hpp"
#include "cuda/bilateral_filter.hpp"
#include "cuda/bilateral_texture_filter.hpp"
#include "cuda/device_image.hpp"
#include "cuda/gradient.hpp"
#include "vip.h"
#include "vip_image_io.hpp"

static int usage() {
    std::fprintf(stderr,
                 "[Usage] vip_filter bilateral IN OUT [ksize] [sigma_space] [sigma_color]\n"
                 "        vip_filter joint IN GUIDE OUT [ksize] [sigma_space] [sigma_color]\n"
                 "        vip_filter adaptive IN OUT [ksize] [sigma_space] [sigma_color]\n"
                 "        vip_filter texture IN OUT [ksize] [nitr]\n"
                 "        vip_filter gradient IN OUT\n"
                 "        vip_filter convert IN OUT\n"
                 "        options: --repeat N\n");
    return 1;
}

// Runs fn once (the output), then `repeat` more times and prints their mean.
template <class F>
static void run_timed(const char* name, int repeat, F&& fn) {
    fn();
    if (repeat <= 0) return;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < repeat; ++i) fn();
    const auto t1 = std::chrono::steady_clock::now();
    std::printf("%-28s : %10.6f [msec]\n", name, std::chrono::duration<double, std::milli>(t1 - t0).count() / repeat);
}

// The public filter calls print launch errors and carry on (the reference's
// CUDASafeCall); a sample must not report success after one.
static bool device_ok() {
    const int rc = vip_device_synchronize();
    if (rc != 0) std::fprintf(stderr, "vip_filter: device error %d\n", rc);
    return rc == 0;
}

int main(int argc, char** argv) {
    int repeat = 0;
    std::vector<std::string> args;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--repeat") && i + 1 < argc) {
            repeat = std::atoi(argv[++i]);
        } else {
            args.emplace_back(argv[i]);
        }
    }
    if (args.size() < 3) return usage();
    const std::string mode = args[0];
    const bool joint = mode == "joint";
    const size_t np = joint ? 4 : 3;  // index of the first numeric parameter
    if (args.size() < np) return usage();
    auto int_arg = [&](size_t i, int def) { return args.size() > i ? std::stoi(args[i]) : def; };
    auto flt_arg = [&](size_t i, float def) { return args.size() > i ? std::stof(args[i]) : def; };
    const std::string out_path = args[np - 1];

    vip_io::Image in, guide;
    try {
        in = vip_io::read_image(args[1]);
        if (joint) guide = vip_io::read_image(args[2]);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Failed to load: %s\n", e.what());
        return 1;
    }
    if (joint && (guide.width != in.width || guide.height != in.height)) {
        std::fprintf(stderr, "guide size %dx%d != image size %dx%d\n", guide.width, guide.height, in.width, in.height);
        return 1;
    }
    const int W = in.width, H = in.height;
    vip_io::Image out;
    out.width = W;
    out.height = H;
    out.channels = 3;
    out.data.resize((size_t)W * H * 3);

    try {
        if (mode == "convert") {
            out = in;
        } else if (mode == "bilateral" || joint || mode == "adaptive" || mode == "texture") {
            DeviceImage<std::uint8_t> d_src(W, H, 3), d_dst(W, H, 3);
            d_src.upload(in.data.data());
            if (mode == "bilateral" || joint) {
                CudaBilateralFilter filter(W, H, int_arg(np, 9), flt_arg(np + 1, 10.f), flt_arg(np + 2, 30.f));
                if (joint) {
                    DeviceImage<std::uint8_t> d_guide(W, H, 3);
                    d_guide.upload(guide.data.data());
                    run_timed("joint bilateral filter", repeat,
                              [&] { filter.joint_bilateral_filter(d_src.get(), d_guide.get(), d_dst.get()); });
                } else {
                    run_timed("bilateral filter", repeat, [&] { filter.bilateral_filter(d_src.get(), d_dst.get()); });
                }
            } else if (mode == "adaptive") {
                CudaAdaptiveBilateralFilter filter(W, H, int_arg(np, 9), flt_arg(np + 1, 10.f), flt_arg(np + 2, 30.f));
                run_timed("adaptive bilateral filter", repeat, [&] { filter.execute(d_src.get(), d_dst.get()); });
            } else {
                CudaBilateralTextureFilter filter(W, H, int_arg(np, 9), int_arg(np + 1, 3));
                run_timed("bilateral texture filter", repeat, [&] { filter.execute(d_src.get(), d_dst.get()); });
            }
            if (!device_ok()) return 2;
            d_dst.download(out.data.data());
        } else if (mode == "gradient") {
            DeviceImage<std::uint8_t> d_src(W, H, 3);
            DeviceImage<float> d_mag(W, H, 1);
            d_src.upload(in.data.data());
            run_timed("gradient", repeat, [&] { cuda_gradient(d_src.get(), d_mag.get(), W, H, 3); });
            if (!device_ok()) return 2;
            std::vector<float> mag((size_t)W * H);
            d_mag.download(mag.data());
            if (vip_io::ends_with(out_path, ".f32")) {
                std::vector<std::uint8_t> bytes(mag.size() * sizeof(float));
                std::memcpy(bytes.data(), mag.data(), bytes.size());
                vip_io::write_file(out_path, bytes);
                return 0;
            }
            // sample/gradient/main.cpp:8-15: img * 255 / max (float image), then a
            // rounding, saturating conversion to 8 bits (cvRound: ties to even)
            double mx = 0.0;
            for (float v : mag) mx = v > mx ? v : mx;
            const float scale = (float)(255.0 / mx);
            out.channels = 1;
            out.data.resize(mag.size());
            for (size_t i = 0; i < mag.size(); ++i) {
                const float v = std::nearbyint(mag[i] * scale);
                out.data[i] = (std::uint8_t)(v != v ? 0.f : v < 0.f ? 0.f : v > 255.f ? 255.f : v);
            }
        } else {
            return usage();
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "vip_filter: %s\n", e.what());
        return 2;
    }
    try {
        vip_io::write_image(out_path, out);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "vip_filter: %s\n", e.what());
        return 1;
    }
    return 0;
}
