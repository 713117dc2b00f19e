// White-box drop-in test of the C++ API (include/cuda/*.hpp + include/impl/*.cuh),
// built with hipcc + rocThrust the way the reference's test binary is built with
// nvcc + thrust (test/CMakeLists.txt:20-39), and driven the way its tests drive the
// filters:
//   * subclasses that call impl_->... without a device sync
//     (test/bilateral_filter.cu:9-33, test/bilateral_texture_filter.cu:115-136);
//   * thrust::device_vector buffers, including the device_vector overloads of the
//     texture stages (src/bilateral_texture_filter_impl.cuh:19-28);
//   * DeviceImage<T> upload/download (src/device_image.cu:5-52) and cuda_gradient<T>.
// Inputs are the reference tests' random_array vectors (tests/golden/random_array_*.bin,
// written by the reference's own generator). Every output is written to OUT_DIR as raw
// bytes; tests/test_gpu_dropin.py compares them with tests/golden/oracle_small.npz.
//
// usage: dropin_test GOLDEN_DIR OUT_DIR
#include <thrust/copy.h>
#include <thrust/device_vector.h>
#include <thrust/host_vector.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "adaptive_bilateral_filter_impl.cuh"  // include/impl, the names test/*.cu include
#include "bilateral_filter_impl.cuh"
#include "bilateral_texture_filter_impl.cuh"
#include "cuda/device_image.hpp"
#include "cuda/gradient.hpp"

#ifndef VIP_HAVE_THRUST
#error "rocThrust overloads of the texture-stage Impl methods were not compiled"
#endif

namespace {

int g_failures = 0;
#define CHECK(cond, ...)                                 \
    do {                                                 \
        if (!(cond)) {                                   \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);           \
            std::fprintf(stderr, "\n");                  \
            ++g_failures;                                \
        }                                                \
    } while (0)

template <class T>
std::vector<T> read_bin(const std::string& path, size_t n) {
    std::vector<T> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    CHECK(f != nullptr, "cannot open %s", path.c_str());
    if (f) {
        const size_t got = std::fread(v.data(), sizeof(T), n, f);
        CHECK(got == n, "%s: %zu of %zu elements", path.c_str(), got, n);
        std::fclose(f);
    }
    return v;
}

template <class T>
void write_bin(const std::string& dir, const char* name, const std::vector<T>& v) {
    const std::string path = dir + "/" + name + ".bin";
    FILE* f = std::fopen(path.c_str(), "wb");
    CHECK(f != nullptr, "cannot write %s", path.c_str());
    if (f) {
        std::fwrite(v.data(), sizeof(T), v.size(), f);
        std::fclose(f);
    }
}

template <class T>
std::vector<T> to_host(const thrust::device_vector<T>& d) {
    std::vector<T> h(d.size());
    thrust::copy(d.begin(), d.end(), h.begin());  // the D2H copy is what synchronises
    return h;
}

// The reference tests' white-box subclasses: impl_ calls, no synchronisation.
class CudaBilateralFilterImpl : public CudaBilateralFilter {
public:
    CudaBilateralFilterImpl(int w, int h, int k = 9, float ss = 10.f, float sc = 30.f)
        : CudaBilateralFilter(w, h, k, ss, sc) {}
    void bilateral_filter(const std::uint8_t* s, std::uint8_t* d) { impl_->bilateral_filter(s, d); }
    void joint_bilateral_filter(const std::uint8_t* s, const std::uint8_t* g, std::uint8_t* d) {
        impl_->joint_bilateral_filter(s, g, d);
    }
};

class CudaAdaptiveBilateralFilterImpl : public CudaAdaptiveBilateralFilter {
public:
    CudaAdaptiveBilateralFilterImpl(int w, int h, int k = 9) : CudaAdaptiveBilateralFilter(w, h, k) {}
    void execute(const std::uint8_t* s, std::uint8_t* d) { impl_->execute(s, d); }
};

class CudaBilateralTextureFilterImpl : public CudaBilateralTextureFilter {
public:
    CudaBilateralTextureFilterImpl(int w, int h, int k = 9, int n = 3) : CudaBilateralTextureFilter(w, h, k, n) {}
    void compute_blur_and_rtv(const thrust::device_vector<std::uint8_t>& img, const thrust::device_vector<float>& mag,
                              thrust::device_vector<float>& blurred, thrust::device_vector<float>& rtv) {
        impl_->compute_blur_and_rtv(img, mag, blurred, rtv);
    }
    void compute_guide(const thrust::device_vector<float>& blurred, const thrust::device_vector<float>& rtv,
                       thrust::device_vector<std::uint8_t>& guide) {
        impl_->compute_guide(blurred, rtv, guide);
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s GOLDEN_DIR OUT_DIR\n", argv[0]);
        return 2;
    }
    const std::string gold = argv[1], out = argv[2];
    constexpr int W = 50, H = 50, N = W * H;

    const auto img = read_bin<std::uint8_t>(gold + "/random_array_u8_7500_255.bin", 3 * N);
    const auto gray = read_bin<std::uint8_t>(gold + "/random_array_u8_2500_255.bin", N);
    const auto mag = read_bin<float>(gold + "/random_array_f32_2500_255.bin", N);
    const auto blurred_in = read_bin<float>(gold + "/random_array_f32_7500_255.bin", 3 * N);
    const auto rtv_in = read_bin<float>(gold + "/random_array_f32_2500_1.bin", N);
    // mt19937(42) % 255 per byte, the reference generator, cross-checked on the fixture
    std::vector<std::uint8_t> tex_in(64 * 48 * 3);
    {
        std::mt19937 gen(42);
        for (auto& v : tex_in) v = (std::uint8_t)(gen() % 255);
        bool same = true;
        for (int i = 0; i < 3 * N; ++i) same = same && tex_in[i] == img[i];
        CHECK(same, "mt19937(42) %% 255 differs from the reference generator's fixture");
    }
    std::vector<std::uint8_t> guide_img(img.rbegin(), img.rend());  // the goldens' JBF guide

    // bilateral / joint bilateral through impl_ on thrust::device_vector buffers
    {
        thrust::device_vector<std::uint8_t> d_src(img.begin(), img.end()), d_dst(3 * N);
        thrust::device_vector<std::uint8_t> d_guide(guide_img.begin(), guide_img.end());
        CudaBilateralFilterImpl bf(W, H, 9);
        bf.bilateral_filter(d_src.data().get(), d_dst.data().get());
        write_bin(out, "bilateral_k9", to_host(d_dst));
        bf.joint_bilateral_filter(d_src.data().get(), d_guide.data().get(), d_dst.data().get());
        write_bin(out, "joint_k9", to_host(d_dst));
        CudaBilateralFilterImpl bf15(W, H, 15);
        bf15.bilateral_filter(d_src.data().get(), d_dst.data().get());
        write_bin(out, "bilateral_k15", to_host(d_dst));
        CudaAdaptiveBilateralFilterImpl abf(W, H, 9);
        abf.execute(d_src.data().get(), d_dst.data().get());
        write_bin(out, "adaptive_k9", to_host(d_dst));
    }
    // the public (blocking) API on DeviceImage buffers
    {
        DeviceImage<std::uint8_t> d_src(W, H, 3), d_dst(W, H, 3);
        d_src.upload(img.data());
        std::vector<std::uint8_t> h(3 * N);
        CudaBilateralFilter(W, H, 31).bilateral_filter(d_src.get(), d_dst.get());
        d_dst.download(h.data());
        write_bin(out, "bilateral_k31", h);
        CudaAdaptiveBilateralFilter(W, H, 15).execute(d_src.get(), d_dst.get());
        d_dst.download(h.data());
        write_bin(out, "adaptive_k15", h);
        DeviceImage<std::uint8_t> d_tex(64, 48, 3), d_tex_out(64, 48, 3);
        d_tex.upload(tex_in.data());
        CudaBilateralTextureFilter(64, 48, 5, 5).execute(d_tex.get(), d_tex_out.get());
        std::vector<std::uint8_t> t(tex_in.size());
        d_tex_out.download(t.data());
        write_bin(out, "texture_k5_n5", t);
    }
    // texture stages through the thrust::device_vector overloads
    for (int k : {5, 9}) {
        thrust::device_vector<std::uint8_t> d_img(img.begin(), img.end());
        thrust::device_vector<float> d_mag(mag.begin(), mag.end()), d_blurred(3 * N), d_rtv(N);
        CudaBilateralTextureFilterImpl tf(W, H, k, 1);
        tf.compute_blur_and_rtv(d_img, d_mag, d_blurred, d_rtv);
        write_bin(out, (std::string("blurred_k") + std::to_string(k)).c_str(), to_host(d_blurred));
        write_bin(out, (std::string("rtv_k") + std::to_string(k)).c_str(), to_host(d_rtv));
        thrust::device_vector<float> d_b(blurred_in.begin(), blurred_in.end()), d_r(rtv_in.begin(), rtv_in.end());
        thrust::device_vector<std::uint8_t> d_g(3 * N);
        tf.compute_guide(d_b, d_r, d_g);
        write_bin(out, (std::string("guide_k") + std::to_string(k)).c_str(), to_host(d_g));
    }
    // cuda_gradient<uint8_t / float>, 1 and 3 channels, on DeviceImage buffers
    {
        DeviceImage<std::uint8_t> d_u1(W, H, 1), d_u3(W, H, 3);
        DeviceImage<float> d_f1(W, H, 1), d_f3(W, H, 3), d_dst(W, H, 1);
        d_u1.upload(gray.data());
        d_u3.upload(img.data());
        d_f1.upload(mag.data());
        d_f3.upload(blurred_in.data());
        std::vector<float> g(N);
        cuda_gradient(d_u1.get(), d_dst.get(), W, H, 1);
        d_dst.download(g.data());
        write_bin(out, "gradient_u8_c1", g);
        cuda_gradient(d_u3.get(), d_dst.get(), W, H, 3);
        d_dst.download(g.data());
        write_bin(out, "gradient_u8_c3", g);
        cuda_gradient(d_f1.get(), d_dst.get(), W, H, 1);
        d_dst.download(g.data());
        write_bin(out, "gradient_f32_c1", g);
        cuda_gradient(d_f3.get(), d_dst.get(), W, H, 3);
        d_dst.download(g.data());
        write_bin(out, "gradient_f32_c3", g);
    }
    // DeviceImage round trip and move semantics (the reference's copyable pimpl double-freed)
    {
        DeviceImage<float> a(W, H, 3);
        a.upload(blurred_in.data());
        DeviceImage<float> b(std::move(a));
        std::vector<float> back(3 * N);
        b.download(back.data());
        CHECK(back == blurred_in, "DeviceImage<float> upload/move/download round trip differs");
    }
    std::printf("dropin_test: %s (%d failures)\n", g_failures ? "FAILED" : "outputs written", g_failures);
    return g_failures ? 1 : 0;
}
