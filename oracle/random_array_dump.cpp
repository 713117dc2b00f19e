// TEST INFRASTRUCTURE ONLY. Driver that runs the reference's own input generator
// (test/random_array.hpp, included from /root/reference/test where it lies) and
// writes raw arrays, so tests/golden can pin the oracle's mt19937 restatement.
// usage: random_array_dump u8 <len> <max> | f32 <len> <max>   (binary on stdout)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "random_array.hpp"

int main(int argc, char** argv) {
    if (argc != 4) return 2;
    const std::size_t len = std::strtoull(argv[2], nullptr, 10);
    if (std::strcmp(argv[1], "u8") == 0) {
        const auto a = random_array<std::uint8_t>(len, (std::uint8_t)std::atoi(argv[3]));
        std::fwrite(a.get(), 1, len, stdout);
    } else {
        const auto a = random_array<float>(len, (float)std::atof(argv[3]));
        std::fwrite(a.get(), sizeof(float), len, stdout);
    }
    return 0;
}
