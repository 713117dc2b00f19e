// Image files for the sample drivers, without OpenCV: PNG (zlib) and binary PPM/PGM.
//
// The reference's samples load images with cv::imread(filename, cv::IMREAD_COLOR)
// (sample/bilateral_filter/main.cpp:20, sample/adaptive_bilateral_filter/main.cpp:20,
// sample/bilateral_texture_filter/main.cpp:19, sample/gradient/main.cpp:23) and hand
// the filters dense interleaved 8-bit BGR. read_image() returns exactly that layout
// with IMREAD_COLOR's conversions:
//   * RGB / RGBA          -> BGR, alpha dropped (not composited)
//   * gray / gray+alpha   -> B = G = R = gray
//   * palette             -> the palette colour (tRNS ignored: alpha is dropped)
//   * 16-bit samples      -> the high byte (libpng's strip_16, what imread does)
//   * 1/2/4-bit gray      -> scaled to 0..255 (libpng's expand_gray_1_2_4_to_8)
// PNG decoding covers every bit depth / colour type of the PNG specification, the five
// row filters and Adam7 interlacing; chunk CRCs are checked. write_image() writes
// 8-bit PNG (RGB or gray; per-row filter chosen by the minimum-sum-of-absolute-
// differences heuristic) or PPM/PGM, chosen by the file extension.
#pragma once

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace vip_io {

struct Image {
    int width = 0, height = 0, channels = 0;  // channels 3 (BGR) or 1 (gray)
    std::vector<std::uint8_t> data;           // dense, row stride width * channels
};

inline std::vector<std::uint8_t> read_file(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open " + path);
    std::vector<std::uint8_t> v;
    std::uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(f);
    return v;
}

inline void write_file(const std::string& path, const std::vector<std::uint8_t>& v) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot create " + path);
    const bool ok = std::fwrite(v.data(), 1, v.size(), f) == v.size();
    if (std::fclose(f) != 0 || !ok) throw std::runtime_error("cannot write " + path);
}

inline bool ends_with(const std::string& s, const char* suffix) {
    const size_t n = std::strlen(suffix);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suffix[i]) return false;
    return true;
}

// ---------------------------------------------------------------------------------
// PNG
// ---------------------------------------------------------------------------------
namespace png {

constexpr std::uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};

inline std::uint32_t be32(const std::uint8_t* p) {
    return (std::uint32_t)p[0] << 24 | (std::uint32_t)p[1] << 16 | (std::uint32_t)p[2] << 8 | p[3];
}

inline int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// Undo the row filters of one (sub)image in place: `raw` holds rows of 1 + rowbytes
// bytes (filter type, then the filtered bytes); `out` receives rows of rowbytes.
inline void unfilter(const std::uint8_t* raw, std::uint8_t* out, int rows, size_t rowbytes, int bpp) {
    std::vector<std::uint8_t> zero(rowbytes, 0);
    for (int y = 0; y < rows; ++y) {
        const std::uint8_t* in = raw + (size_t)y * (rowbytes + 1);
        const int ft = in[0];
        ++in;
        std::uint8_t* cur = out + (size_t)y * rowbytes;
        const std::uint8_t* prev = y ? out + (size_t)(y - 1) * rowbytes : zero.data();
        for (size_t i = 0; i < rowbytes; ++i) {
            const int a = i >= (size_t)bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= (size_t)bpp ? prev[i - bpp] : 0;
            int pred;
            switch (ft) {
                case 0: pred = 0; break;
                case 1: pred = a; break;
                case 2: pred = b; break;
                case 3: pred = (a + b) >> 1; break;
                case 4: pred = paeth(a, b, c); break;
                default: throw std::runtime_error("PNG: bad row filter type " + std::to_string(ft));
            }
            cur[i] = (std::uint8_t)(in[i] + pred);
        }
    }
}

inline Image decode(const std::vector<std::uint8_t>& f) {
    if (f.size() < 8 || std::memcmp(f.data(), kSig, 8) != 0) throw std::runtime_error("not a PNG file");
    size_t pos = 8;
    int W = 0, H = 0, depth = 0, ctype = -1, interlace = 0;
    std::vector<std::uint8_t> idat, plte;
    bool seen_end = false;
    while (pos + 12 <= f.size()) {
        const std::uint32_t len = be32(&f[pos]);
        if (len > f.size() - pos - 12) throw std::runtime_error("PNG: truncated chunk");
        const std::uint8_t* type = &f[pos + 4];
        const std::uint8_t* body = type + 4;
        if (crc32(crc32(0L, Z_NULL, 0), type, len + 4) != be32(body + len))
            throw std::runtime_error("PNG: chunk CRC mismatch");
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) throw std::runtime_error("PNG: bad IHDR");
            W = (int)be32(body);
            H = (int)be32(body + 4);
            depth = body[8];
            ctype = body[9];
            if (body[10] != 0 || body[11] != 0) throw std::runtime_error("PNG: unknown compression/filter method");
            interlace = body[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            seen_end = true;
            break;
        } else if (!(type[0] & 0x20)) {
            throw std::runtime_error("PNG: unknown critical chunk");
        }
        pos += 12 + len;
    }
    if (!seen_end || W <= 0 || H <= 0 || W > (1 << 24) || H > (1 << 24)) throw std::runtime_error("PNG: bad header");
    int spp;  // samples per pixel
    switch (ctype) {
        case 0: spp = 1; break;
        case 2: spp = 3; break;
        case 3: spp = 1; break;
        case 4: spp = 2; break;
        case 6: spp = 4; break;
        default: throw std::runtime_error("PNG: bad colour type");
    }
    const bool depth_ok = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                          (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                          ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
    if (!depth_ok || interlace > 1) throw std::runtime_error("PNG: unsupported bit depth / interlace");
    if (ctype == 3 && (plte.empty() || plte.size() % 3)) throw std::runtime_error("PNG: missing palette");
    const int bits = spp * depth;
    const int bpp = std::max(1, bits / 8);
    auto rowbytes = [&](int w) { return ((size_t)w * bits + 7) / 8; };

    // Adam7 passes (x0, y0, dx, dy); a non-interlaced image is the single pass (0, 0, 1, 1)
    static const int kAdam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                     {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    static const int kFlat[1][4] = {{0, 0, 1, 1}};
    const int npass = interlace ? 7 : 1;
    const int (*passes)[4] = interlace ? kAdam7 : kFlat;
    size_t total = 0;
    for (int p = 0; p < npass; ++p) {
        const int pw = (W - passes[p][0] + passes[p][2] - 1) / passes[p][2];
        const int ph = (H - passes[p][1] + passes[p][3] - 1) / passes[p][3];
        if (pw > 0 && ph > 0) total += (size_t)ph * (rowbytes(pw) + 1);
    }
    std::vector<std::uint8_t> raw(total);
    {
        z_stream zs{};
        if (inflateInit(&zs) != Z_OK) throw std::runtime_error("PNG: inflateInit failed");
        zs.next_in = idat.data();
        zs.avail_in = (uInt)idat.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        const int rc = inflate(&zs, Z_FINISH);
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if ((rc != Z_STREAM_END && rc != Z_BUF_ERROR) || got != raw.size())
            throw std::runtime_error("PNG: corrupt or short image data");
    }

    // samples of the whole image, 16-bit reduced to the high byte, sub-byte gray scaled
    std::vector<std::uint8_t> px((size_t)W * H * spp);
    std::vector<std::uint8_t> sub;
    size_t off = 0;
    for (int p = 0; p < npass; ++p) {
        const int x0 = passes[p][0], y0 = passes[p][1], dx = passes[p][2], dy = passes[p][3];
        const int pw = (W - x0 + dx - 1) / dx, ph = (H - y0 + dy - 1) / dy;
        if (pw <= 0 || ph <= 0) continue;
        const size_t rb = rowbytes(pw);
        sub.resize(rb * ph);
        unfilter(raw.data() + off, sub.data(), ph, rb, bpp);
        off += (size_t)ph * (rb + 1);
        for (int y = 0; y < ph; ++y) {
            const std::uint8_t* r = sub.data() + (size_t)y * rb;
            for (int x = 0; x < pw; ++x) {
                std::uint8_t* o = px.data() + ((size_t)(y0 + y * dy) * W + x0 + x * dx) * spp;
                for (int s = 0; s < spp; ++s) {
                    const size_t si = (size_t)x * spp + s;
                    int v;
                    if (depth == 16) {
                        v = r[2 * si];
                    } else if (depth == 8) {
                        v = r[si];
                    } else {
                        const size_t bit = si * depth;
                        v = (r[bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
                        if (ctype == 0) v = v * 255 / ((1 << depth) - 1);
                    }
                    o[s] = (std::uint8_t)v;
                }
            }
        }
    }

    Image img;
    img.width = W;
    img.height = H;
    img.channels = 3;
    img.data.resize((size_t)W * H * 3);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const std::uint8_t* s = px.data() + i * spp;
        std::uint8_t* d = img.data.data() + i * 3;
        if (ctype == 3) {
            if ((size_t)s[0] * 3 + 2 >= plte.size()) throw std::runtime_error("PNG: palette index out of range");
            const std::uint8_t* c = plte.data() + (size_t)s[0] * 3;
            d[0] = c[2], d[1] = c[1], d[2] = c[0];
        } else if (spp <= 2) {
            d[0] = d[1] = d[2] = s[0];
        } else {
            d[0] = s[2], d[1] = s[1], d[2] = s[0];
        }
    }
    return img;
}

inline void put32(std::vector<std::uint8_t>& v, std::uint32_t x) {
    v.push_back((std::uint8_t)(x >> 24));
    v.push_back((std::uint8_t)(x >> 16));
    v.push_back((std::uint8_t)(x >> 8));
    v.push_back((std::uint8_t)x);
}

inline void chunk(std::vector<std::uint8_t>& out, const char* type, const std::uint8_t* body, size_t len) {
    put32(out, (std::uint32_t)len);
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), body, body + len);
    put32(out, (std::uint32_t)crc32(crc32(0L, Z_NULL, 0), out.data() + at, (uInt)(len + 4)));
}

// 8-bit RGB (from BGR) or gray PNG, non-interlaced.
inline std::vector<std::uint8_t> encode(const Image& img) {
    const int C = img.channels;
    if (C != 1 && C != 3) throw std::runtime_error("PNG: 1 or 3 channels");
    const size_t rb = (size_t)img.width * C;
    std::vector<std::uint8_t> filt((rb + 1) * img.height);
    std::vector<std::uint8_t> row(rb), zero(rb, 0), cand(rb), best(rb);
    std::vector<std::uint8_t> prev_rgb(rb, 0);
    for (int y = 0; y < img.height; ++y) {
        const std::uint8_t* s = img.data.data() + (size_t)y * rb;
        for (int x = 0; x < img.width; ++x)
            for (int c = 0; c < C; ++c) row[(size_t)x * C + c] = s[(size_t)x * C + (C == 3 ? 2 - c : 0)];
        const std::uint8_t* prev = y ? prev_rgb.data() : zero.data();
        long best_cost = -1;
        int best_ft = 0;
        for (int ft = 0; ft < 5; ++ft) {
            long cost = 0;
            for (size_t i = 0; i < rb; ++i) {
                const int a = i >= (size_t)C ? row[i - C] : 0, b = prev[i], c = i >= (size_t)C ? prev[i - C] : 0;
                const int pred = ft == 0 ? 0 : ft == 1 ? a : ft == 2 ? b : ft == 3 ? (a + b) >> 1 : paeth(a, b, c);
                cand[i] = (std::uint8_t)(row[i] - pred);
                cost += cand[i] < 128 ? cand[i] : 256 - cand[i];
            }
            if (best_cost < 0 || cost < best_cost) {
                best_cost = cost;
                best_ft = ft;
                best.swap(cand);
            }
        }
        std::uint8_t* o = filt.data() + (size_t)y * (rb + 1);
        o[0] = (std::uint8_t)best_ft;
        std::memcpy(o + 1, best.data(), rb);
        prev_rgb.swap(row);
        row.resize(rb);
    }
    uLongf zlen = compressBound((uLong)filt.size());
    std::vector<std::uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, filt.data(), (uLong)filt.size(), 6) != Z_OK)
        throw std::runtime_error("PNG: compress failed");
    std::vector<std::uint8_t> out(kSig, kSig + 8);
    std::uint8_t ihdr[13];
    for (int i = 0; i < 4; ++i) {
        ihdr[i] = (std::uint8_t)(img.width >> (24 - 8 * i));
        ihdr[4 + i] = (std::uint8_t)(img.height >> (24 - 8 * i));
    }
    ihdr[8] = 8;
    ihdr[9] = C == 3 ? 2 : 0;
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    chunk(out, "IHDR", ihdr, 13);
    chunk(out, "IDAT", z.data(), zlen);
    chunk(out, "IEND", nullptr, 0);
    return out;
}

}  // namespace png

// ---------------------------------------------------------------------------------
// binary PPM (P6) / PGM (P5), maxval <= 65535 (16-bit samples keep the high byte)
// ---------------------------------------------------------------------------------
namespace pnm {

inline Image decode(const std::vector<std::uint8_t>& f) {
    if (f.size() < 2 || f[0] != 'P' || (f[1] != '5' && f[1] != '6')) throw std::runtime_error("not a P5/P6 file");
    size_t pos = 2;
    long vals[3];
    for (long& v : vals) {
        for (;;) {  // whitespace and comments
            while (pos < f.size() && std::isspace(f[pos])) ++pos;
            if (pos < f.size() && f[pos] == '#') {
                while (pos < f.size() && f[pos] != '\n') ++pos;
            } else {
                break;
            }
        }
        if (pos >= f.size() || !std::isdigit(f[pos])) throw std::runtime_error("PNM: bad header");
        v = 0;
        while (pos < f.size() && std::isdigit(f[pos]) && v < (1L << 30)) v = v * 10 + (f[pos++] - '0');
    }
    ++pos;  // the single whitespace byte before the raster
    const int C = f[1] == '6' ? 3 : 1;
    const long W = vals[0], H = vals[1], maxv = vals[2];
    if (W <= 0 || H <= 0 || W > (1 << 24) || H > (1 << 24) || maxv <= 0 || maxv > 65535)
        throw std::runtime_error("PNM: bad size");
    const int bytes = maxv > 255 ? 2 : 1;
    if (f.size() < pos + (size_t)W * H * C * bytes) throw std::runtime_error("PNM: truncated raster");
    Image img;
    img.width = (int)W;
    img.height = (int)H;
    img.channels = 3;
    img.data.resize((size_t)W * H * 3);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        std::uint8_t s[3];
        for (int c = 0; c < C; ++c) s[c] = f[pos + (i * C + c) * bytes];
        std::uint8_t* d = img.data.data() + i * 3;
        if (C == 1)
            d[0] = d[1] = d[2] = s[0];
        else
            d[0] = s[2], d[1] = s[1], d[2] = s[0];
    }
    return img;
}

inline std::vector<std::uint8_t> encode(const Image& img) {
    const int C = img.channels;
    const std::string hdr =
        std::string(C == 3 ? "P6\n" : "P5\n") + std::to_string(img.width) + " " + std::to_string(img.height) + "\n255\n";
    std::vector<std::uint8_t> out(hdr.begin(), hdr.end());
    const size_t n = (size_t)img.width * img.height;
    out.reserve(out.size() + n * C);
    for (size_t i = 0; i < n; ++i) {
        if (C == 1) {
            out.push_back(img.data[i]);
        } else {
            out.push_back(img.data[i * 3 + 2]);
            out.push_back(img.data[i * 3 + 1]);
            out.push_back(img.data[i * 3]);
        }
    }
    return out;
}

}  // namespace pnm

// BGR, like cv::imread(path, cv::IMREAD_COLOR); the format is taken from the file's
// signature, not its name.
inline Image read_image(const std::string& path) {
    const std::vector<std::uint8_t> f = read_file(path);
    if (f.size() >= 8 && std::memcmp(f.data(), png::kSig, 8) == 0) return png::decode(f);
    if (f.size() >= 2 && f[0] == 'P' && (f[1] == '5' || f[1] == '6')) return pnm::decode(f);
    throw std::runtime_error(path + ": not a PNG, PPM or PGM file");
}

// .png -> PNG, .ppm / .pgm / .pnm -> binary PNM; img is BGR (3 channels) or gray (1).
inline void write_image(const std::string& path, const Image& img) {
    if ((img.channels != 1 && img.channels != 3) || img.data.size() != (size_t)img.width * img.height * img.channels)
        throw std::runtime_error("write_image: bad image");
    if (ends_with(path, ".png")) {
        write_file(path, png::encode(img));
    } else if (ends_with(path, ".ppm") || ends_with(path, ".pgm") || ends_with(path, ".pnm")) {
        write_file(path, pnm::encode(img));
    } else {
        throw std::runtime_error(path + ": unknown image extension (.png, .ppm, .pgm)");
    }
}

}  // namespace vip_io
