// image.hpp — RGB8 image output: PNG (zlib-compressed, as image::RgbImage::save does for
// "output.png", src/main.rs:66) and binary PPM (the CPU config's "PPM out").
#pragma once
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace rt_host {

inline void write_ppm(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgb) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open " + path);
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    const size_t n = (size_t)w * h * 3;
    const bool ok = std::fwrite(rgb, 1, n, f) == n;
    std::fclose(f);
    if (!ok) throw std::runtime_error("short write to " + path);
}

inline void write_png(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgb) {
    auto be32 = [](std::vector<uint8_t>& v, uint32_t x) {
        v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
    };
    auto chunk = [&](std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
        be32(out, (uint32_t)data.size());
        std::vector<uint8_t> td(type, type + 4);
        td.insert(td.end(), data.begin(), data.end());
        out.insert(out.end(), td.begin(), td.end());
        be32(out, (uint32_t)crc32(0L, td.data(), (uInt)td.size()));
    };
    std::vector<uint8_t> raw;   // filter byte 0 (None) + row
    raw.reserve((size_t)h * (3 * (size_t)w + 1));
    for (uint32_t y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb + (size_t)y * w * 3, rgb + (size_t)(y + 1) * w * 3);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) throw std::runtime_error("zlib failed");
    z.resize(zlen);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    be32(ihdr, w); be32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, truecolour RGB, deflate, adaptive filter, no interlace
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open " + path);
    const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    std::fclose(f);
    if (!ok) throw std::runtime_error("short write to " + path);
}

inline void save_image(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgb) {
    if (path.size() >= 4 && (path.compare(path.size() - 4, 4, ".ppm") == 0)) write_ppm(path, w, h, rgb);
    else write_png(path, w, h, rgb);
}

}  // namespace rt_host
