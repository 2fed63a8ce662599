// image_io.cpp -- rt_write_image: the reference's output step (bmp.rs:8-19 saves the
// Color::as_u8 RGB8 buffer through the `image` crate; main.rs names the file
// "<unix seconds>.png").  PNG (stored deflate blocks), BMP (24-bit, bottom-up) or binary
// PPM by the file's extension.  Host code: no device involved.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rt_api.h"

namespace {

static bool write_bmp(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    uint32_t row = (w * 3 + 3) & ~3u;
    uint32_t size = 54 + row * h;
    uint8_t hdr[54] = {'B', 'M'};
    auto put32 = [&](int off, uint32_t v) {
        for (int i = 0; i < 4; i++) hdr[off + i] = (uint8_t)(v >> (8 * i));
    };
    put32(2, size);
    put32(10, 54);
    put32(14, 40);
    put32(18, w);
    put32(22, h);
    hdr[26] = 1;
    hdr[28] = 24;
    put32(34, row * h);
    std::fwrite(hdr, 1, 54, f);
    std::vector<uint8_t> line(row, 0);
    for (uint32_t y = 0; y < h; y++) {
        uint32_t v = h - 1 - y;  // bottom-up
        for (uint32_t u = 0; u < w; u++) {
            const uint8_t* p = &rgb[((size_t)v * w + u) * 3];
            line[u * 3 + 0] = p[2];
            line[u * 3 + 1] = p[1];
            line[u * 3 + 2] = p[0];
        }
        std::fwrite(line.data(), 1, row, f);
    }
    std::fclose(f);
    return true;
}

static bool write_ppm(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::fwrite(rgb.data(), 1, rgb.size(), f);
    std::fclose(f);
    return true;
}

// PNG, 8-bit RGB, zlib stream of stored (uncompressed) deflate blocks: what the
// reference's image crate writes for "<t>.png", minus the compression.
static uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t v = i;
            for (int k = 0; k < 8; k++) v = (v & 1) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
            table[i] = v;
        }
        init = true;
    }
    c = ~c;
    for (size_t i = 0; i < n; i++) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

static bool write_png(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
    std::vector<uint8_t> raw;  // filter byte 0 + scanline
    raw.reserve((size_t)h * (w * 3 + 1));
    for (uint32_t v = 0; v < h; v++) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb.begin() + (size_t)v * w * 3, rgb.begin() + (size_t)(v + 1) * w * 3);
    }
    std::vector<uint8_t> z = {0x78, 0x01};
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
        size_t len = std::min<size_t>(65535, raw.size() - off);
        bool last = off + len >= raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)len);
        z.push_back((uint8_t)(len >> 8));
        z.push_back((uint8_t)~len);
        z.push_back((uint8_t)(~len >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + len);
        if (last) break;
    }
    uint32_t a = 1, b = 0;  // Adler-32
    for (uint8_t x : raw) {
        a = (a + x) % 65521u;
        b = (b + a) % 65521u;
    }
    uint32_t adler = (b << 16) | a;
    for (int i = 3; i >= 0; i--) z.push_back((uint8_t)(adler >> (8 * i)));
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    auto be32 = [](uint8_t* p, uint32_t v) {
        for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (24 - 8 * i));
    };
    auto chunk = [&](const char* type, const uint8_t* data, size_t n) {
        std::vector<uint8_t> c(8 + n + 4);
        be32(c.data(), (uint32_t)n);
        std::memcpy(c.data() + 4, type, 4);
        if (n) std::memcpy(c.data() + 8, data, n);
        be32(c.data() + 8 + n, crc32(c.data() + 4, 4 + n));
        std::fwrite(c.data(), 1, c.size(), f);
    };
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::fwrite(sig, 1, 8, f);
    uint8_t ihdr[13];
    be32(ihdr, w);
    be32(ihdr + 4, h);
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 2;   // RGB
    ihdr[10] = 0;  // deflate
    ihdr[11] = 0;  // adaptive filtering (all rows filter 0)
    ihdr[12] = 0;  // no interlace
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), z.size());
    chunk("IEND", nullptr, 0);
    std::fclose(f);
    return true;
}

static bool save_any(const std::string& path, const std::vector<uint8_t>& rgb8, uint32_t w, uint32_t h) {
    auto ends = [&](const char* e) {
        size_t n = std::strlen(e);
        return path.size() > n && path.compare(path.size() - n, n, e) == 0;
    };
    if (ends(".ppm")) return write_ppm(path, rgb8, w, h);
    if (ends(".bmp")) return write_bmp(path, rgb8, w, h);
    return write_png(path, rgb8, w, h);
}

}  // namespace

extern "C" rt_status rt_write_image(const char* path, const uint8_t* rgb8, uint32_t x_res, uint32_t y_res) {
    if (!path || !rgb8 || x_res == 0 || y_res == 0) return RT_ERR_INVALID_ARG;
    std::vector<uint8_t> v(rgb8, rgb8 + (size_t)x_res * y_res * 3);
    return save_any(path, v, x_res, y_res) ? RT_OK : RT_ERR_INVALID_ARG;
}
