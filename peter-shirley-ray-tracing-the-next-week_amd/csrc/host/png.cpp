// png.cpp — PNG reader for image_texture assets (the reference loads them with the
// vendored stb_image, main.cpp:93: `stbi_load("picture.png", &nx, &ny, &nn, 0)`).
//
// Supports what the reference's asset path needs: 8-bit, non-interlaced, colour
// types gray / gray+alpha / RGB / RGBA / palette, all five scanline filters, and
// returns the channels as stored (req_comp == 0), like stbi_load.  Ancillary chunks
// (iCCP, pHYs, gAMA, ...) are ignored, as stb_image ignores them.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtnw.h"

namespace rtnw {

namespace {
uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}
}  // namespace

unsigned char *png_decode(const unsigned char *buf, size_t len, int *x, int *y, int *comp, std::string *err) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (len < 8 || std::memcmp(buf, sig, 8) != 0) { *err = "not a PNG"; return nullptr; }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, palette;
    size_t i = 8;
    while (i + 12 <= len) {
        const uint32_t n = be32(buf + i);
        const char *t = (const char *)buf + i + 4;
        const uint8_t *d = buf + i + 8;
        if (i + 12 + (size_t)n > len) { *err = "truncated chunk"; return nullptr; }
        if (!std::memcmp(t, "IHDR", 4)) {
            w = be32(d); h = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (!std::memcmp(t, "PLTE", 4)) {
            palette.assign(d, d + n);
        } else if (!std::memcmp(t, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + n);
        } else if (!std::memcmp(t, "IEND", 4)) {
            break;
        }
        i += 12 + n;
    }
    if (depth != 8 || interlace != 0 || w == 0 || h == 0) { *err = "only 8-bit non-interlaced PNG is supported"; return nullptr; }
    int ch;
    switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: *err = "bad PNG colour type"; return nullptr;
    }
    const size_t stride = (size_t)w * ch;
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK || rawlen != raw.size()) {
        *err = "PNG inflate failed";
        return nullptr;
    }
    std::vector<uint8_t> img(stride * h);
    for (uint32_t r = 0; r < h; r++) {
        const uint8_t f = raw[r * (stride + 1)];
        const uint8_t *src = &raw[r * (stride + 1) + 1];
        uint8_t *dst = &img[r * stride];
        const uint8_t *up = r ? &img[(r - 1) * stride] : nullptr;
        for (size_t k = 0; k < stride; k++) {
            const int a = k >= (size_t)ch ? dst[k - ch] : 0;
            const int b = up ? up[k] : 0;
            const int c = (up && k >= (size_t)ch) ? up[k - ch] : 0;
            int v = src[k];
            switch (f) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: *err = "bad PNG filter"; return nullptr;
            }
            dst[k] = (uint8_t)v;
        }
    }
    int out_ch = ch;
    if (ctype == 3) {   // palette -> RGB(A) as stb_image expands it
        out_ch = 3;
        std::vector<uint8_t> rgb((size_t)w * h * 3);
        for (size_t p = 0; p < (size_t)w * h; p++)
            for (int k = 0; k < 3; k++) rgb[3 * p + k] = 3 * (size_t)img[p] + k < palette.size() ? palette[3 * img[p] + k] : 0;
        img.swap(rgb);
    }
    unsigned char *out = (unsigned char *)std::malloc(img.size());
    std::memcpy(out, img.data(), img.size());
    *x = (int)w;
    *y = (int)h;
    *comp = out_ch;
    return out;
}

unsigned char *stbi_load(const char *filename, int *x, int *y, int *comp, int req_comp) {
    if (req_comp != 0) return nullptr;   // the reference only asks for the stored channels
    FILE *f = std::fopen(filename, "rb");
    if (!f) return nullptr;   // stbi_load returns NULL; the reference does not check (main.cpp:93)
    std::vector<unsigned char> buf;
    unsigned char tmp[65536];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    std::fclose(f);
    std::string err;
    return png_decode(buf.data(), buf.size(), x, y, comp, &err);
}

}  // namespace rtnw
