// Host PNG decoder for the KITTI loader (scipy.misc.imread of the
// reference's merge / gt_image_2 PNGs, Network/model/FCN.py:267-268).
// 8-bit greyscale / RGB / RGBA / grey+alpha, non-interlaced: chunk walk,
// zlib inflate of the IDAT stream, per-row filter reversal (None, Sub, Up,
// Average, Paeth; PNG spec 9.2).  Called through ctypes, which releases the
// GIL, so loader threads decode in parallel (PIL's decoder holds it).
// Pixel values are fixed by the format: identical to PIL's for these files.
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include <vector>

#include "../../include/segkern.h"

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct Header {
    int w, h, channels, color_type;
};

int parse_header(const uint8_t* buf, size_t n, Header* hd) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (!buf || n < 33 || memcmp(buf, sig, 8) != 0) return SEG_EINVAL;
    if (be32(buf + 8) != 13 || memcmp(buf + 12, "IHDR", 4) != 0) return SEG_EINVAL;
    const uint8_t* d = buf + 16;
    const uint32_t w = be32(d), h = be32(d + 4);
    const int depth = d[8], ct = d[9], interlace = d[12];
    if (w == 0 || h == 0 || w > (1u << 16) || h > (1u << 16) || depth != 8 || interlace != 0 || d[10] != 0 || d[11] != 0)
        return SEG_EINVAL;
    int ch;
    switch (ct) {
        case 0: ch = 1; break;
        case 2: ch = 3; break;
        case 4: ch = 2; break;
        case 6: ch = 4; break;
        default: return SEG_EINVAL;   // palette images: caller decodes another way
    }
    hd->w = (int)w;
    hd->h = (int)h;
    hd->channels = ch;
    hd->color_type = ct;
    return SEG_OK;
}

inline uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return (uint8_t)(pb <= pc ? b : c);
}

}  // namespace

extern "C" int seg_png_info(const void* buf, size_t n, int* h, int* w, int* channels) {
    Header hd;
    const int st = parse_header(static_cast<const uint8_t*>(buf), n, &hd);
    if (st) return st;
    if (h) *h = hd.h;
    if (w) *w = hd.w;
    if (channels) *channels = hd.channels;
    return SEG_OK;
}

extern "C" int seg_png_decode(const void* buf_, size_t n, void* out_, size_t out_bytes) {
    const uint8_t* buf = static_cast<const uint8_t*>(buf_);
    uint8_t* out = static_cast<uint8_t*>(out_);
    Header hd;
    int st = parse_header(buf, n, &hd);
    if (st) return st;
    const size_t stride = (size_t)hd.w * hd.channels;
    if (!out || out_bytes < stride * hd.h) return SEG_EINVAL;

    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return SEG_EINVAL;
    std::vector<uint8_t> raw((stride + 1) * hd.h);
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    size_t pos = 8;
    bool done = false;
    int zr = Z_OK;
    while (pos + 12 <= n && !done) {
        const uint32_t len = be32(buf + pos);
        const uint8_t* type = buf + pos + 4;
        if (pos + 12 + (size_t)len > n) break;
        if (memcmp(type, "IDAT", 4) == 0) {
            zs.next_in = const_cast<uint8_t*>(buf + pos + 8);
            zs.avail_in = len;
            while (zs.avail_in > 0 && zs.avail_out > 0) {
                zr = inflate(&zs, Z_NO_FLUSH);
                if (zr == Z_STREAM_END) break;
                if (zr != Z_OK) break;
            }
            if (zr != Z_OK && zr != Z_STREAM_END) break;
        } else if (memcmp(type, "IEND", 4) == 0) {
            done = true;
        }
        pos += 12 + (size_t)len;
    }
    inflateEnd(&zs);
    if ((zr != Z_OK && zr != Z_STREAM_END) || zs.avail_out != 0) return SEG_EINVAL;

    const int bpp = hd.channels;
    for (int y = 0; y < hd.h; ++y) {
        const uint8_t* r = raw.data() + (size_t)y * (stride + 1);
        const uint8_t f = r[0];
        const uint8_t* s = r + 1;
        uint8_t* o = out + (size_t)y * stride;
        const uint8_t* up = y ? o - stride : nullptr;
        switch (f) {
            case 0: memcpy(o, s, stride); break;
            case 1:
                for (size_t i = 0; i < stride; ++i) o[i] = (uint8_t)(s[i] + (i >= (size_t)bpp ? o[i - bpp] : 0));
                break;
            case 2:
                for (size_t i = 0; i < stride; ++i) o[i] = (uint8_t)(s[i] + (up ? up[i] : 0));
                break;
            case 3:
                for (size_t i = 0; i < stride; ++i) {
                    const int a = i >= (size_t)bpp ? o[i - bpp] : 0, b = up ? up[i] : 0;
                    o[i] = (uint8_t)(s[i] + ((a + b) >> 1));
                }
                break;
            case 4:
                for (size_t i = 0; i < stride; ++i) {
                    const int a = i >= (size_t)bpp ? o[i - bpp] : 0, b = up ? up[i] : 0;
                    const int c = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
                    o[i] = (uint8_t)(s[i] + paeth(a, b, c));
                }
                break;
            default: return SEG_EINVAL;
        }
    }
    return SEG_OK;
}
