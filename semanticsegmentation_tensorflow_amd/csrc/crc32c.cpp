// CRC-32C (Castagnoli) for TF tensor-bundle checkpoints (host code).
//
// tf.train.Saver's V2 format stores, per tensor, the masked CRC-32C of its
// bytes in the .index SSTable and checks it on restore; the SSTable blocks
// carry masked CRC-32C trailers too (LevelDB table format).  Slicing-by-8
// table implementation (reflected polynomial 0x82F63B78).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/segkern.h"

namespace {

struct Tables {
    uint32_t t[8][256];
    Tables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int j = 1; j < 8; ++j) t[j][i] = (t[j - 1][i] >> 8) ^ t[0][t[j - 1][i] & 0xFF];
    }
};

const Tables& tables() {
    static const Tables tb;
    return tb;
}

}  // namespace

extern "C" uint32_t seg_crc32c(const void* data, size_t n, uint32_t crc) {
    const Tables& tb = tables();
    const uint8_t* p = static_cast<const uint8_t*>(data);
    uint32_t c = ~crc;
    while (n && ((uintptr_t)p & 7)) {
        c = (c >> 8) ^ tb.t[0][(c ^ *p++) & 0xFF];
        --n;
    }
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        w ^= c;
        c = tb.t[7][w & 0xFF] ^ tb.t[6][(w >> 8) & 0xFF] ^ tb.t[5][(w >> 16) & 0xFF] ^ tb.t[4][(w >> 24) & 0xFF] ^
            tb.t[3][(w >> 32) & 0xFF] ^ tb.t[2][(w >> 40) & 0xFF] ^ tb.t[1][(w >> 48) & 0xFF] ^ tb.t[0][w >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ tb.t[0][(c ^ *p++) & 0xFF];
    return ~c;
}
