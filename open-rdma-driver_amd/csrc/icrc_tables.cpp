// icrc_tables.cpp — host construction of the 160 KiB LDS table image (layout: icrc_internal.h).
//
// All tables are GF(2)-linear maps of the reflected CRC-32 state (polynomial 0xEDB88320,
// the crc32fast / CRC-32/ISO-HDLC polynomial used by compute_icrc,
// packet_processor.rs:276): M = "advance the state over 4 zero bytes".
#include <cstring>

#include "icrc_internal.h"

namespace icrc {
namespace {

struct ByteTable {
    uint32_t t[256];
    ByteTable() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
            t[i] = c;
        }
    }
};

const ByteTable &byte_table() {
    static const ByteTable bt;
    return bt;
}

// Columns of M^e: col[b] = M^e(1 << b); M^e(v) = XOR of col[b] over set bits of v.
struct Matrix {
    uint32_t col[32];
    uint32_t apply(uint32_t v) const {
        uint32_t r = 0;
        for (int b = 0; b < 32; b++)
            if (v >> b & 1u) r ^= col[b];
        return r;
    }
};

Matrix matrix_pow(uint32_t e) {
    Matrix m;
    for (int b = 0; b < 32; b++) m.col[b] = advance_words(1u << b, e);
    return m;
}

}  // namespace

uint32_t advance_words(uint32_t state, uint32_t nwords) {
    const uint32_t *t = byte_table().t;
    for (uint32_t i = 0; i < 4u * nwords; i++) state = (state >> 8) ^ t[state & 0xffu];
    return state;
}

// Row width W words (64: one packet per wavefront; 8: eight packets per wavefront).
static void build_image(uint32_t *img, uint32_t W) {
    std::memset(img, 0, kLdsBytes);
    const Matrix mb = matrix_pow(W);
    for (uint32_t b = 0; b < 4; b++) {
        for (uint32_t x = 0; x < 256; x++) {
            const uint32_t v = mb.apply(x << (8 * b));
            for (uint32_t copy = 0; copy < 32; copy++) {
                const uint32_t addr = (b >> 1) * 65536u + x * 256u + (b & 1u) * 128u + copy * 4u;
                img[addr / 4] = v;
            }
        }
    }
    for (uint32_t lane = 0; lane < 64; lane++) {
        const Matrix mf = matrix_pow(W - (lane % W));
        for (uint32_t n = 0; n < 8; n++) {
            for (uint32_t v = 0; v < 16; v++) {
                const uint32_t addr = kFinalBase + (n * 16u + v) * 256u + lane * 4u;
                img[addr / 4] = mf.apply(v << (4 * n));
            }
        }
    }
}

void append_compact_image(uint32_t *img) {
    uint32_t *c = img + kLdsWords;
    for (uint32_t b = 0; b < 4; b++)
        for (uint32_t x = 0; x < 256; x++) c[b * 256u + x] = img[((b >> 1) * 65536u + x * 256u + (b & 1u) * 128u) / 4u];
    std::memcpy(c + 1024, img + kFinalBase / 4u, kLdsBytes - kFinalBase);
}

void build_table_image(uint32_t *img) { build_image(img, 64); }

void build_table_image_oct(uint32_t *img) { build_image(img, 8); }

}  // namespace icrc
