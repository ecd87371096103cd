// icrc_device.h — device helpers shared by the HIP kernels (icrc_kernels.hip, icrc_oct.hip).
// Included inside namespace icrc { namespace { ... } } of each translation unit.
#pragma once
#include <hip/hip_runtime.h>

#include "icrc_internal.h"

namespace icrc {
namespace {


constexpr int kGroup = 8;  // long-packet path: rows (256 B per wave each) loaded together

__device__ __forceinline__ uint32_t lds_at(const char *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

struct LaneConsts {
    // v_perm_b32 source: byte0 = this lane's bank slot (lane & 31) * 4 in the even tables,
    // byte1 = the same slot + 128 in the odd tables, byte2 = 0x01 (the second 64 KiB region).
    uint32_t pc;
    uint32_t fin;  // per-lane final-table base
    uint32_t rx_src4, rx_cls, rx_mask;  // receive-parse descriptor layout (rx_lane_init), rx kernel only
};

// Table addresses of the four state bytes, one v_perm_b32 each: byte b of s lands in
// address bits 8..15, the lane slot in bits 0..7, the region (b >> 1) in bit 16.
constexpr uint32_t kSel0 = 0x0C0C0400u;  // [slot,   s.b0, 0,    0]
constexpr uint32_t kSel1 = 0x0C0C0501u;  // [slot+128, s.b1, 0,  0]
constexpr uint32_t kSel2 = 0x0C020600u;  // [slot,   s.b2, 0x01, 0]
constexpr uint32_t kSel3 = 0x0C020701u;  // [slot+128, s.b3, 0x01, 0]

// Three-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// M^64(s) ^ u: four byte lookups; u is folded in with the first two reads (two v_bitop3).
__device__ __forceinline__ uint32_t step_m64(const char *lds, uint32_t s, uint32_t u, const LaneConsts &c) {
    const uint32_t r0 = lds_at(lds, __builtin_amdgcn_perm(s, c.pc, kSel0));
    const uint32_t r1 = lds_at(lds, __builtin_amdgcn_perm(s, c.pc, kSel1));
    const uint32_t r2 = lds_at(lds, __builtin_amdgcn_perm(s, c.pc, kSel2));
    const uint32_t r3 = lds_at(lds, __builtin_amdgcn_perm(s, c.pc, kSel3));
    return xor3(xor3(u, r0, r1), r2, r3);
}

// This wave's packets [lo, hi) of a workgroup range of 16 x chunk packets from g0: equal shares,
// or (skew != 0, chunk a multiple of 64) wave slot k takes 1 + skew (3 - 2 (k >> 2)) / 1024 of
// the average, in whole units of 8 << (skew >> 12) packets (a multiple of 8 dividing 64), the
// oldest waves of each SIMD the most (kWaveSkew, icrc_internal.h).
__device__ __forceinline__ void wave_range(uint64_t g0, uint32_t chunk, uint32_t wave, uint32_t skew, uint64_t &lo,
                                           uint64_t &hi) {
    const uint32_t unit = 8u << ((skew >> 12) & 3u);
    skew &= 0xFFFu;
    if (skew == 0u || chunk < 64u) {
        lo = g0 + static_cast<uint64_t>(wave) * chunk;
        hi = lo + chunk;
        return;
    }
    const uint64_t U = 16u * static_cast<uint64_t>(chunk) / unit;  // the workgroup's units
    auto start = [&](uint32_t k) __attribute__((always_inline)) -> uint64_t {
        const int f = static_cast<int>(k >> 2), r = static_cast<int>(k & 3u);
        const int64_t num = 1024 * static_cast<int64_t>(k) + static_cast<int64_t>(skew) * (4 * f * (4 - f) + r * (3 - 2 * f));
        return U * static_cast<uint64_t>(num) / (16u * 1024u);
    };
    lo = g0 + unit * start(wave);
    hi = g0 + unit * start(wave + 1u);
}

__device__ __forceinline__ uint32_t mul_m64(const char *lds, uint32_t s, const LaneConsts &c) {
    return step_m64(lds, s, 0u, c);
}

// (a << 8) | b in one VALU op.  hipcc splits bfe-then-shift into shift + and + add (3 ops);
// the asm keeps v_bfe_u32 + v_lshl_or_b32.
__device__ __forceinline__ uint32_t lshl8_or(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// M^(64-lane)(acc) via 8 nibble lookups into this lane's private tables.  fin (kFinalBase +
// lane * 4) has address bits 8..11 clear: the nibble goes there with one v_lshl_or_b32, and
// n * 4096 rides in the ds_read offset field (2 VALU per lookup).
__device__ __forceinline__ uint32_t final_mul(const char *lds, uint32_t acc, uint32_t fin) {
    uint32_t r[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) r[n] = lds_at(lds, lshl8_or(__builtin_amdgcn_ubfe(acc, 4 * n, 4), fin) + n * 4096u);
    return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// XOR over the 64 lanes with DPP (VALU, no LDS round trips): two quad permutes and two
// row rotations leave every lane of each 16-lane row holding the row's XOR; the four row
// values are combined on the scalar unit.  Returns a wave-uniform value.
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x124, 0xF, 0xF, true));  // row_ror:4
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x128, 0xF, 0xF, true));  // row_ror:8
    return __builtin_amdgcn_readlane(x, 0) ^ __builtin_amdgcn_readlane(x, 16) ^
           __builtin_amdgcn_readlane(x, 32) ^ __builtin_amdgcn_readlane(x, 48);
}

// Fast path (4-aligned packet, L % 4 == 0): OR-masks of the stream words that carry the
// FF prefix (k = 0) and the masked header bytes (packet.rs offsets 1, 8, 10-11, 26-27, 32).
// Branch-free: bit j of kMaskedBytes = stream byte j is forced to 0xFF (prefix bytes 0-3,
// packet bytes 1, 8, 10, 11, 26, 27, 32 -> stream bytes 5, 12, 14, 15, 30, 31, 36); the
// nibble of word k is widened to byte masks (bit t -> byte t) with one multiply.
// (Divergent compare chains here made hipcc fall back to s_waitcnt vmcnt(0), draining the
// prefetched loads of the next packet.)
__device__ __forceinline__ uint32_t head_mask(int k) {
    const uint32_t kk = static_cast<uint32_t>(k);  // k < 0 wraps large -> 0
    // nibble of word k (k = 0..15) from one 64-bit constant: no select chain (hipcc turned the
    // two-level select into divergent branches)
    uint32_t nib = static_cast<uint32_t>(0x00000010C000D02Full >> ((kk & 15u) * 4u)) & 15u;
    nib = kk < 16u ? nib : 0u;
    const uint32_t bits = (nib * 0x00204081u) & 0x01010101u;  // bit t -> byte t's low bit
    // byte selectors 0x0C / 0x0D of v_perm_b32 yield 0x00 / 0xFF (x 0xFF without v_mul_lo_u32,
    // which a shift-subtract gets folded back into)
    return __builtin_amdgcn_perm(0u, 0u, 0x0C0C0C0Cu | bits);
}

__device__ __forceinline__ uint32_t fast_packet_state(const char *lds, const uint8_t *pkt,
                                                      uint32_t Ld, const LaneConsts &c,
                                                      uint32_t lane) {
    const int N = 1 + static_cast<int>(Ld >> 2);
    const int R = (N + 63) >> 6;
    const int k0 = N - 64 * R;
    // Out-of-range words (k < 1, i.e. before the packet) read as 0 through the descriptor.
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(pkt), 0, static_cast<int>(Ld), 0x00020000);
    const uint32_t vbase = 4u * static_cast<uint32_t>(k0 - 1 + static_cast<int>(lane));
    uint32_t acc = 0;
    for (int g = 0; g < R; g += kGroup) {
        uint32_t u[kGroup];
#pragma unroll
        for (int j = 0; j < kGroup; ++j)
            u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(vbase + 256u * static_cast<uint32_t>(g + j)), 0, 0);
        if (g == 0) {
            const int k = k0 + static_cast<int>(lane);
            u[0] |= head_mask(k);
            u[1] |= head_mask(k + 64);
            acc = u[0];
#pragma unroll
            for (int j = 1; j < kGroup; ++j)
                if (j < R) acc = mul_m64(lds, acc, c) ^ u[j];
        } else {
#pragma unroll
            for (int j = 0; j < kGroup; ++j)
                if (g + j < R) acc = mul_m64(lds, acc, c) ^ u[j];
        }
    }
    return acc;
}

// Generic path: any alignment, any length >= 44.  The stream is front-padded with
// z = (-(4 + Ld)) mod 4 zero bytes (free leading zeros) so that it ends on a word.
__device__ __forceinline__ uint32_t slow_word(const uint8_t *pkt, int k, int z) {
    if (k < 0) return 0u;
    uint32_t w = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = 4 * k + t - z;  // index in FF x 4 ‖ masked packet
        uint32_t b;
        if (j < 0) {
            b = 0u;
        } else if (j < 4) {
            b = 0xffu;
        } else {
            const uint32_t o = static_cast<uint32_t>(j - 4);
            b = pkt[o];
            if (o == 1 || o == 8 || o == 10 || o == 11 || o == 26 || o == 27 || o == 32) b = 0xffu;
        }
        w |= b << (8 * t);
    }
    return w;
}

__device__ __forceinline__ uint32_t slow_packet_state(const char *lds, const uint8_t *pkt,
                                                      uint32_t Ld, const LaneConsts &c,
                                                      uint32_t lane) {
    const uint32_t T = 4u + Ld;
    const int z = static_cast<int>((4u - (T & 3u)) & 3u);
    const int N = static_cast<int>((T + static_cast<uint32_t>(z)) >> 2);
    const int R = (N + 63) >> 6;
    const int k0 = N - 64 * R;
    uint32_t acc = 0;
    for (int r = 0; r < R; ++r) {
        const uint32_t u = slow_word(pkt, k0 + 64 * r + static_cast<int>(lane), z);
        acc = (r == 0) ? u : (mul_m64(lds, acc, c) ^ u);
    }
    return acc;
}

// Epilogue of one packet: trailer handling (lane 0 stores) and the per-packet result —
// compute: the ICRC; verify: ICRC_VERIFY_OK / _MISMATCH.  The result is wave-uniform.
template <int MODE>
__device__ __forceinline__ uint32_t packet_result(const BatchParams &p, uint8_t *pkt, uint32_t Ld, uint32_t crc,
                                                  bool aligned, uint32_t lane) {
    uint8_t *tr = pkt + Ld;
    if (MODE == kCompute) {
        if (p.trailer && lane == 0) {
            if (aligned) {
                *reinterpret_cast<uint32_t *>(tr) = crc;
            } else {
                tr[0] = static_cast<uint8_t>(crc);
                tr[1] = static_cast<uint8_t>(crc >> 8);
                tr[2] = static_cast<uint8_t>(crc >> 16);
                tr[3] = static_cast<uint8_t>(crc >> 24);
            }
        }
        return crc;
    } else {
        uint32_t stored;  // every lane reads the same 4 bytes (one cache line)
        if (aligned) {
            stored = *reinterpret_cast<const uint32_t *>(tr);
        } else {
            stored = static_cast<uint32_t>(tr[0]) | (static_cast<uint32_t>(tr[1]) << 8) |
                     (static_cast<uint32_t>(tr[2]) << 16) | (static_cast<uint32_t>(tr[3]) << 24);
        }
        const uint32_t ok = __builtin_amdgcn_readfirstlane(stored == crc ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH);
        if (p.trailer && lane == 0) {  // is_icrc_valid zeroes the trailer (packet_processor.rs:350)
            if (aligned) {
                *reinterpret_cast<uint32_t *>(tr) = 0u;
            } else {
                tr[0] = tr[1] = tr[2] = tr[3] = 0;
            }
        }
        return ok;
    }
}

// One packet, any length/alignment, no pipelining (variant 0, and irregular packets).
// Returns the packet's result value (see packet_result; bad length -> 0 / ICRC_VERIFY_BADLEN).
template <int MODE>
__device__ __forceinline__ uint32_t handle_packet(const BatchParams &p, uint8_t *pkt, uint32_t L, const char *lds,
                                                  const LaneConsts &c, uint32_t lane) {
    if (L < ICRC_MIN_PACKET) {
        if (lane == 0 && p.nerr) atomicAdd(p.nerr, 1u);
        return MODE == kCompute ? 0u : ICRC_VERIFY_BADLEN;
    }
    const uint32_t Ld = L - 4u;
    const bool fast = ((reinterpret_cast<uintptr_t>(pkt) | static_cast<uintptr_t>(L)) & 3u) == 0;
    const uint32_t acc = fast ? fast_packet_state(lds, pkt, Ld, c, lane) : slow_packet_state(lds, pkt, Ld, c, lane);
    return packet_result<MODE>(p, pkt, Ld, ~wave_xor(final_mul(lds, acc, c.fin)), fast, lane);
}

// SYS: a system-scope store (written through to host memory, complete once acknowledged) — the
// ring's results, which the host reads as soon as the job's done word arrives.
template <int MODE, bool SYS = false>
__device__ __forceinline__ void store_result(const BatchParams &p, uint32_t i, uint32_t r) {
    if (MODE == kCompute) {
        if (SYS && p.out)
            __hip_atomic_store(p.out + i, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (p.out)
            p.out[i] = r;
    } else {
        if (p.ok) p.ok[i] = static_cast<uint8_t>(r);
    }
}

// Per-wave result buffer: result of packet q goes to lane (q & 63) of one VGPR; 64 results
// leave as one coalesced store (256 B of ICRCs or 64 B of ok bytes).
struct ResultBuf {
    uint32_t v;       // per lane
    uint64_t valid;   // uniform lane mask
};

__device__ __forceinline__ void rb_put(ResultBuf &rb, uint32_t q, uint32_t r) {
    rb.v = (__lane_id() == (q & 63u)) ? r : rb.v;
    rb.valid |= 1ull << (q & 63u);
}

template <int MODE, bool SYS = false>
__device__ __forceinline__ void rb_flush(const BatchParams &p, ResultBuf &rb, uint32_t base, uint32_t lane) {
    if ((rb.valid >> lane) & 1ull) store_result<MODE, SYS>(p, base + lane, rb.v);
    rb.valid = 0;
}


template <int V>
struct IntC {
    static constexpr int value = V;
};
// Compile-time unrolled loop: f(IntC<0>), f(IntC<1>), ... while f returns true.
template <int N, int I = 0, class F>
__device__ __forceinline__ bool static_for(F &&f) {
    if constexpr (I < N) {
        if (!f(IntC<I>{})) return false;
        return static_for<N, I + 1>(f);
    } else {
        return true;
    }
}

// Packets per wave (contiguous chunks): whole 64-packet blocks, so that results leave as whole
// 256-byte lines, unless the batch is too small to give every wave a block — then as few as one
// packet per wave, so that a small batch (a 16 MiB message: 4096 packets) still spreads over
// every wave of the grid.
__device__ __forceinline__ uint32_t wave_chunk(uint32_t n, uint32_t tw) {
    const uint32_t c = (n + tw - 1) / tw;
    return c > 32u ? (c + 63u) & ~63u : c;
}

// v_readlane as an unsigned value (the builtin returns int: widening it directly to 64 bits
// sign-extends offsets >= 2 GiB).
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
// ---- verify as a compute over the trailer -------------------------------------------------
// The ICRC is CRC-32/ISO-HDLC and the trailer holds it little-endian, so the ICRC computed over
// the packet WITH its trailer as the stream's last word is the CRC-32 residue 0x2144DF1C exactly
// when the trailer is right (is_icrc_valid, packet_processor.rs:341-353).  The pipelined kernels
// verify that way: the trailer is one more stream word of the rows they load anyway, instead of a
// load of its own.  Stream words: compute 1 + (L - 4) / 4 (the FF prefix word and the bytes
// before the trailer), verify one more.
constexpr uint32_t kIcrcResidue = 0x2144DF1Cu;
template <int MODE>
__device__ __forceinline__ uint32_t stream_words(uint32_t L) {
    return MODE == kVerify ? 1u + (L >> 2) : 1u + ((L - 4u) >> 2);
}

// ---- the table image into LDS ------------------------------------------------------------
// From its compact form (icrc_internal.h, stored after the full image): thread t of the
// 1024-thread workgroup reads bulk entry t = B_b[x] (b = t >> 8, x = t & 255) and writes its 32
// bank copies (128 contiguous bytes) as eight 16-byte stores, the k-th at chunk (k + x) & 7 so
// that neighbouring lanes write different banks; plus two 16-byte pieces of the final tables.
// table_fetch only issues the loads (a kernel can issue its first packet loads before it waits
// for them); table_store writes LDS and joins the workgroup barrier.
struct TableShare {
    uint32_t bulk;
    uint4 fin[2];
};
static_assert(kThreadsPerGroup == 1024 && (kLdsBytes - kFinalBase) == 2u * 16u * kThreadsPerGroup, "table share");
__device__ __forceinline__ void table_fetch(TableShare &t, const uint32_t *table) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(table + kLdsWords), 0,
                                                                        static_cast<int>(kCompactWords * 4u), 0x00020000);
    t.bulk = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(4u * threadIdx.x), 0, 0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(4096u + 16u * (threadIdx.x + k * 1024u)), 0, 0);
        t.fin[k] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}
__device__ __forceinline__ void table_store(const TableShare &t, uint4 *lds4) {
    const uint32_t b = threadIdx.x >> 8, x = threadIdx.x & 255u;
    const uint32_t row = ((b >> 1) * 65536u + x * 256u + (b & 1u) * 128u) / 16u;  // first uint4 of the 32 copies
    const uint4 v = make_uint4(t.bulk, t.bulk, t.bulk, t.bulk);
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) lds4[row + ((k + x) & 7u)] = v;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) lds4[kFinalBase / 16u + threadIdx.x + k * 1024u] = t.fin[k];
    __syncthreads();
}
__device__ __forceinline__ void table_fill(uint4 *lds4, const uint32_t *table) {
    TableShare t;
    table_fetch(t, table);
    table_store(t, lds4);
}

constexpr int kStreamAux = 2;  // nt: packets are read once (MI355X_MICROARCH.md nt-weights); +7 % on C1

// ---- helpers of the multi-packet-per-wave kernel (icrc_oct.hip) ----------------------------------
__device__ __forceinline__ uint32_t bperm(uint32_t src_lane, uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src_lane << 2), static_cast<int>(v)));
}

// XOR over each W-lane packet group (DPP quad_perm x2, then row_ror 4, 8 for W = 16 or
// row_half_mirror for W = 8): every lane gets its group's XOR.
template <int W>
__device__ __forceinline__ uint32_t group_xor(uint32_t x) {
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0xB1, 0xF, 0xF, true));
    x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x4E, 0xF, 0xF, true));
    if constexpr (W == 16) {
        x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x124, 0xF, 0xF, true));
        x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x128, 0xF, 0xF, true));
    } else {
        static_assert(W == 8, "packet groups of 8 or 16 lanes");
        x ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x141, 0xF, 0xF, true));
    }
    return x;
}

// Generic per-packet path on the W-lane tables (group 0 computes; wave-uniform result).
template <int MODE, int W>
__device__ __forceinline__ uint32_t group_slow_packet(const BatchParams &p, uint8_t *pkt, uint32_t L, const char *lds,
                                                     const LaneConsts &c, uint32_t lane) {
    if (L < ICRC_MIN_PACKET) {
        if (lane == 0 && p.nerr) atomicAdd(p.nerr, 1u);
        return MODE == kCompute ? 0u : ICRC_VERIFY_BADLEN;
    }
    const uint32_t Ld = L - 4u;
    const bool aligned = ((reinterpret_cast<uintptr_t>(pkt) | static_cast<uintptr_t>(L)) & 3u) == 0;
    const uint32_t T = 4u + Ld;
    const int z = static_cast<int>((4u - (T & 3u)) & 3u);
    const int N = static_cast<int>((T + static_cast<uint32_t>(z)) >> 2);
    const int R = (N + W - 1) / W;
    const int k0 = N - W * R;
    const int col = static_cast<int>(lane & (W - 1u));
    const bool g0 = lane < static_cast<uint32_t>(W);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(pkt, 0, aligned ? static_cast<int>(Ld) : 0, 0x00020000);
    uint32_t acc = 0;
    for (int r = 0; r < R; ++r) {
        const int k = k0 + W * r + col;
        uint32_t u;
        if (aligned) {
            u = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(4u * static_cast<uint32_t>(k - 1)), 0, 0);
            u |= head_mask(k);
        } else {
            u = g0 ? slow_word(pkt, k, z) : 0u;
        }
        u = g0 ? u : 0u;
        acc = step_m64(lds, acc, u, c);
    }
    const uint32_t crc = ~readlane_u32(group_xor<W>(final_mul(lds, acc, c.fin)), 0);
    return packet_result<MODE>(p, pkt, Ld, crc, aligned, lane);
}


}  // namespace
}  // namespace icrc
