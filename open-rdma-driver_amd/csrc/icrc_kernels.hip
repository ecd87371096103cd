// icrc_kernels.hip — CDNA4 (gfx950) kernels of the ICRC engine.
//
// What is computed (bit-exact with the reference compute_icrc,
// blue-rdma-device/src/third_party/net/packet_processor.rs:275-301):
//
//   icrc(pkt, L) = CRC32_ISO_HDLC( FF x 8 ‖ mask(pkt[0..40)) ‖ pkt[40 .. L-4) )
//   mask: bytes 1, 8, 10, 11, 26, 27, 32 := 0xFF   (packet.rs:140-142, 443-498)
//
// Restated as a raw (init 0, no xorout) reflected CRC over the word stream
//   u_0 = FF FF FF FF,  u_k = masked pkt word k-1  (k = 1 .. N-1, N = 1 + (L-4)/4)
// because init 0xFFFFFFFF over a message that starts with FF x 4 cancels to zeros, and
// leading zero words do not move a raw CRC.  With M = "advance the state over 4 zero
// bytes" (a GF(2)-linear map):   S = XOR_k M^(N-k)(u_k),   icrc = ~S.
//
// Mapping (one wavefront per packet): the stream is END-aligned into rows of 64 words;
// lane l of row r holds word k = k0 + 64 r + l (k0 = N - 64 R <= 0, words k < 0 are the
// free leading zeros).  Each row is one coalesced 256-byte buffer_load_dword per lane.
// Lane l keeps a Horner accumulator over its word column,
//     acc_l <- M^64(acc_l) ^ u          (4 LDS table lookups: M^64 is byte-sliced)
// and at the end the packet state is   S = XOR_l M^(64-l)(acc_l)   — the per-lane
// multiplier depends only on the lane (the stream is end-aligned), applied with 8
// nibble lookups into per-lane tables, then an XOR reduction across the wavefront.
// No MFMA: this is GF(2) arithmetic; the bound is HBM bandwidth.
//
// LDS holds 160 KiB of tables (layout in icrc_internal.h): the bulk tables are replicated
// 32x so that lane l always reads bank (l & 31) — conflict-free ds_read_b32.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "icrc_device.h"
#include "icrc_internal.h"

namespace icrc {
namespace {
// ---- pipelined path -----------------------------------------------------------------------
// A wave walks its packets q = 0, 1, 2, ... (packet index first + q * tw) in sets of S
// packets processed together (S independent CRC chains for ILP); the loads of set t + D are
// issued before set t is processed (a D-deep register ring), so each wave keeps ~D*S packets
// (~4 KiB each) in flight against the ~3 us loaded HBM latency.
constexpr int kRows = 17;  // rows held in registers per packet: L <= 4352 (every MTU <= 4096)

struct SlotMeta {
    uint8_t *pkt;
    uint32_t L;
    int R;      // rows (regular packets)
    int k0;     // stream index of lane 0 in row 0
    int kind;   // 0 = no packet, 1 = regular (aligned, 44 <= L, R <= kRows), 2 = irregular
};

// Ragged batches: (offset, len) of 64 consecutive packets of this wave's chunk, one per lane
// (one coalesced load each), read back with v_readlane at a wave-uniform index.
struct MetaBlock {
    uint32_t off_lo, off_hi, len;  // per lane
    int block;                     // uniform
};

__device__ __forceinline__ uint64_t meta_off(const MetaBlock &mb, int l) {
    return static_cast<uint64_t>(readlane_u32(mb.off_lo, l)) | (static_cast<uint64_t>(readlane_u32(mb.off_hi, l)) << 32);
}

__device__ __forceinline__ void meta_fetch(const BatchParams &p, MetaBlock &mb, uint32_t lo, uint32_t hi,
                                           int block, uint32_t lane) {
    const uint32_t i = lo + static_cast<uint32_t>(block) * 64u + lane;
    uint64_t off = 0;
    uint32_t len = 0;
    if (i < hi) {
        off = p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride;
        len = p.len ? p.len[i] : p.ulen;
    }
    mb.off_lo = static_cast<uint32_t>(off);
    mb.off_hi = static_cast<uint32_t>(off >> 32);
    mb.len = len;
    mb.block = block;
}

// LONG: the long-packet half of a split batch — packets with L < p.split_len belong to the short-
// packet kernel and leave the slot empty (kind 0: no loads, no result).
template <bool LONG = false>
__device__ __forceinline__ void slot_meta(const BatchParams &p, MetaBlock &mb, bool ragged, uint32_t lo,
                                          uint32_t q, uint32_t nq, uint32_t lane, SlotMeta &m) {
    m.kind = 0;
    m.R = 0;
    m.k0 = 0;
    m.pkt = p.base;
    m.L = 0;
    if (q >= nq) return;
    uint64_t off;
    uint32_t L;
    if (ragged) {
        const int block = static_cast<int>(q >> 6);
        if (block != mb.block) meta_fetch(p, mb, lo, lo + nq, block, lane);
        const int l = static_cast<int>(q & 63u);
        off = meta_off(mb, l);
        L = readlane_u32(mb.len, l);
    } else {
        off = static_cast<uint64_t>(lo + q) * p.stride;
        L = p.ulen;
    }
    if (LONG && L < p.split_len) return;
    m.pkt = p.base + off;
    m.L = L;
    m.kind = 2;
    if (L >= ICRC_MIN_PACKET && ((reinterpret_cast<uintptr_t>(m.pkt) | static_cast<uintptr_t>(L)) & 3u) == 0) {
        const int N = 1 + static_cast<int>((L - 4u) >> 2);
        const int R = (N + 63) >> 6;
        if (R <= kRows) {
            m.kind = 1;
            m.R = R;
            m.k0 = N - 64 * R;
        }
    }
}

// Loads of one packet's rows; rows past the
// packet and every row of a non-regular slot read 0 through the descriptor's range check.
// ABL = mode | (cache policy << 2): mode 0 real, 1 loads only, 2 CRC only; policy = the aux
// operand of the row loads (0 default, 2 nt: read-once stream).
constexpr int abl_mode(int abl) { return abl & 3; }
constexpr int abl_aux(int abl) { return abl >> 2; }

template <int ABL>
__device__ __forceinline__ void slot_load(const SlotMeta &m, uint32_t lane, uint32_t (&u)[kRows]) {
    if constexpr (abl_mode(ABL) == 2) {
#pragma unroll
        for (int j = 0; j < kRows; ++j) u[j] = lane * 0x9E3779B9u + static_cast<uint32_t>(j) * 0x85EBCA6Bu;
        return;
    }
    constexpr int kAux = abl_aux(ABL);
    const int nrec = m.kind == 1 ? static_cast<int>(m.L - 4u) : 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(m.pkt, 0, nrec, 0x00020000);
    const uint32_t vbase = 4u * static_cast<uint32_t>(m.k0 - 1 + static_cast<int>(lane));
    // Always kRows loads, no branch: hipcc's static vmcnt accounting takes the minimum over
    // all paths, so a conditional load block anywhere in the ring turns the waits for the
    // current packet into vmcnt(0) and drains the prefetch of the next one.
#pragma unroll
    for (int j = 0; j < kRows; ++j)
        u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(vbase + 256u * j), 0, kAux);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// ---- receive parse (icrc_rx_parse_device) --------------------------------------------------
// `hdr` holds packet word w (bytes 4w .. 4w+3, LE, zero past L-4) in lane w for w < 18: the
// IPv4 + UDP + BTH + up to 32 bytes of extension headers.  Restates to_rdma_message
// (packet_processor.rs:18-71) on the UDP payload with the ICRC stripped; field getters
// packet.rs:57-98 (BTH), 173-183 (RETH), 222-232 (AETH), 249-251 (Immediate).  Lane k < 18
// stores dword k of the 72-byte icrc_rx_desc.
// Per-lane constants of the descriptor layout, set once per kernel (rx_lane_init): descriptor
// dword `lane` <- header word src (a big-endian field, byte-swapped), kept when its class is
// present.   dword: 0 va.lo  1 va.hi  2 sec.lo  3 sec.hi  7 rkey  8 dlen  9 sec rkey  10 sec dlen
//                   11 imm  12 dqpn  13 psn  14 aeth msn   <- header words 11 10 15 14 12 13 16 17
//                   14 8 9 10.   Classes: 1 RETH, 2 secondary RETH, 4 Imm, 8 AETH, 16 BTH.
__device__ __forceinline__ void rx_lane_init(LaneConsts &c, uint32_t lane) {
    uint32_t src = 0, cls = 0;
    src = lane == 0u ? 11u : src;
    src = lane == 1u ? 10u : src;
    src = lane == 2u ? 15u : src;
    src = lane == 3u ? 14u : src;
    src = lane == 7u ? 12u : src;
    src = lane == 8u ? 13u : src;
    src = lane == 9u ? 16u : src;
    src = lane == 10u ? 17u : src;
    src = lane == 11u ? 14u : src;
    src = lane == 12u ? 8u : src;
    src = lane == 13u ? 9u : src;
    src = lane == 14u ? 10u : src;
    cls = (lane <= 1u || lane == 7u || lane == 8u) ? 1u : cls;
    cls = (lane == 2u || lane == 3u || lane == 9u || lane == 10u) ? 2u : cls;
    cls = lane == 11u ? 4u : cls;
    cls = lane == 14u ? 8u : cls;
    cls = (lane == 12u || lane == 13u) ? 16u : cls;
    c.rx_src4 = src << 2;
    c.rx_cls = cls;
    c.rx_mask = (lane >= 12u && lane <= 14u) ? 0xFFFFFFu : 0xFFFFFFFFu;
}

// `hdr` holds packet word w (bytes 4w .. 4w+3, LE, zero past L-4) in lane w for w < 18: the
// IPv4 + UDP + BTH + up to 32 bytes of extension headers.  Restates to_rdma_message
// (packet_processor.rs:18-71) on the UDP payload with the ICRC stripped; field getters
// packet.rs:57-98 (BTH), 173-183 (RETH), 222-232 (AETH), 249-251 (Immediate).  Lane k < 18
// stores dword k of the 72-byte icrc_rx_desc.  The packet-wide fields are decoded on the
// scalar unit (three v_readlane), the per-lane ones take one ds_bpermute + v_perm + a class
// test, and the six computed dwords are selected into their lanes.
__device__ __forceinline__ void rx_store(icrc_rx_desc *rx, uint32_t i, uint32_t hdr, uint64_t off, uint32_t L,
                                         uint32_t icrc_ok, uint32_t lane, const LaneConsts &c) {
    const uint32_t w7 = readlane_u32(hdr, 7), w9 = readlane_u32(hdr, 9), w10 = readlane_u32(hdr, 10);
    const uint32_t op = w7 & 0x1Fu, tran = (w7 >> 5) & 7u, fl = (w7 >> 8) & 0xFFu, pad = (fl >> 5) & 3u;
    // header struct size per opcode (packet.rs:427-438): BthReth 28, +Imm 32, DoubleReth 44, Aeth 16
    const uint32_t hs = (op == 0x09u || op == 0x0Bu) ? 32u
                      : (op == 0x0Cu)                 ? 44u
                      : (op == 0x11u)                 ? 16u
                      : (op >= 0x06u && op <= 0x10u)  ? 28u
                                                      : 0u;
    const uint32_t status = (L < ICRC_MIN_PACKET)   ? ICRC_RX_TRUNCATED
                          : (hs == 0u)              ? ICRC_RX_INVALID_OPCODE
                          : (tran > 6u)             ? ICRC_RX_INVALID_TRANS_TYPE
                          : (L - 32u < hs + pad)    ? ICRC_RX_TRUNCATED  // buf_size = L - 28 - 4
                                                    : ICRC_RX_OK;
    const bool ack = hs == 16u;
    const bool ok = status == ICRC_RX_OK;
    const uint32_t flags = ((fl & 0x80u) ? ICRC_RX_SOLICITED : 0u) | ((w9 & 0x80u) ? ICRC_RX_ACK_REQ : 0u) |
                           (ack ? ICRC_RX_ACKNOWLEDGE : 0u) | (hs == 32u ? ICRC_RX_HAS_IMM : 0u) |
                           (hs == 44u ? ICRC_RX_HAS_SECONDARY_RETH : 0u);
    const uint32_t code = ack ? (w10 >> 5) & 3u : 0u, value = ack ? w10 & 0x1Fu : 0u;
    const uint64_t poff = off + 28u + hs;
    // present classes: General metadata has a RETH, Acknowledge an AETH; none on error
    const uint32_t en = ok ? ((ack ? 8u : 1u) | (hs == 44u ? 2u : 0u) | (hs == 32u ? 4u : 0u) | 16u) : 0u;

    const uint32_t g = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(c.rx_src4), static_cast<int>(hdr)));
    uint32_t v = __builtin_amdgcn_perm(g, g, 0x00010203u) & c.rx_mask;  // bswap32
    v = (c.rx_cls & en) ? v : 0u;
    auto put = [&](uint32_t x, uint32_t l) __attribute__((always_inline)) { v = lane == l ? x : v; };
    put(ok ? static_cast<uint32_t>(poff) : 0u, 4);
    put(ok ? static_cast<uint32_t>(poff >> 32) : 0u, 5);
    put(ok ? L - 32u - hs - pad : 0u, 6);
    put(ok ? (bswap16(w7 >> 16) | (op << 16) | (tran << 24)) : 0u, 15);
    put(ok ? (flags | (pad << 8) | (code << 16) | (value << 24)) : 0u, 16);
    put((icrc_ok & 0xFFu) | (status << 8), 17);
    if (lane < 18u) reinterpret_cast<uint32_t *>(rx + i)[lane] = v;
}

// Header words of a packet at any alignment, byte-wise (generic path).
__device__ __forceinline__ uint32_t rx_header_bytes(const uint8_t *pkt, uint32_t L, uint32_t lane) {
    uint32_t w = 0;
    if (lane < 18u && L >= 4u) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t o = 4u * lane + t;
            w |= (o < L - 4u ? static_cast<uint32_t>(pkt[o]) : 0u) << (8 * t);
        }
    }
    return w;
}

// PARSE: gather packet words 0..17 into lanes 0..17 from the first two rows as loaded (raw, before
// the ICRC masks): word w sits in row j, lane w + 1 - k0 - 64 j.
__device__ __forceinline__ uint32_t rx_gather_header(uint32_t row0, uint32_t row1, int k0, uint32_t lane) {
    const int s0 = static_cast<int>(lane) + 1 - k0;
    const int s1 = s0 - 64;
    const uint32_t v0 = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute((s0 & 63) << 2, static_cast<int>(row0)));
    const uint32_t v1 = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute((s1 & 63) << 2, static_cast<int>(row1)));
    return (s0 >= 0 && s0 < 64) ? v0 : ((s1 >= 0 && s1 < 64) ? v1 : 0u);
}

// Process one set of S packets (wave-local sequence numbers q0 .. q0+S-1); results go to
// the wave's result buffer.
// PARSE: 0 off; 1 receive parse (rx_store); 3 diagnostic: the raw header words stored, no decode.
template <int MODE, int S, int ABL, int PARSE = 0>
__device__ __forceinline__ void process_set(const BatchParams &p, const char *lds, const LaneConsts &c,
                                            uint32_t lane, const SlotMeta (&m)[S], uint32_t (&u)[S][kRows],
                                            uint32_t q0, ResultBuf &rb, uint32_t lo = 0) {
    int rmax = 0;
    bool same = true;  // every slot regular with the same row count (the common case)
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (m[s].kind == 1 && m[s].R > rmax) rmax = m[s].R;
        same = same && m[s].kind == 1 && m[s].R == m[0].R;
    }
    if (rmax > 0) {
        uint32_t acc[S];
        uint32_t hdr[S];  // PARSE: packet word w in lane w (w < 18), from rows 0 and 1 as loaded
        if constexpr (PARSE) {
#pragma unroll
            for (int s = 0; s < S; ++s) hdr[s] = rx_gather_header(u[s][0], u[s][1], m[s].k0, lane);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k = m[s].k0 + static_cast<int>(lane);
            acc[s] = u[s][0] | head_mask(k);
            u[s][1] |= head_mask(k + 64);
        }
        // One straight-line block per row for all S chains (the scheduler interleaves them).
        if (same && rmax == kRows) {  // full-MTU packets (4 KiB): no per-row guard branches
#pragma unroll
            for (int j = 1; j < kRows; ++j) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    if constexpr (abl_mode(ABL) == 1) acc[s] ^= u[s][j];
                    else acc[s] = step_m64(lds, acc[s], u[s][j], c);
                }
            }
        } else if (same) {
#pragma unroll
            for (int j = 1; j < kRows; ++j) {
                if (j < rmax) {
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        if constexpr (abl_mode(ABL) == 1) acc[s] ^= u[s][j];
                        else acc[s] = step_m64(lds, acc[s], u[s][j], c);
                    }
                }
            }
        } else {
            // a chain past its own last row keeps its value through a select
#pragma unroll
            for (int j = 1; j < kRows; ++j) {
                if (j < rmax) {
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        if constexpr (abl_mode(ABL) == 1) {
                            acc[s] ^= u[s][j];
                        } else {
                            const uint32_t t = step_m64(lds, acc[s], u[s][j], c);
                            acc[s] = (j < m[s].R) ? t : acc[s];
                        }
                    }
                }
            }
        }
        uint32_t fin[S];
#pragma unroll
        for (int s = 0; s < S; ++s) fin[s] = final_mul(lds, acc[s], c.fin);
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (m[s].kind == 1) {
                const uint32_t r = packet_result<MODE>(p, m[s].pkt, m[s].L - 4u, ~wave_xor(fin[s]), true, lane);
                rb_put(rb, q0 + s, r);
                if constexpr (PARSE == 3) {
                    if (lane < 18u) reinterpret_cast<uint32_t *>(p.rx + lo + q0 + s)[lane] = hdr[s] ^ r;
                } else if constexpr (PARSE) {
                    rx_store(p.rx, lo + q0 + s, hdr[s], static_cast<uint64_t>(m[s].pkt - p.base), m[s].L, r, lane, c);
                }
            }
    }
#pragma unroll
    for (int s = 0; s < S; ++s)
        if (m[s].kind == 2) {
            uint32_t hdr_slow = 0;
            if constexpr (PARSE) hdr_slow = rx_header_bytes(m[s].pkt, m[s].L, lane);  // before any trailer zeroing
            const uint32_t r = handle_packet<MODE>(p, m[s].pkt, m[s].L, lds, c, lane);
            rb_put(rb, q0 + s, r);
            if constexpr (PARSE)
                rx_store(p.rx, lo + q0 + s, hdr_slow, static_cast<uint64_t>(m[s].pkt - p.base), m[s].L, r, lane, c);
        }
}

// A wave owns the contiguous packet range [lo, lo + nq) and walks it in sets of S packets
// (S independent CRC chains for ILP); the loads of set t + D are issued before set t is
// processed (a D-deep register ring), keeping ~D*S packets in flight per wave against the
// ~3 us loaded HBM latency.  Results leave 64 at a time as coalesced stores.
template <int MODE, int S, int D, int ABL, int PARSE = 0, bool LONG = false>
__device__ __forceinline__ void run_pipelined(const BatchParams &p, const char *lds, const LaneConsts &c,
                                              uint32_t lane, uint32_t lo, uint32_t nq) {
    constexpr int B = D + 1;
    static_assert(64 % S == 0, "sets must not straddle a 64-packet result block");
    if (nq == 0) return;
    const uint32_t nsets = (nq + S - 1) / S;
    const bool ragged = p.off != nullptr || p.len != nullptr;
    MetaBlock mb;
    mb.block = -1;
    mb.off_lo = mb.off_hi = mb.len = 0;
    ResultBuf rb;
    rb.v = 0;
    rb.valid = 0;
    SlotMeta m[B][S];
    uint32_t u[B][S][kRows];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        if (static_cast<uint32_t>(d) < nsets) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                slot_meta<LONG>(p, mb, ragged, lo, d * S + s, nq, lane, m[d][s]);
                slot_load<ABL>(m[d][s], lane, u[d][s]);
            }
        }
    }
    for (uint32_t t = 0; t < nsets; t += B) {
        const bool cont = static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            constexpr int bp = (b + D) % B;
            const uint32_t ts = t + b;
            if (ts >= nsets) return false;
            const uint32_t tp = ts + D;
            // unconditional: past the end slot_meta yields kind 0 (zero-size descriptor)
#pragma unroll
            for (int s = 0; s < S; ++s) {
                slot_meta<LONG>(p, mb, ragged, lo, tp * S + s, nq, lane, m[bp][s]);
                slot_load<ABL>(m[bp][s], lane, u[bp][s]);
            }
            const uint32_t q0 = ts * S;
            process_set<MODE, S, ABL, PARSE>(p, lds, c, lane, m[b], u[b], q0, rb, lo);
            const uint32_t qn = q0 + S;  // next unprocessed
            if ((qn & 63u) == 0 || qn >= nq) rb_flush<MODE>(p, rb, lo + ((q0 >> 6) << 6), lane);
            return true;
        });
        if (!cont) return;
    }
}

// ---- long packets of a ragged batch (hybrid dispatch) ------------------------------------------
// The one-packet pipeline (S = 1, D-deep prefetch) over only the packets with L >= p.split_len;
// the quad kernel (icrc_quad.hip) takes the shorter ones, whose per-packet costs it divides by
// four.  Long packets stay here because one contiguous 256-byte row per wave instruction
// streams from HBM at ~6.2 TB/s, while four packets per instruction stop at ~4.5 TB/s
// (profiles/r01_membench.json, patterns D and E).  The walk skips short packets with the
// ballot of each 64-packet meta block; results are kept per block and stored 64 at a time.
template <int MODE, int D, int ABL>
__device__ __forceinline__ void run_pipelined_long(const BatchParams &p, const char *lds, const LaneConsts &c,
                                                   uint32_t lane, uint32_t lo, uint32_t nq) {
    constexpr int B = D + 1;
    if (nq == 0) return;
    MetaBlock mb;
    mb.block = -1;
    mb.off_lo = mb.off_hi = mb.len = 0;
    uint64_t lmask = 0;  // long packets of mb
    uint32_t qn = 0;     // next candidate (load side)
    ResultBuf rb;
    rb.v = 0;
    rb.valid = 0;
    int rb_block = -1;
    SlotMeta m[B][1];
    uint32_t qs[B];
    uint32_t u[B][1][kRows];
    int inflight = 0;

    auto next = [&](SlotMeta &sm, uint32_t &q) __attribute__((always_inline)) {
        sm.kind = 0;
        sm.R = 0;
        sm.k0 = 0;
        sm.pkt = p.base;
        sm.L = 0;
        q = 0xFFFFFFFFu;
        while (qn < nq) {
            const int blk = static_cast<int>(qn >> 6);
            if (blk != mb.block) {
                meta_fetch(p, mb, lo, lo + nq, blk, lane);
                lmask = __ballot(static_cast<uint32_t>(blk) * 64u + lane < nq && mb.len >= p.split_len);
            }
            const uint64_t mask = lmask & (~0ull << (qn & 63u));
            if (mask == 0) {
                qn = static_cast<uint32_t>(blk + 1) * 64u;
                continue;
            }
            const int l = __builtin_ctzll(mask);
            q = static_cast<uint32_t>(blk) * 64u + static_cast<uint32_t>(l);
            qn = q + 1u;
            const uint64_t off = meta_off(mb, l);
            const uint32_t L = readlane_u32(mb.len, l);
            sm.pkt = p.base + off;
            sm.L = L;
            sm.kind = 2;
            if (((reinterpret_cast<uintptr_t>(sm.pkt) | static_cast<uintptr_t>(L)) & 3u) == 0) {
                const int N = 1 + static_cast<int>((L - 4u) >> 2);
                const int R = (N + 63) >> 6;
                if (R <= kRows) {
                    sm.kind = 1;
                    sm.R = R;
                    sm.k0 = N - 64 * R;
                }
            }
            return;
        }
    };

#pragma unroll
    for (int d = 0; d < D; ++d) {
        next(m[d][0], qs[d]);
        slot_load<ABL>(m[d][0], lane, u[d][0]);
        if (m[d][0].kind) inflight += 1;
    }
    for (;;) {
        static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            constexpr int bp = (b + D) % B;
            next(m[bp][0], qs[bp]);
            slot_load<ABL>(m[bp][0], lane, u[bp][0]);
            if (m[bp][0].kind) inflight += 1;
            if (m[b][0].kind) {
                const int blk = static_cast<int>(qs[b] >> 6);
                if (blk != rb_block) {
                    if (rb.valid) rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
                    rb_block = blk;
                }
                process_set<MODE, 1, ABL>(p, lds, c, lane, m[b], u[b], qs[b], rb, lo);
                inflight -= 1;
            }
            return true;
        });
        if (qn >= nq && inflight == 0) break;
    }
    if (rb.valid) rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
}

// Default (COMPACT = false): per wave, the C1 pipeline (S = 2 chains, D = 1) over the wave's whole
// chunk with short packets left as empty slots when long packets are dense — on an all-long ragged
// batch it runs at the strided rate (1 Mi x 4156 B: 0.75 ms split vs 0.80-0.87 with the walker) —
// and the compacting S = 1 walker above when they are sparse (on a mixed-MTU batch the dense walk
// costs 1.32 ms against 0.49).  COMPACT = true: the walker always (A/B: variant 200 + q).
template <int MODE, bool COMPACT>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_long_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(p.table);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += kThreadsPerGroup) lds4[i] = src[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t tw = gridDim.x * kWavesPerGroup;
    const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
    const uint32_t chunk = wave_chunk(p.n, tw);
    const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
    if constexpr (COMPACT) {
        run_pipelined_long<MODE, 1, kStreamAux << 2>(p, lds, c, lane, lo, nq);
    } else {
        // Per wave, by the density of long packets in its first 64-packet block: dense (>= 3/4,
        // e.g. a 4 KiB WRITE stream) -> the C1 pipeline with short packets as empty slots; sparse
        // (a mixed-MTU batch: ~1.5 % long) -> the compacting walker, which visits long packets only.
        const uint32_t L0 = lane < nq ? (p.len ? p.len[lo + lane] : p.ulen) : 0u;
        const uint64_t lm = __ballot(lane < nq && L0 >= p.split_len);
        const uint32_t nb = nq < 64u ? nq : 64u;
        if (4u * static_cast<uint32_t>(__builtin_popcountll(lm)) >= 3u * nb)
            run_pipelined<MODE, 2, 1, kStreamAux << 2, 0, true>(p, lds, c, lane, lo, nq);
        else
            run_pipelined_long<MODE, 1, kStreamAux << 2>(p, lds, c, lane, lo, nq);
    }
}

// ---- row-stream path ------------------------------------------------------------------------
// A wave's chunk is one flat sequence of 256-byte rows (the sum of R over its regular packets,
// in packet order).  A ring of RD row loads stays in flight (RD * 256 B per wave); the
// process side consumes rows in the same order, restarting the Horner accumulator at each
// packet's first row and finalising at its last.  A short packet costs only its own rows,
// a long one needs no special path, and every ring load is unconditional (exact vmcnt
// accounting).  Misaligned packets and L % 4 != 0 are skipped by the stream and done by a
// tail loop; L < 44 packets are recorded as errors when the process cursor passes them.
struct RowCursor {  // wave-uniform
    uint32_t q;     // packet sequence number within the chunk
    int j;          // row within the packet
    int R;          // rows of the current packet (0 = past the end)
    int k0;
    uint8_t *pkt;
    uint32_t L;
};

// R >= 1: regular packet; 0: L < 44 (error); -1: irregular (generic path).
__device__ __forceinline__ int classify(const uint8_t *pkt, uint32_t L, int &k0) {
    if (L < ICRC_MIN_PACKET) return 0;
    if (((reinterpret_cast<uintptr_t>(pkt) | static_cast<uintptr_t>(L)) & 3u) != 0) return -1;
    const int N = 1 + static_cast<int>((L - 4u) >> 2);
    const int R = (N + 63) >> 6;
    k0 = N - 64 * R;
    return R;
}

__device__ __forceinline__ void meta_read(const MetaBlock &mb, uint32_t q, uint64_t &off, uint32_t &L) {
    const int l = static_cast<int>(q & 63u);
    off = meta_off(mb, l);
    L = readlane_u32(mb.len, l);
}

// Result buffer keyed by 64-packet block: switching block flushes the previous one.
template <int MODE>
__device__ __forceinline__ void rb_record(const BatchParams &p, ResultBuf &rb, int &rb_block, uint32_t lo,
                                          uint32_t q, uint32_t r, uint32_t lane) {
    const int blk = static_cast<int>(q >> 6);
    if (blk != rb_block) {
        if (rb.valid) rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
        rb_block = blk;
    }
    rb_put(rb, q, r);
}

template <int MODE, int RD, bool PARSE = false>
__device__ __forceinline__ void run_rowstream(const BatchParams &p, const char *lds, const LaneConsts &c,
                                              uint32_t lane, uint32_t lo, uint32_t nq) {
    if (nq == 0) return;
    const bool ragged = p.off != nullptr || p.len != nullptr;
    MetaBlock ml, mprev;  // load-side block and the one before it (the process side lags)
    ml.block = mprev.block = -1;
    ml.off_lo = ml.off_hi = ml.len = 0;
    mprev.off_lo = mprev.off_hi = mprev.len = 0;
    bool irregular = false;
    ResultBuf rb;
    rb.v = 0;
    rb.valid = 0;
    int rb_block = -1;

    auto meta_at = [&](uint32_t q, bool load_side, uint64_t &off, uint32_t &L) __attribute__((always_inline)) {
        if (!ragged) {
            off = static_cast<uint64_t>(lo + q) * p.stride;
            L = p.ulen;
            return;
        }
        const int blk = static_cast<int>(q >> 6);
        if (load_side) {
            if (blk != ml.block) {
                mprev = ml;
                meta_fetch(p, ml, lo, lo + nq, blk, lane);
            }
            meta_read(ml, q, off, L);
        } else if (blk == ml.block) {
            meta_read(ml, q, off, L);
        } else if (blk == mprev.block) {
            meta_read(mprev, q, off, L);
        } else {  // only after a long run of skipped packets
            MetaBlock t;
            meta_fetch(p, t, lo, lo + nq, blk, lane);
            meta_read(t, q, off, L);
        }
    };

    // Advance a cursor to the next packet that has rows.  The process side also records
    // L < 44 packets as errors and notes irregular ones for the tail loop.
    auto next_packet = [&](RowCursor &cur, bool load_side) __attribute__((always_inline)) {
        for (;;) {
            cur.q += 1u;
            if (cur.q >= nq) {
                cur.R = 0;
                cur.pkt = p.base;
                cur.L = 0;
                cur.k0 = 0;
                cur.j = 0;
                return;
            }
            uint64_t off;
            uint32_t L;
            meta_at(cur.q, load_side, off, L);
            uint8_t *pkt = p.base + off;
            int k0 = 0;
            const int R = classify(pkt, L, k0);
            if (R > 0) {
                cur.R = R;
                cur.k0 = k0;
                cur.pkt = pkt;
                cur.L = L;
                cur.j = 0;
                return;
            }
            if (!load_side) {
                if (R < 0) {
                    irregular = true;
                } else {
                    if (lane == 0 && p.nerr) atomicAdd(p.nerr, 1u);
                    rb_record<MODE>(p, rb, rb_block, lo, cur.q, MODE == kCompute ? 0u : ICRC_VERIFY_BADLEN, lane);
                    if constexpr (PARSE) rx_store(p.rx, lo + cur.q, 0u, off, L, ICRC_VERIFY_BADLEN, lane, c);
                }
            }
        }
    };

    RowCursor lc, pc;
    lc.q = pc.q = 0xFFFFFFFFu;
    next_packet(lc, true);
    next_packet(pc, false);

    // one row load per ring slot; past the end the descriptor has zero size (load -> 0)
    auto load_row = [&](uint32_t &dst) __attribute__((always_inline)) {
        const int nrec = lc.R > 0 ? static_cast<int>(lc.L - 4u) : 0;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(lc.pkt, 0, nrec, 0x00020000);
        const uint32_t voff = 4u * static_cast<uint32_t>(lc.k0 - 1 + static_cast<int>(lane)) + 256u * static_cast<uint32_t>(lc.j);
        dst = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(voff), 0, kStreamAux);
        if (lc.R > 0) {
            lc.j += 1;
            if (lc.j == lc.R) next_packet(lc, true);
        }
    };

    uint32_t ring[RD];
    static_for<RD>([&](auto ic) __attribute__((always_inline)) -> bool {
        load_row(ring[decltype(ic)::value]);
        return true;
    });

    uint32_t acc = 0;
    uint32_t hdr = 0;  // PARSE: packet word w in lane w (w < 18), gathered from rows 0 and 1
    while (pc.R > 0) {
        static_for<RD>([&](auto ic) __attribute__((always_inline)) -> bool {
            constexpr int i = decltype(ic)::value;
            if (pc.R == 0) return false;
            uint32_t u = ring[i];
            if constexpr (PARSE) {
                if (pc.j < 2) {
                    const int sl = static_cast<int>(lane) + 1 - pc.k0 - 64 * pc.j;  // lane holding word `lane`
                    const uint32_t v = static_cast<uint32_t>(
                        __builtin_amdgcn_ds_bpermute((sl & 63) << 2, static_cast<int>(u)));
                    hdr = (sl >= 0 && sl < 64) ? v : (pc.j == 0 ? 0u : hdr);
                }
            }
            if (pc.j < 2) u |= head_mask(pc.k0 + static_cast<int>(lane) + 64 * pc.j);
            if (pc.j == 0) acc = u;
            else acc = step_m64(lds, acc, u, c);
            pc.j += 1;
            if (pc.j == pc.R) {
                const uint32_t crc = ~wave_xor(final_mul(lds, acc, c.fin));
                const uint32_t r = packet_result<MODE>(p, pc.pkt, pc.L - 4u, crc, true, lane);
                rb_record<MODE>(p, rb, rb_block, lo, pc.q, r, lane);
                if constexpr (PARSE)
                    rx_store(p.rx, lo + pc.q, hdr, static_cast<uint64_t>(pc.pkt - p.base), pc.L, r, lane, c);
                next_packet(pc, false);
            }
            load_row(ring[i]);
            return true;
        });
    }
    if (rb.valid) rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);

    if (irregular) {  // misaligned packets / L % 4 != 0: the generic per-packet path
        MetaBlock t;
        t.block = -1;
        t.off_lo = t.off_hi = t.len = 0;
        for (uint32_t q = 0; q < nq; ++q) {
            uint64_t off;
            uint32_t L;
            if (!ragged) {
                off = static_cast<uint64_t>(lo + q) * p.stride;
                L = p.ulen;
            } else {
                const int blk = static_cast<int>(q >> 6);
                if (blk != t.block) meta_fetch(p, t, lo, lo + nq, blk, lane);
                meta_read(t, q, off, L);
            }
            uint8_t *pkt = p.base + off;
            int k0 = 0;
            if (classify(pkt, L, k0) < 0) {
                uint32_t hdr_slow = 0;
                if constexpr (PARSE) hdr_slow = rx_header_bytes(pkt, L, lane);  // before the trailer is zeroed
                const uint32_t r = handle_packet<MODE>(p, pkt, L, lds, c, lane);
                if (lane == 0) store_result<MODE>(p, lo + q, r);
                if constexpr (PARSE) rx_store(p.rx, lo + q, hdr_slow, off, L, r, lane, c);
            }
        }
    }
}

// Kernel variants (runtime-selected, identical results):
//   0            one packet per wave at a time, no pipelining, strided packet assignment
//   S, D, ABL    pipelined with S chains and a D-deep ring over a contiguous packet chunk per
//                wave; ABL = 0 (real), 1 (loads only, no CRC: a memory-pipeline bound),
//                2 (CRC only, no loads: a compute bound).
template <int MODE, int S, int D, int ABL>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_batch_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(p.table);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += kThreadsPerGroup) lds4[i] = src[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;

    const uint32_t tw = gridDim.x * kWavesPerGroup;
    const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
    if constexpr (S < 0) {
        const uint32_t chunk = wave_chunk(p.n, tw);
        const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
        if (lo64 >= p.n) return;
        const uint32_t lo = static_cast<uint32_t>(lo64);
        const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
        run_rowstream<MODE, -S>(p, lds, c, lane, lo, nq);
    } else if constexpr (S == 0) {
        for (uint32_t i = gw; i < p.n; i += tw) {
            const uint64_t off = p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride;
            const uint32_t L = p.len ? p.len[i] : p.ulen;
            const uint32_t r = handle_packet<MODE>(p, p.base + off, L, lds, c, lane);
            if (lane == 0) store_result<MODE>(p, i, r);
        }
    } else {
        // contiguous chunks, 64-packet aligned so result stores are whole blocks
        const uint32_t chunk = wave_chunk(p.n, tw);
        const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
        if (lo64 >= p.n) return;
        const uint32_t lo = static_cast<uint32_t>(lo64);
        const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
        run_pipelined<MODE, S, D, ABL>(p, lds, c, lane, lo, nq);
    }
}

// Receive: verify + strip + parse — the default pipelined path (variant 13) with the header
// words gathered from each packet's first two rows.
template <int S, int D, int PARSE = 1>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_rx_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(p.table);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += kThreadsPerGroup) lds4[i] = src[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    rx_lane_init(c, lane);
    const uint32_t tw = gridDim.x * kWavesPerGroup;
    const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
    const uint32_t chunk = wave_chunk(p.n, tw);
    const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
    run_pipelined<kVerify, S, D, kStreamAux << 2, PARSE>(p, lds, c, lane, lo, nq);
}

// ---- receive parse, pass 2 (icrc_rx_parse_device default) ----------------------------------
// Why two passes: on gfx950 VMEM loads and stores share vmcnt, and with both kinds in flight the
// compiler can only wait for zero — a 72-byte descriptor store per packet inside the CRC pipeline
// drains its prefetch every packet (the fused kernel: 0.84-0.92 ms on 1 Mi x 4156 B against 0.70
// for verify alone; storing the raw header words without any decode costs the same).  So pass 1 is
// the plain verify dispatch into the caller's ok array (or a stream-ordered scratch array), and
// this pass re-reads each packet's first 72 bytes (~2 % of the packet bytes) and
// writes the descriptors.  A wave takes 64 packets: header words are loaded three packets per
// instruction (18 lanes each, contiguous), transposed through LDS to lane = packet for the decode
// (to_rdma_message, packet_processor.rs:18-71, as rx_store), and transposed back so the 64
// descriptors (4608 contiguous bytes) leave as 18 coalesced dword stores.
constexpr uint32_t kRxStride = 19;  // LDS words per packet row (odd: conflict-free lane = packet reads)

__global__ __launch_bounds__(256) void icrc_rx_desc_kernel(BatchParams p) {
    __shared__ uint32_t sh_all[4 * 64 * kRxStride];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *sh = sh_all + wave * 64u * kRxStride;
    const uint32_t tw = gridDim.x * 4u;
    const uint32_t g = lane / 18u, w = lane - 18u * g;  // header-load layout: packet group, word
    for (uint32_t base = (blockIdx.x * 4u + wave) * 64u; base < p.n; base += tw * 64u) {
        const uint32_t i = base + lane;
        const bool in = i < p.n;
        const uint64_t off = in ? (p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride) : 0u;
        const uint32_t L = in ? (p.len ? p.len[i] : p.ulen) : 0u;
        const uint32_t okb = in ? p.ok[i] : 0u;  // from the verify pass
        const uint8_t *pkt = p.base + off;
        const bool fast = L >= ICRC_MIN_PACKET && ((reinterpret_cast<uintptr_t>(pkt) | static_cast<uintptr_t>(L)) & 3u) == 0;
        const uint32_t olo = static_cast<uint32_t>(off), ohi = static_cast<uint32_t>(off >> 32);
        const uint32_t lf = fast ? L : 0u;  // 0: not loaded here (short / irregular)
#pragma unroll
        for (uint32_t r = 0; r < 22; ++r) {  // 3 packets per round, 66 >= 64
            const uint32_t j = 3u * r + g;
            const int src = static_cast<int>((j & 63u) << 2);
            const uint32_t jl = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(lf)));
            const uint32_t jlo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(olo)));
            const uint32_t jhi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(ohi)));
            uint32_t v = 0u;
            if (g < 3u && j < 64u && 4u * w + 8u <= jl) {  // jl = 0 for packets not on this path
                const uint8_t *q = p.base + (static_cast<uint64_t>(jlo) | (static_cast<uint64_t>(jhi) << 32));
                v = reinterpret_cast<const uint32_t *>(q)[w];
            }
            if (g < 3u && j < 64u) sh[j * kRxStride + w] = v;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t h[18];
#pragma unroll
        for (uint32_t k = 0; k < 18; ++k) h[k] = sh[lane * kRxStride + k];
        if (!fast && L >= ICRC_MIN_PACKET) {  // misaligned or L % 4 != 0: byte-wise, this lane only
#pragma unroll
            for (uint32_t k = 0; k < 18; ++k) {
                uint32_t x = 0;
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) {
                    const uint32_t o = 4u * k + t;
                    x |= (o + 4u < L ? static_cast<uint32_t>(pkt[o]) : 0u) << (8u * t);
                }
                h[k] = x;
            }
        }
        const bool valid = L >= ICRC_MIN_PACKET;
        const uint32_t w7 = h[7], w9 = h[9], w10 = h[10];
        const uint32_t op = w7 & 0x1Fu, tran = (w7 >> 5) & 7u, fl = (w7 >> 8) & 0xFFu, pad = (fl >> 5) & 3u;
        // header struct size per opcode (packet.rs:427-438): BthReth 28, +Imm 32, DoubleReth 44, Aeth 16
        const uint32_t hs = (op == 0x09u || op == 0x0Bu) ? 32u
                          : (op == 0x0Cu)                 ? 44u
                          : (op == 0x11u)                 ? 16u
                          : (op >= 0x06u && op <= 0x10u)  ? 28u
                                                          : 0u;
        const uint32_t status = !valid                  ? ICRC_RX_TRUNCATED
                              : (hs == 0u)              ? ICRC_RX_INVALID_OPCODE
                              : (tran > 6u)             ? ICRC_RX_INVALID_TRANS_TYPE
                              : (L - 32u < hs + pad)    ? ICRC_RX_TRUNCATED  // buf_size = L - 28 - 4
                                                        : ICRC_RX_OK;
        const bool ack = hs == 16u;
        const bool ok = status == ICRC_RX_OK;
        const uint32_t flags = ((fl & 0x80u) ? ICRC_RX_SOLICITED : 0u) | ((w9 & 0x80u) ? ICRC_RX_ACK_REQ : 0u) |
                               (ack ? ICRC_RX_ACKNOWLEDGE : 0u) | (hs == 32u ? ICRC_RX_HAS_IMM : 0u) |
                               (hs == 44u ? ICRC_RX_HAS_SECONDARY_RETH : 0u);
        const uint32_t code = ack ? (w10 >> 5) & 3u : 0u, value = ack ? w10 & 0x1Fu : 0u;
        const uint64_t poff = off + 28u + hs;
        // present classes: General metadata has a RETH, Acknowledge an AETH; none on error
        const bool reth = ok && !ack, sec = ok && hs == 44u, imm = ok && hs == 32u, aeth = ok && ack;
        uint32_t v[18];
        v[0] = reth ? bswap32(h[11]) : 0u;  // RETH va (big-endian u64, bytes 40-47)
        v[1] = reth ? bswap32(h[10]) : 0u;
        v[2] = sec ? bswap32(h[15]) : 0u;   // secondary RETH va (bytes 56-63)
        v[3] = sec ? bswap32(h[14]) : 0u;
        v[4] = ok ? static_cast<uint32_t>(poff) : 0u;
        v[5] = ok ? static_cast<uint32_t>(poff >> 32) : 0u;
        v[6] = ok ? L - 32u - hs - pad : 0u;
        v[7] = reth ? bswap32(h[12]) : 0u;  // rkey, dlen
        v[8] = reth ? bswap32(h[13]) : 0u;
        v[9] = sec ? bswap32(h[16]) : 0u;
        v[10] = sec ? bswap32(h[17]) : 0u;
        v[11] = imm ? bswap32(h[14]) : 0u;
        v[12] = ok ? bswap32(h[8]) & 0xFFFFFFu : 0u;     // dqpn
        v[13] = ok ? bswap32(h[9]) & 0xFFFFFFu : 0u;     // psn
        v[14] = aeth ? bswap32(h[10]) & 0xFFFFFFu : 0u;  // AETH msn
        v[15] = ok ? (bswap16(w7 >> 16) | (op << 16) | (tran << 24)) : 0u;
        v[16] = ok ? (flags | (pad << 8) | (code << 16) | (value << 24)) : 0u;
        v[17] = (okb & 0xFFu) | (status << 8);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t k = 0; k < 18; ++k) sh[lane * kRxStride + k] = v[k];
        __builtin_amdgcn_wave_barrier();
        const uint32_t cnt = p.n - base < 64u ? p.n - base : 64u;
        uint32_t *dst = reinterpret_cast<uint32_t *>(p.rx + base);
#pragma unroll
        for (uint32_t t = 0; t < 18; ++t) {
            const uint32_t idx = t * 64u + lane, pk = idx / 18u, k = idx - 18u * pk;
            if (pk < cnt) dst[idx] = sh[pk * kRxStride + k];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- fused send packetizer (WRITE / READ RESPONSE messages) -----------------------------------
// One wavefront per packet, the same row-stream ring as above, but a "row" is built rather
// than read: header words come from the message descriptor (computed on the scalar unit,
// placed per lane by selects), payload words from the memory-region buffer (one coalesced
// buffer_load_dword per lane per row).  Each word is stored to the wire buffer and folded into
// the ICRC in the same step; the ICRC is the trailer.  Byte-identical to PacketWriter::write.

struct PacketHdr {  // wave-uniform; words are the LE u32 of header bytes 4w .. 4w+3
    uint32_t w[14];
};

// Segment s of a message (generate_segments_from_request + Write::handle / ReadResponse::handle)
struct SegInfo {
    uint32_t start, len, L, pad;
    uint64_t out;       // packet offset in d_wire
    uint64_t src;       // payload offset in d_src
    int R, k0;
};

struct MsgRegs {  // the 88-byte icrc_write_msg in scalar registers (uniform)
    uint32_t s[22];
    int idx;  // message index held, -1 = none
};

__device__ __forceinline__ uint32_t msg_u32(const MsgRegs &m, int dw) { return m.s[dw]; }
__device__ __forceinline__ uint64_t msg_u64(const MsgRegs &m, int dw) {
    return static_cast<uint64_t>(msg_u32(m, dw)) | (static_cast<uint64_t>(msg_u32(m, dw + 1)) << 32);
}
// icrc_write_msg dword offsets
enum : int {
    kMLocalVa = 0, kMRemoteVa = 2, kMPayloadOff = 4, kMOutOff = 6, kMTotal = 8, kMRethLen = 9, kMPmtu = 10,
    kMRkey = 11, kMDqpn = 12, kMPsn = 13, kMSrcIp = 14, kMDstIp = 15, kMFirst = 16, kMNpk = 17, kMSlot = 18,
    kMMsnId = 19, kMKind = 20, kMsgDwords = 22
};
static_assert(sizeof(icrc_write_msg) == 4 * kMsgDwords, "icrc_write_msg layout");

// Message descriptors are read with scalar loads (uniform index, constant address space): they
// count in lgkmcnt, so fetching one inside the row ring leaves the ring's vmcnt accounting exact
// (a vector load there made every wait vmcnt(0)).
using ConstU32 = const __attribute__((address_space(4))) uint32_t;

__device__ __forceinline__ uint32_t msg_first_packet(const icrc_write_msg *msgs, int idx) {
    return ((ConstU32 *)reinterpret_cast<uintptr_t>(msgs + idx))[16];  // icrc_write_msg::first_packet
}

__device__ __forceinline__ void msg_fetch(const icrc_write_msg *msgs, uint32_t nmsgs, int idx, MsgRegs &m,
                                          uint32_t lane) {
    (void)lane;
    m.idx = idx;
    if (static_cast<uint32_t>(idx) < nmsgs) {
        ConstU32 *w = (ConstU32 *)reinterpret_cast<uintptr_t>(msgs + idx);
#pragma unroll
        for (int i = 0; i < kMsgDwords; ++i) m.s[i] = w[i];
    } else {
#pragma unroll
        for (int i = 0; i < kMsgDwords; ++i) m.s[i] = 0u;
    }
}

__device__ __forceinline__ void seg_info(const MsgRegs &m, uint32_t s, SegInfo &g) {
    const uint32_t total = msg_u32(m, kMTotal), pmtu = msg_u32(m, kMPmtu);
    const bool by_remote = ((msg_u32(m, kMKind) >> 16) & ICRC_WRITE_SEG_BY_REMOTE_VA) != 0u;
    const uint32_t lva = by_remote ? msg_u32(m, kMRemoteVa) : msg_u32(m, kMLocalVa);  // low 32 bits (constant index: m stays in registers)
    uint32_t first = pmtu - lva % pmtu;
    first = total < first ? total : first;
    if (s == 0) {
        g.start = 0;
        g.len = first;
    } else {
        g.start = first + (s - 1) * pmtu;
        const uint32_t rem = total - g.start;
        g.len = rem < pmtu ? rem : pmtu;
    }
    g.pad = (4u - (g.len & 3u)) & 3u;
    g.L = 56u + g.len + g.pad + 4u;
    g.out = msg_u64(m, kMOutOff) + static_cast<uint64_t>(s) * msg_u32(m, kMSlot);
    g.src = msg_u64(m, kMPayloadOff) + g.start;
    const int N = 1 + static_cast<int>((g.L - 4u) >> 2);
    g.R = (N + 63) >> 6;
    g.k0 = N - 64 * g.R;
}


// IPv4 (write_ip_udp_header, packet_processor.rs:307-332) + UDP + BTH (set_from_common_meta,
// packet.rs:145-153 on a zeroed buffer) + RETH (197-201).
__device__ __forceinline__ void build_header(const MsgRegs &m, uint32_t s, const SegInfo &g, PacketHdr &h) {
    const uint32_t n = msg_u32(m, kMNpk);
    const uint32_t kind = msg_u32(m, kMKind) & 0xffu, tran = (msg_u32(m, kMKind) >> 8) & 0xffu;
    const bool only = n == 1u, last = s + 1u == n;
    uint32_t op;
    if (kind == 0u) op = only ? 0x0Au : (s == 0u ? 0x06u : (last ? 0x08u : 0x07u));
    else op = only ? 0x10u : (s == 0u ? 0x0Du : (last ? 0x0Fu : 0x0Eu));
    const uint32_t ack = (only || last) ? 1u : 0u;
    const uint32_t msn_id = msg_u32(m, kMMsnId), msn = msn_id & 0xffffu, ipid = msn_id >> 16;
    const uint32_t psn = (msg_u32(m, kMPsn) + s) & 0xffffffu;
    const uint64_t va = msg_u64(m, kMRemoteVa) + g.start;
    h.w[0] = 0x45u | (((g.L >> 8) & 0xffu) << 16) | ((g.L & 0xffu) << 24);
    h.w[1] = bswap16(ipid);
    h.w[2] = 0x1140u;  // TTL 64, protocol UDP, checksum 0
    h.w[3] = bswap32(msg_u32(m, kMSrcIp));
    h.w[4] = bswap32(msg_u32(m, kMDstIp));
    h.w[5] = bswap16(4791u) | (bswap16(4791u) << 16);
    h.w[6] = bswap16(g.L - 20u);
    h.w[7] = (((tran << 5) & 0xffu) | op) | ((g.pad << 5) << 8) | (bswap16(msn) << 16);
    h.w[8] = bswap32(msg_u32(m, kMDqpn) & 0xffffffu);
    h.w[9] = bswap32(psn) | (ack << 7);
    h.w[10] = bswap32(static_cast<uint32_t>(va >> 32));
    h.w[11] = bswap32(static_cast<uint32_t>(va));
    h.w[12] = bswap32(msg_u32(m, kMRkey));
    h.w[13] = bswap32(msg_u32(m, kMRethLen));
    if ((msg_u32(m, kMKind) >> 16) & ICRC_WRITE_FILL_IPV4_CSUM) {
        // RFC 791 one's-complement sum of the ten big-endian 16-bit header words
        const uint32_t src = msg_u32(m, kMSrcIp), dst = msg_u32(m, kMDstIp);
        uint32_t sum = 0x4500u + (g.L & 0xFFFFu) + ipid + 0x4011u + (src >> 16) + (src & 0xFFFFu) + (dst >> 16) +
                       (dst & 0xFFFFu);
        sum = (sum & 0xFFFFu) + (sum >> 16);
        sum = (sum & 0xFFFFu) + (sum >> 16);
        h.w[2] |= bswap16(~sum & 0xFFFFu) << 16;
    }
}

__device__ __forceinline__ uint32_t header_word(const PacketHdr &h, int pw) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) v = (pw == i) ? h.w[i] : v;
    return v;
}

// Word pw of the packet for the byte-wise path: header, payload bytes from d_src, zero pad.
__device__ __forceinline__ uint32_t packet_word_bytes(const PacketHdr &h, const uint8_t *src, uint64_t src_bytes,
                                                      const SegInfo &g, int pw) {
    if (pw < 0) return 0u;
    if (pw < 14) return header_word(h, pw);
    uint32_t w = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint32_t q = 4u * static_cast<uint32_t>(pw) + t - 56u;
        const uint64_t a = g.src + q;
        const uint32_t b = (q < g.len && a < src_bytes) ? src[a] : 0u;
        w |= b << (8 * t);
    }
    return w;
}

template <int RD>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_packetize_kernel(const uint8_t *src, uint64_t src_bytes,
                                                                          const icrc_write_msg *msgs, uint32_t nmsgs,
                                                                          uint32_t npk, uint8_t *wire, uint64_t wire_bytes,
                                                                          uint32_t *pkt_len,
                                                                          uint32_t *icrc_out, const uint32_t *table) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    {
        const uint4 *t4 = reinterpret_cast<const uint4 *>(table);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += kThreadsPerGroup) lds4[i] = t4[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t tw = gridDim.x * kWavesPerGroup;
    const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
    const uint32_t chunk = wave_chunk(npk, tw);
    const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
    if (lo64 >= npk) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t hi = (npk - lo) < chunk ? npk : lo + chunk;

    // message holding packet lo: binary search on first_packet
    int mlo = 0, mhi = static_cast<int>(nmsgs) - 1;
    while (mlo < mhi) {
        const int mid = (mlo + mhi + 1) >> 1;
        if (msg_first_packet(msgs, mid) <= lo) mlo = mid;
        else mhi = mid - 1;
    }
    mlo = __builtin_amdgcn_readfirstlane(mlo);

    // cursors: packet index, its message (one dword per lane), segment, row
    struct Cur {
        uint32_t pk;
        MsgRegs m;
        SegInfo g;
        int j;
        bool fast, fits;
    };
    Cur lc, pc;
    // cur.fits: the packet has a message, a non-zero pmtu, its payload inside d_src and its slot
    // inside d_wire; cur.fast: it fits and both payload and slot are 4-byte aligned.
    auto locate = [&](Cur &cur, uint32_t pk) __attribute__((always_inline)) {
        cur.pk = pk;
        cur.j = 0;
        cur.fast = cur.fits = false;
        cur.g.R = 0;
        cur.g.L = 0;
        cur.g.k0 = 0;
        cur.g.src = 0;
        cur.g.out = 0;
        cur.g.len = 0;
        if (pk >= hi) return;
        while (cur.m.idx < static_cast<int>(nmsgs) &&
               (cur.m.idx < 0 || pk >= msg_u32(cur.m, kMFirst) + msg_u32(cur.m, kMNpk))) {
            const int next = cur.m.idx < 0 ? mlo : cur.m.idx + 1;
            msg_fetch(msgs, nmsgs, next, cur.m, lane);
        }
        if (cur.m.idx >= static_cast<int>(nmsgs) || pk < msg_u32(cur.m, kMFirst) || msg_u32(cur.m, kMPmtu) == 0u)
            return;
        SegInfo g;
        seg_info(cur.m, pk - msg_u32(cur.m, kMFirst), g);
        cur.fits = g.len <= src_bytes && g.src <= src_bytes - g.len && g.L <= wire_bytes &&
                   g.out <= wire_bytes - g.L && g.len <= 0x10000u;
        if (!cur.fits) return;
        cur.fast = ((reinterpret_cast<uintptr_t>(src) + g.src) & 3u) == 0 &&
                   ((reinterpret_cast<uintptr_t>(wire) + g.out) & 3u) == 0;
        cur.g = g;
    };
    auto advance = [&](Cur &cur) __attribute__((always_inline)) {  // next packet taking the fast path
        uint32_t pk = cur.pk + 1u;
        for (;;) {
            locate(cur, pk);
            if (pk >= hi || cur.fast) return;
            ++pk;
        }
    };
    lc.m.idx = pc.m.idx = -1;
    bool slow_seen = false;
    locate(lc, lo);
    if (!lc.fast) advance(lc);
    locate(pc, lo);
    if (!pc.fast) {
        slow_seen = pc.pk < hi;
        advance(pc);
    }

    ResultBuf rb_len, rb_crc;
    rb_len.v = rb_crc.v = 0;
    rb_len.valid = rb_crc.valid = 0;
    int rb_block = -1;
    auto record = [&](uint32_t pk, uint32_t L, uint32_t crc) __attribute__((always_inline)) {
        const int blk = static_cast<int>(pk >> 6);
        if (blk != rb_block) {
            if (rb_len.valid) {
                const uint32_t base = static_cast<uint32_t>(rb_block) * 64u + lane;
                if ((rb_len.valid >> lane) & 1ull) {
                    if (pkt_len) pkt_len[base] = rb_len.v;
                    if (icrc_out) icrc_out[base] = rb_crc.v;
                }
                rb_len.valid = rb_crc.valid = 0;
            }
            rb_block = blk;
        }
        rb_put(rb_len, pk, L);
        rb_put(rb_crc, pk, crc);
    };

    auto load_row = [&](uint32_t &dst) __attribute__((always_inline)) {
        const int nrec = lc.g.R > 0 ? static_cast<int>((lc.g.len + 3u) & ~3u) : 0;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(src) + (lc.g.R > 0 ? lc.g.src : 0), 0, nrec, 0x00020000);
        // payload byte offset of this lane's word: 4 * pw - 56 (negative -> out of range -> 0)
        const uint32_t voff = 4u * static_cast<uint32_t>(lc.g.k0 - 1 + static_cast<int>(lane) + 64 * lc.j) - 56u;
        dst = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(voff), 0, 0);  // default policy: copies run ~6 % faster than nt (r01_membench_copy.json)
        if (lc.g.R > 0) {
            lc.j += 1;
            if (lc.j == lc.g.R) advance(lc);
        }
    };

    constexpr int kRD = RD;
    uint32_t ring[kRD];
    static_for<kRD>([&](auto ic) __attribute__((always_inline)) -> bool {
        load_row(ring[decltype(ic)::value]);
        return true;
    });
    PacketHdr h;
    uint32_t hvec = 0;  // header word w in lane w (w < 14), one ds_bpermute per header row
    auto spread_header = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 14; ++k) hvec = lane == static_cast<uint32_t>(k) ? h.w[k] : hvec;
    };
    if (pc.pk < hi) {
        build_header(pc.m, pc.pk - msg_u32(pc.m, kMFirst), pc.g, h);
        spread_header();
    }
    uint32_t acc = 0;
    while (pc.pk < hi) {
        static_for<kRD>([&](auto ic) __attribute__((always_inline)) -> bool {
            constexpr int i = decltype(ic)::value;
            if (pc.pk >= hi) return false;
            const int pw = pc.g.k0 - 1 + static_cast<int>(lane) + 64 * pc.j;
            uint32_t w = ring[i];
            // last payload word (only in the packet's last row): keep only the payload bytes
            if (pc.j == pc.g.R - 1) {
                const int room = static_cast<int>(56u + pc.g.len) - 4 * pw;  // payload bytes from this word on
                if (room < 4) w = room <= 0 ? 0u : (w & ((1u << (8 * room)) - 1u));
            }
            if (pc.j < 2) {  // header words: lane w of hvec holds header word w
                const uint32_t hw = static_cast<uint32_t>(
                    __builtin_amdgcn_ds_bpermute(static_cast<int>(static_cast<uint32_t>(pw) << 2), static_cast<int>(hvec)));
                w = (pw >= 0 && pw < 14) ? hw : w;
            }
            const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(wire + pc.g.out, 0,
                                                                                static_cast<int>(pc.g.L - 4u), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(w, os, static_cast<int>(4u * static_cast<uint32_t>(pw)), 0, 0);
            uint32_t u = w;
            if (pc.j < 2) u |= head_mask(pw + 1);
            if (pc.j == 0) acc = u;
            else acc = step_m64(lds, acc, u, c);
            pc.j += 1;
            if (pc.j == pc.g.R) {
                const uint32_t crc = ~wave_xor(final_mul(lds, acc, c.fin));
                if (lane == 0) *reinterpret_cast<uint32_t *>(wire + pc.g.out + pc.g.L - 4u) = crc;
                record(pc.pk, pc.g.L, crc);
                const uint32_t before = pc.pk;
                advance(pc);
                if (pc.pk != before + 1u && before + 1u < hi) slow_seen = true;
                if (pc.pk < hi) {
                    build_header(pc.m, pc.pk - msg_u32(pc.m, kMFirst), pc.g, h);
                    spread_header();
                }
            }
            load_row(ring[i]);
            return true;
        });
    }
    if (rb_len.valid && (rb_len.valid >> lane) & 1ull) {
        const uint32_t base = static_cast<uint32_t>(rb_block) * 64u + lane;
        if (pkt_len) pkt_len[base] = rb_len.v;
        if (icrc_out) icrc_out[base] = rb_crc.v;
    }

    // Byte-wise path for packets whose payload or slot is not 4-byte aligned; packets that do not
    // fit (no message, payload outside d_src, slot outside d_wire) report length 0.
    if (slow_seen) {
        Cur sc;
        sc.m.idx = -1;
        for (uint32_t pk = lo; pk < hi; ++pk) {
            locate(sc, pk);
            if (sc.fast) continue;
            if (!sc.fits) {
                if (lane == 0) {
                    if (pkt_len) pkt_len[pk] = 0u;
                    if (icrc_out) icrc_out[pk] = 0u;
                }
                continue;
            }
            PacketHdr hs;
            build_header(sc.m, pk - msg_u32(sc.m, kMFirst), sc.g, hs);
            uint8_t *out = wire + sc.g.out;
            uint32_t a = 0;
            for (int r = 0; r < sc.g.R; ++r) {
                const int pw = sc.g.k0 - 1 + static_cast<int>(lane) + 64 * r;
                const uint32_t w = packet_word_bytes(hs, src, src_bytes, sc.g, pw);
                if (pw >= 0 && static_cast<uint32_t>(4 * pw) < sc.g.L - 4u) {
                    out[4 * pw] = static_cast<uint8_t>(w);
                    out[4 * pw + 1] = static_cast<uint8_t>(w >> 8);
                    out[4 * pw + 2] = static_cast<uint8_t>(w >> 16);
                    out[4 * pw + 3] = static_cast<uint8_t>(w >> 24);
                }
                uint32_t u = w;
                if (r < 2) u |= head_mask(pw + 1);
                a = (r == 0) ? u : step_m64(lds, a, u, c);
            }
            const uint32_t crc = ~wave_xor(final_mul(lds, a, c.fin));
            if (lane == 0) {
                uint8_t *t = out + sc.g.L - 4u;
                t[0] = static_cast<uint8_t>(crc);
                t[1] = static_cast<uint8_t>(crc >> 8);
                t[2] = static_cast<uint8_t>(crc >> 16);
                t[3] = static_cast<uint8_t>(crc >> 24);
                if (pkt_len) pkt_len[pk] = sc.g.L;
                if (icrc_out) icrc_out[pk] = crc;
            }
        }
    }
}

// ---- batched IPv4 header checksum (responser.rs:321-338) ---------------------------------------
// One thread per packet: 20 header bytes, ten big-endian words, end-around carry, complement.
__global__ __launch_bounds__(256) void icrc_ipv4_checksum_kernel(uint8_t *base, const uint64_t *off, uint64_t stride,
                                                                 uint32_t n, uint16_t *csum, int fill) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    uint8_t *h = base + (off ? off[i] : static_cast<uint64_t>(i) * stride);
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < 20; k += 2) {
        const uint32_t w = (static_cast<uint32_t>(h[k]) << 8) | h[k + 1];
        sum += (fill && k == 10) ? 0u : w;
    }
    while (sum >> 16) sum = (sum & 0xFFFFu) + (sum >> 16);
    const uint32_t c = ~sum & 0xFFFFu;
    if (fill) {
        h[10] = static_cast<uint8_t>(c >> 8);
        h[11] = static_cast<uint8_t>(c);
    }
    if (csum) csum[i] = static_cast<uint16_t>(c);
}

// ---- packet synthesis ----------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t synth_byte(const icrc_synth_desc &d, const uint8_t *hdr, uint32_t q) {
    if (q < d.hdr_len) return hdr[static_cast<uint64_t>(d.hdr_index) * 64u + q];
    const uint32_t pq = q - d.hdr_len;
    if (pq < d.payload_len) {
        const uint64_t pos = d.payload_pos + pq;
        return static_cast<uint32_t>(mix64(d.payload_key + (pos >> 3)) >> (8u * static_cast<uint32_t>(pos & 7u))) & 0xffu;
    }
    return 0u;
}

__global__ __launch_bounds__(256) void icrc_synth_kernel(uint8_t *base, const icrc_synth_desc *desc,
                                                          const uint8_t *hdr, uint32_t n) {
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const icrc_synth_desc d = desc[i];
        uint8_t *pkt = base + d.offset;
        const uint32_t nw = d.total_len >> 2;
        const bool aligned = ((reinterpret_cast<uintptr_t>(pkt) | d.payload_pos) & 3u) == 0;
        for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
            const uint32_t b0 = 4u * w;
            uint32_t val;
            if (aligned && b0 + 4u <= d.hdr_len) {
                val = *reinterpret_cast<const uint32_t *>(hdr + static_cast<uint64_t>(d.hdr_index) * 64u + b0);
            } else if (aligned && b0 >= d.hdr_len && b0 + 4u <= d.hdr_len + d.payload_len) {
                const uint64_t pos = d.payload_pos + (b0 - d.hdr_len);
                val = static_cast<uint32_t>(mix64(d.payload_key + (pos >> 3)) >> (8u * static_cast<uint32_t>(pos & 7u)));
            } else {
                val = synth_byte(d, hdr, b0) | (synth_byte(d, hdr, b0 + 1) << 8) |
                      (synth_byte(d, hdr, b0 + 2) << 16) | (synth_byte(d, hdr, b0 + 3) << 24);
            }
            if (aligned) {
                *reinterpret_cast<uint32_t *>(pkt + b0) = val;
            } else {
                pkt[b0] = static_cast<uint8_t>(val);
                pkt[b0 + 1] = static_cast<uint8_t>(val >> 8);
                pkt[b0 + 2] = static_cast<uint8_t>(val >> 16);
                pkt[b0 + 3] = static_cast<uint8_t>(val >> 24);
            }
        }
        for (uint32_t q = (nw << 2) + threadIdx.x; q < d.total_len; q += blockDim.x)
            pkt[q] = static_cast<uint8_t>(synth_byte(d, hdr, q));
    }
}

}  // namespace

#define ICRC_LAUNCH(S, D, A) \
    hipLaunchKernelGGL((icrc_batch_kernel<MODE, S, D, A>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p)
#define ICRC_QUAD(V) (void)launch_quad(MODE, V, p, grid, s)

template <int MODE>
static void launch_mode(const BatchParams &p, int grid, hipStream_t s) {
    switch (p.variant) {
    case 0: ICRC_LAUNCH(0, 1, 0); break;
    case 1: ICRC_LAUNCH(1, 1, 0); break;
    case 2: ICRC_LAUNCH(2, 1, 0); break;
    case 3: ICRC_LAUNCH(1, 2, 0); break;
    case 4: ICRC_LAUNCH(1, 3, 0); break;
    case 5: ICRC_LAUNCH(2, 2, 0); break;
    case 6: ICRC_LAUNCH(1, 2, 1); break;  // diagnostic: loads only
    case 7: ICRC_LAUNCH(1, 2, 2); break;  // diagnostic: CRC only
    case 8: ICRC_LAUNCH(2, 1, 2); break;  // diagnostic: CRC only, 2 chains
    case 9: ICRC_LAUNCH(2, 1, 1); break;  // diagnostic: loads only, 2 chains
    case 10: ICRC_LAUNCH(-16, 0, 0); break;  // row stream, 16 rows in flight per wave
    case 11: ICRC_LAUNCH(-24, 0, 0); break;  // row stream, 24 rows
    case 12: ICRC_LAUNCH(-32, 0, 0); break;  // row stream, 32 rows
    case 13: ICRC_LAUNCH(1, 1, 2 << 2); break;      // variant 1, nt row loads
    case 14: ICRC_LAUNCH(1, 2, 2 << 2); break;      // variant 3, nt row loads
    case 15: ICRC_LAUNCH(1, 2, 1 | (2 << 2)); break;  // diagnostic: loads only, nt
    case 16: ICRC_LAUNCH(2, 1, 2 << 2); break;      // variant 2, nt row loads
    case 17: ICRC_LAUNCH(1, 3, 2 << 2); break;      // variant 4, nt row loads
    case 18: ICRC_LAUNCH(1, 2, 2 | (2 << 2)); break;  // diagnostic: CRC only (same code shape as 15)
    case 19:  // four packets per wave (icrc_quad.hip): K rows per chunk, D chunks in flight
    case 20:
    case 21:
    case 22:  // diagnostic: quad kernel, loads only
    case 23:  // diagnostic: quad kernel, no loads
    case 24:  // eight packets per wave (W = 8)
    case 25:
    case 26:
    case 27:
    case 28:
    case 29:
    case 30:
    case 31:
    case 32:
    case 33:
    case 34:
    case 35:
    case 36:
    case 37:
    case 38: ICRC_QUAD(p.variant); break;
    default: ICRC_LAUNCH(1, 2, 0); break;
    }
}
#undef ICRC_LAUNCH
#undef ICRC_QUAD

int launch_long(int mode, const BatchParams &p, int grid, void *stream) {
    if (grid < 1) grid = 1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool compact = p.long_variant == 1;
    if (mode == kCompute) {
        if (compact) hipLaunchKernelGGL((icrc_long_kernel<kCompute, true>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
        else hipLaunchKernelGGL((icrc_long_kernel<kCompute, false>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    } else {
        if (compact) hipLaunchKernelGGL((icrc_long_kernel<kVerify, true>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
        else hipLaunchKernelGGL((icrc_long_kernel<kVerify, false>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    }
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_batch(int mode, const BatchParams &p, int grid, void *stream) {
    if (grid < 1) grid = 1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (mode == kCompute) launch_mode<kCompute>(p, grid, s);
    else launch_mode<kVerify>(p, grid, s);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_synth(uint8_t *base, const icrc_synth_desc *desc, const uint8_t *hdr, uint32_t n,
                 void *stream) {
    if (n == 0) return ICRC_OK;
    const uint32_t grid = n < 65536u ? n : 65536u;
    hipLaunchKernelGGL(icrc_synth_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       base, desc, hdr, n);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_rx(const BatchParams &p, int grid, void *stream) {
    if (p.n == 0) return ICRC_OK;
    if (grid < 1) grid = 1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (p.variant) {  // A/B: 1 (S = 2, D = 1), 2 (S = 1, D = 2), 3 diagnostic (raw header words)
    case 2: hipLaunchKernelGGL((icrc_rx_kernel<1, 2>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
    case 3: hipLaunchKernelGGL((icrc_rx_kernel<2, 1, 3>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
    default: hipLaunchKernelGGL((icrc_rx_kernel<2, 1>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
    }
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_rx_desc(const BatchParams &p, int num_cu, void *stream) {
    if (p.n == 0) return ICRC_OK;
    const uint64_t want = (static_cast<uint64_t>(p.n) + 255u) / 256u;
    const uint64_t cap = static_cast<uint64_t>(num_cu > 0 ? num_cu : 1) * 16u;  // 64 waves per CU
    const int grid = static_cast<int>(want < cap ? want : cap);
    hipLaunchKernelGGL(icrc_rx_desc_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_ipv4_checksum(uint8_t *base, const uint64_t *off, uint64_t stride, uint32_t n, uint16_t *csum, int fill,
                         void *stream) {
    if (n == 0) return ICRC_OK;
    hipLaunchKernelGGL(icrc_ipv4_checksum_kernel, dim3((n + 255u) / 256u), dim3(256), 0,
                       static_cast<hipStream_t>(stream), base, off, stride, n, csum, fill);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_packetize(const PacketizeParams &p, int grid, void *stream) {
    if (p.npackets == 0) return ICRC_OK;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((icrc_packetize_kernel<16>), dim3(grid), dim3(kThreadsPerGroup), 0,
                       static_cast<hipStream_t>(stream), p.src, p.src_bytes, p.msgs, p.nmsgs, p.npackets, p.wire,
                       p.wire_bytes, p.pkt_len, p.icrc, p.table);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc
