// icrc_long.h — the one-packet-per-wave pipeline (C1 and the long half of a ragged batch), shared
// by icrc_kernels.hip (the batch and long-packet kernels) and icrc_oct.hip (the fused hybrid
// kernel, whose long-packet workgroups run long_body).  The algorithm and the lane mapping are
// described at the top of icrc_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

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

// the packet at byte offset `off` of length L into slot m (kind 1 regular / 2 irregular; LONG:
// kind 0 for the short-packet kernel's packets)
template <int MODE, bool LONG>
__device__ __forceinline__ void slot_classify(const BatchParams &p, uint64_t off, uint32_t L, SlotMeta &m) {
    if (LONG && L < p.split_len) return;
    m.pkt = p.base + off;
    m.L = L;
    m.kind = 2;
    if (L >= ICRC_MIN_PACKET && ((reinterpret_cast<uintptr_t>(m.pkt) | static_cast<uintptr_t>(L)) & 3u) == 0) {
        const int N = static_cast<int>(stream_words<MODE>(L));
        const int R = (N + 63) >> 6;
        if (R <= kRows) {
            m.kind = 1;
            m.R = R;
            m.k0 = N - 64 * R;
        }
    }
}

// LONG: the long-packet half of a split batch — packets with L < p.split_len belong to the short-
// packet kernel and leave the slot empty (kind 0: no loads, no result).
template <int MODE, bool LONG = false>
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
    slot_classify<MODE, LONG>(p, off, L, m);
}

// Loads of one packet's rows; rows past the
// packet and every row of a non-regular slot read 0 through the descriptor's range check.
// The ring's policy: the cache policy of its row loads (the aux operand: 0 default, 2 nt, a
// read-once stream) and whether the wave raises its priority around a load burst.  The product
// runs Ring<kStreamAux> (and Ring<kStreamAux, false>, A/B variant 17).  The A/B library also
// instantiates RingAblation<...> (ICRC_AB_BUILD), which switch a part off so that its cost can be
// measured on the same build (results wrong by design).
template <int AUX, bool PRIO = true>
struct Ring {
    static constexpr int kAux = AUX;
    static constexpr bool kPrio = PRIO;
    static constexpr bool kLoads = true;   // the row loads (else synthetic rows: a compute bound)
    static constexpr bool kSteps = true;   // the row steps (else the rows XOR-folded: a memory-pipeline bound)
    static constexpr bool kFinal = true;   // the per-lane final products M^(64 - l)
    static constexpr bool kStores = true;  // the result stores of every block
    // ragged batches on the long-packet half's dense walk: each packet's (offset, length) by scalar
    // loads one set ahead of its row loads (run_pipelined SM; the vector blocks are a conditional
    // vector load inside the ring: 4.8 % slower on 1 Mi x 4156 B ragged,
    // profiles/r04_ab_ragged_scalar_meta.jsonl).  The batch kernel keeps the vector blocks: its
    // small batches (a wave per packet) wait longer for a scalar load.
    static constexpr bool kScalarMeta = true;
    static constexpr bool kSysStores = false;  // results by system-scope stores (RingHostResults)
};
// The submission ring's jobs (icrc_ring_kernel.hip): results written through to host memory, so the
// job needs no L2 write-back before its done word (a system-scope release fence cost ~4 us per
// 64-packet job, scripts/gpu_r05_ring_ab.sh).
struct RingHostResults : Ring<kStreamAux> {
    static constexpr bool kSysStores = true;
};
#ifdef ICRC_AB_BUILD
// (A/B, ICRC_AB_LONG_VMETA=1: the hybrid's dense long walk) the default ring with the (offset,
// length) of ragged batches in 64-packet vector blocks (the ring before round 4's scalar loads)
struct RingVectorMeta : Ring<kStreamAux> {
    static constexpr bool kScalarMeta = false;
};
// LOADS_ONLY: variants 15, 19 (the loads-only denominator bench.py reports); CRC_ONLY: 18;
// NO_FINAL: 21; NO_STORE: 22 (the result stores of every block but the chunk's last); BARE: 23
// (loads only, without the final products and the per-block stores: the bare read walk).
enum RingCut { kCutLoadsOnly, kCutCrcOnly, kCutNoFinal, kCutNoStore, kCutBare };
template <int AUX, int CUT>
struct RingAblation : Ring<AUX> {
    static constexpr bool kLoads = CUT != kCutCrcOnly;
    static constexpr bool kSteps = CUT != kCutLoadsOnly && CUT != kCutBare;
    static constexpr bool kFinal = CUT != kCutNoFinal && CUT != kCutBare;
    static constexpr bool kStores = CUT != kCutNoStore && CUT != kCutBare;
};
#endif

// Verify runs over the trailer as the stream's last word (kIcrcResidue, icrc_device.h): the same
// kRows loads per slot as compute.
template <int MODE>
constexpr int ring_words() { return kRows; }

// TRAILER: the row holding the trailer's line (the last) and the verify trailer word load with the
// default policy, so the line is in L2 when the trailer store / zeroing follows
// (scripts/trailerbench.hip T9: 0.8615 vs 0.877 ms with every row nt).
template <class A, int MODE, bool TRAILER = false>
__device__ __forceinline__ void slot_load(const SlotMeta &m, uint32_t lane, uint32_t (&u)[ring_words<MODE>()]) {
    if constexpr (!A::kLoads) {
#pragma unroll
        for (int j = 0; j < ring_words<MODE>(); ++j) u[j] = lane * 0x9E3779B9u + static_cast<uint32_t>(j) * 0x85EBCA6Bu;
        return;
    }
    constexpr int kAux = A::kAux;
    // compute reads [0, L-4); verify also the trailer [L-4, L): it is the last word of the loaded
    // rows (verify by residue, kIcrcResidue)
    const int nrec = m.kind == 1 ? static_cast<int>(MODE == kVerify ? m.L : m.L - 4u) : 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(m.pkt, 0, nrec, 0x00020000);
    const uint32_t vbase = 4u * static_cast<uint32_t>(m.k0 - 1 + static_cast<int>(lane));
    // Always the same loads, no branch: hipcc's static vmcnt accounting takes the minimum over
    // all paths, so a conditional load block anywhere in the ring turns the waits for the
    // current packet into vmcnt(0) and drains the prefetch of the next one.
    constexpr int kAuxLast = TRAILER ? 0 : kAux;
#pragma unroll
    for (int j = 0; j < kRows - 1; ++j)
        u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(vbase + 256u * j), 0, kAux);
    u[kRows - 1] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(vbase + 256u * (kRows - 1)), 0, kAuxLast);
}

// Result of a regular packet of the pipelined path, from registers only: compute -> the ICRC;
// verify -> OK / MISMATCH: the ICRC over the packet with its trailer against kIcrcResidue.  TRAILER: the one
// trailer store of the packet (compute: the ICRC, PacketWriter::write, packet_processor.rs:263;
// verify: zeros, is_icrc_valid, 350) as a buffer store that every lane issues, lane 0 in range
// (no branch, so the ring's vmcnt accounting stays exact; an empty slot's descriptor has size 0).
template <int MODE, bool TRAILER>
__device__ __forceinline__ uint32_t regular_result(const SlotMeta &m, uint32_t crc, uint32_t lane) {
    if constexpr (TRAILER) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(m.pkt, 0, m.kind == 1 ? static_cast<int>(m.L) : 0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(MODE == kCompute ? crc : 0u, rs,
                                              static_cast<int>(lane == 0 ? m.L - 4u : 0x80000000u), 0, 0);
    }
    if constexpr (MODE == kCompute) return crc;
    else return crc == kIcrcResidue ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH;
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

// The header masks of rows 0 and 1 for the last k0 seen (k0 is wave-uniform and, in a strided
// batch, the same for every packet: the masks are computed once per wave instead of per packet).
struct HeadMasks {
    int k0;
    uint32_t m0, m1;
};
__device__ __forceinline__ void head_masks_init(HeadMasks &hm) {
    hm.k0 = INT32_MIN;
    hm.m0 = hm.m1 = 0;
}

// Lane = packet decode of one receive descriptor (to_rdma_message, packet_processor.rs:18-71, on
// the UDP payload with the ICRC stripped; field getters packet.rs:57-98 BTH, 173-183 RETH, 222-232
// AETH, 249-251 Immediate).  h[k] = packet word k (bytes 4k..4k+3, LE), zero where the packet has
// no such word before its trailer (words 0..6, IPv4 and UDP, are not read); okb = the verify
// result byte.  v = the 18 dwords of
// icrc_rx_desc.  Shared by the descriptor pass (icrc_rx_desc_kernel) and the fused parse below.
__device__ __forceinline__ void rx_decode(const uint32_t (&h)[18], uint64_t off, uint32_t L, uint32_t okb,
                                          uint32_t (&v)[18]) {
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
}

// ---- the descriptor pass's block (icrc_rx_desc_kernel, icrc_kernels.hip; the one-pass ragged
// receive's sweep, icrc_oct.hip) --------------------------------------------------------------
// Packets base .. base + cnt - 1 whose bit is set in keep get their descriptors (the others are
// neither read nor written).  Header words are loaded three packets per instruction (11 lanes
// each, words 7..17 -- bytes 28..71: rx_decode reads nothing of the IPv4 / UDP header, so those
// lines are not fetched), transposed through LDS (sh: 64 x kRxStride words of this wave) to lane =
// packet for the decode, and transposed back so the descriptors leave as 18 coalesced dword stores.
constexpr uint32_t kRxStride = 19;  // LDS words per packet row (odd: conflict-free lane = packet reads)
constexpr uint32_t kRxWord0 = 7, kRxHdrWords = 11;             // header words the decode reads: 7..17
constexpr uint32_t kRxGroups = 64u / kRxHdrWords;              // packets per load round (5)
constexpr uint32_t kRxRounds = (64u + kRxGroups - 1u) / kRxGroups;  // 13
__device__ __forceinline__ void rx_desc_block(const BatchParams &p, uint32_t *sh, uint32_t base, uint32_t cnt, uint64_t keep,
                                              uint32_t lane) {
    const uint32_t g = lane / kRxHdrWords, w = kRxWord0 + lane - kRxHdrWords * g;
    {
        const uint32_t i = base + lane;
        const bool in = lane < cnt && ((keep >> lane) & 1ull);
        const uint64_t off = in ? (p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride) : 0u;
        const uint32_t L = in ? (p.len ? p.len[i] : p.ulen) : 0u;
        const uint32_t okb = in ? p.ok[i] : 0u;  // from the verify pass
        const uint8_t *pkt = p.base + off;
        const bool fast = L >= ICRC_MIN_PACKET && ((reinterpret_cast<uintptr_t>(pkt) | static_cast<uintptr_t>(L)) & 3u) == 0;
        const uint32_t olo = static_cast<uint32_t>(off), ohi = static_cast<uint32_t>(off >> 32);
        const uint32_t lf = fast ? L : 0u;  // 0: not loaded here (short / irregular)
        // All 22 rounds of header loads go out before any is used (a load under a branch made every
        // round wait for the one before: 60-76 us per 786 K packets), so every lane loads: one with
        // nothing to load reads the first word of the group's first fast packet and drops it.
        const uint64_t fm = __builtin_amdgcn_ballot_w64(fast);
        if (fm != 0u) {
            const int f0 = __builtin_ctzll(fm);
            const uint32_t dlo = static_cast<uint32_t>(__builtin_amdgcn_readlane(olo, f0));  // int: no sign extension
            const uint32_t dhi = static_cast<uint32_t>(__builtin_amdgcn_readlane(ohi, f0));
            const uint8_t *dq = p.base + (static_cast<uint64_t>(dlo) | (static_cast<uint64_t>(dhi) << 32));
            uint32_t hv[kRxRounds];
#pragma unroll
            for (uint32_t r = 0; r < kRxRounds; ++r) {  // kRxGroups packets per round
                const uint32_t j = kRxGroups * r + g;
                const int src = static_cast<int>((j & 63u) << 2);
                const uint32_t jl = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(lf)));
                const uint32_t jlo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(olo)));
                const uint32_t jhi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(ohi)));
                const bool k = g < kRxGroups && j < 64u && 4u * w + 8u <= jl;  // jl = 0 for packets not on this path
                const uint8_t *q =
                    k ? p.base + (static_cast<uint64_t>(jlo) | (static_cast<uint64_t>(jhi) << 32)) + 4u * w : dq;
                hv[r] = *reinterpret_cast<const uint32_t *>(q);
            }
#pragma unroll
            for (uint32_t r = 0; r < kRxRounds; ++r) {
                const uint32_t j = kRxGroups * r + g;
                if (g < kRxGroups && j < 64u) sh[j * kRxStride + w] = hv[r];
            }
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t h[18];
#pragma unroll
        for (uint32_t k = 0; k < 18; ++k) {  // words not loaded (dummy reads, short packets, 0..6) read as 0
            const uint32_t x = k >= kRxWord0 ? sh[lane * kRxStride + k] : 0u;
            h[k] = (fast && 4u * k + 8u <= L) ? x : 0u;
        }
        if (!fast && L >= ICRC_MIN_PACKET) {  // misaligned or L % 4 != 0: byte-wise, this lane only
#pragma unroll
            for (uint32_t k = kRxWord0; k < 18; ++k) {
                uint32_t x = 0;
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) {
                    const uint32_t o = 4u * k + t;
                    x |= (o + 4u < L ? static_cast<uint32_t>(pkt[o]) : 0u) << (8u * t);
                }
                h[k] = x;
            }
        }
        uint32_t v[18];
        rx_decode(h, off, L, okb, v);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t k = 0; k < 18; ++k) sh[lane * kRxStride + k] = v[k];
        __builtin_amdgcn_wave_barrier();
        uint32_t *dst = reinterpret_cast<uint32_t *>(p.rx + base);
#pragma unroll
        for (uint32_t t = 0; t < 18; ++t) {
            const uint32_t idx = t * 64u + lane, pk = idx / 18u, k = idx - 18u * pk;
            if (pk < cnt && ((keep >> pk) & 1ull)) dst[idx] = sh[pk * kRxStride + k];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// PARSE = 2, the fused receive parse of the one-packet pipeline (small batches, icrc_rx_kernel):
// no store per packet (a store in the ring makes hipcc wait for zero there, draining the prefetch).  Each packet's header words
// (lane w = word w, from its rows as loaded), offset and length go into lane q & 63 of these
// registers (v_readlane / v_writelane, uniform lanes); when the 64-packet block's results leave,
// the block is decoded lane = packet (rx_decode) and its descriptors leave with them, as 18 buffer
// stores (lanes without a packet of this kernel out of range).
// Only words 7..17 are kept (BTH from byte 28, extension headers): the decode reads no IPv4 / UDP
// word, and every register here is one fewer for the ring.
constexpr int kRxW0 = 7, kRxWords = 18 - kRxW0;
struct RxAcc {
    uint32_t h[kRxWords];  // h[k - kRxW0] = packet word k
    uint32_t off_lo, off_hi, len;
    uint64_t have;  // block lanes holding a packet
};

__device__ __forceinline__ void rx_acc_init(RxAcc &a) {
#pragma unroll
    for (int k = 0; k < kRxWords; ++k) a.h[k] = 0u;
    a.off_lo = a.off_hi = a.len = 0u;
    a.have = 0ull;
}

// old with lane l replaced by v (v and l wave-uniform).  hipcc has no builtin for v_writelane_b32;
// the LLVM intrinsic is bound by name (the backend puts the lane select in m0, as gfx9's one
// constant-bus read per VALU op requires).
extern "C" __device__ int icrc_llvm_writelane(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t writelane_u32(uint32_t v, uint32_t l, uint32_t old) {
    return static_cast<uint32_t>(icrc_llvm_writelane(static_cast<int>(v), static_cast<int>(l), static_cast<int>(old)));
}

// hdr: packet word w in lane w (w < 18); words at or past the trailer (4 w + 8 > L) are dropped.
__device__ __forceinline__ void rx_acc_put(RxAcc &a, uint32_t hdr, uint32_t qb, uint64_t off, uint32_t L) {
    // word k to lane qb: a ds_bpermute broadcast of lane k and a lane select (no VALU -> SGPR ->
    // VALU round trip per word, as v_readlane + v_writelane would take)
    const bool me = __lane_id() == qb;
#pragma unroll
    for (int k = kRxW0; k < 18; ++k) {
        const uint32_t w = 4u * static_cast<uint32_t>(k) + 8u <= L ? bperm(static_cast<uint32_t>(k), hdr) : 0u;
        a.h[k - kRxW0] = me ? w : a.h[k - kRxW0];
    }
    a.off_lo = me ? static_cast<uint32_t>(off) : a.off_lo;
    a.off_hi = me ? static_cast<uint32_t>(off >> 32) : a.off_hi;
    a.len = me ? L : a.len;
    a.have |= 1ull << qb;
}

// The block's descriptors (packets base .. base + 63; okv lane q = packet q's verify result).
// Every lane issues every store (out of range without a packet): no branch around a store.  The
// fields follow rx_decode; each dword is formed just before its store (sched_barrier) so the flush
// needs few registers beside the ring's.
__device__ __forceinline__ void rx_acc_flush(const BatchParams &p, RxAcc &a, uint32_t base, uint32_t okv, uint32_t lane) {
    const uint32_t L = a.len;
    const uint32_t w7 = a.h[7 - kRxW0], w9 = a.h[9 - kRxW0], w10 = a.h[10 - kRxW0];
    const uint32_t op = w7 & 0x1Fu, tran = (w7 >> 5) & 7u, fl = (w7 >> 8) & 0xFFu, pad = (fl >> 5) & 3u;
    const uint32_t hs = (op == 0x09u || op == 0x0Bu) ? 32u
                      : (op == 0x0Cu)                 ? 44u
                      : (op == 0x11u)                 ? 16u
                      : (op >= 0x06u && op <= 0x10u)  ? 28u
                                                      : 0u;
    const uint32_t status = (L < ICRC_MIN_PACKET)   ? ICRC_RX_TRUNCATED
                          : (hs == 0u)              ? ICRC_RX_INVALID_OPCODE
                          : (tran > 6u)             ? ICRC_RX_INVALID_TRANS_TYPE
                          : (L - 32u < hs + pad)    ? ICRC_RX_TRUNCATED
                                                    : ICRC_RX_OK;
    const bool ack = hs == 16u, ok = status == ICRC_RX_OK;
    const bool reth = ok && !ack, sec = ok && hs == 44u, imm = ok && hs == 32u, aeth = ok && ack;
    const uint64_t poff = (static_cast<uint64_t>(a.off_lo) | (static_cast<uint64_t>(a.off_hi) << 32)) + 28u + hs;
    const bool mine = (a.have >> lane) & 1ull;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t *>(p.rx + base), 0, static_cast<int>(64u * sizeof(icrc_rx_desc)), 0x00020000);
    auto st = [&](int k, uint32_t v) __attribute__((always_inline)) {
        __builtin_amdgcn_raw_buffer_store_b32(v, rs, static_cast<int>(mine ? lane * 72u + 4u * k : 0x80000000u), 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto hw = [&](int k) __attribute__((always_inline)) { return a.h[k - kRxW0]; };
    st(0, reth ? bswap32(hw(11)) : 0u);  // RETH va (big-endian u64, bytes 40-47)
    st(1, reth ? bswap32(hw(10)) : 0u);
    st(2, sec ? bswap32(hw(15)) : 0u);   // secondary RETH va (bytes 56-63)
    st(3, sec ? bswap32(hw(14)) : 0u);
    st(4, ok ? static_cast<uint32_t>(poff) : 0u);
    st(5, ok ? static_cast<uint32_t>(poff >> 32) : 0u);
    st(6, ok ? L - 32u - hs - pad : 0u);
    st(7, reth ? bswap32(hw(12)) : 0u);  // rkey, dlen
    st(8, reth ? bswap32(hw(13)) : 0u);
    st(9, sec ? bswap32(hw(16)) : 0u);
    st(10, sec ? bswap32(hw(17)) : 0u);
    st(11, imm ? bswap32(hw(14)) : 0u);
    st(12, ok ? bswap32(hw(8)) & 0xFFFFFFu : 0u);     // dqpn
    st(13, ok ? bswap32(w9) & 0xFFFFFFu : 0u);        // psn
    st(14, aeth ? bswap32(w10) & 0xFFFFFFu : 0u);     // AETH msn
    st(15, ok ? (bswap16(w7 >> 16) | (op << 16) | (tran << 24)) : 0u);
    const uint32_t flags = ((fl & 0x80u) ? ICRC_RX_SOLICITED : 0u) | ((w9 & 0x80u) ? ICRC_RX_ACK_REQ : 0u) |
                           (ack ? ICRC_RX_ACKNOWLEDGE : 0u) | (hs == 32u ? ICRC_RX_HAS_IMM : 0u) |
                           (hs == 44u ? ICRC_RX_HAS_SECONDARY_RETH : 0u);
    const uint32_t code = ack ? (w10 >> 5) & 3u : 0u, value = ack ? w10 & 0x1Fu : 0u;
    st(16, ok ? (flags | (pad << 8) | (code << 16) | (value << 24)) : 0u);
    st(17, (okv & 0xFFu) | (status << 8));
    a.have = 0ull;
}

// Process one set of S packets (wave-local sequence numbers q0 .. q0+S-1); results go to
// the wave's result buffer.
// PARSE: 0 off; 1 receive parse, a descriptor store per packet (rx_store; A/B variant 301);
// 2 receive parse into RxAcc (the fused receive of small batches).
template <int MODE, int S, class A, int PARSE = 0, bool TRAILER = false>
__device__ __forceinline__ void process_set(const BatchParams &p, const char *lds, const LaneConsts &c,
                                            uint32_t lane, const SlotMeta (&m)[S],
                                            uint32_t (&u)[S][ring_words<MODE>()], uint32_t q0, ResultBuf &rb,
                                            HeadMasks &hm, RxAcc &ra, uint32_t lo = 0) {
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
        if constexpr (PARSE == 2) {  // into RxAcc now, so hdr is not live across the row steps
#pragma unroll
            for (int s = 0; s < S; ++s)
                if (m[s].kind == 1)
                    rx_acc_put(ra, hdr[s], (q0 + s) & 63u, static_cast<uint64_t>(m[s].pkt - p.base), m[s].L);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if (m[s].kind == 1 && m[s].k0 != hm.k0) {  // uniform branch, no memory access
                hm.k0 = m[s].k0;
                hm.m0 = head_mask(hm.k0 + static_cast<int>(lane));
                hm.m1 = head_mask(hm.k0 + static_cast<int>(lane) + 64);
            }
            acc[s] = u[s][0] | hm.m0;  // slots of kind != 1 are never stored
            u[s][1] |= hm.m1;
        }
        // One straight-line block per row for all S chains (the scheduler interleaves them).
        if (same && rmax == kRows) {  // full-MTU packets (4 KiB): no per-row guard branches
#pragma unroll
            for (int j = 1; j < kRows; ++j) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    if constexpr (!A::kSteps) acc[s] ^= u[s][j];
                    else acc[s] = step_m64(lds, acc[s], u[s][j], c);
                }
            }
        } else if (same) {
#pragma unroll
            for (int j = 1; j < kRows; ++j) {
                if (j < rmax) {
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        if constexpr (!A::kSteps) acc[s] ^= u[s][j];
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
                        if constexpr (!A::kSteps) {
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
        for (int s = 0; s < S; ++s) fin[s] = A::kFinal ? final_mul(lds, acc[s], c.fin) : acc[s];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t r = regular_result<MODE, TRAILER>(m[s], ~wave_xor(fin[s]), lane);
            if (m[s].kind == 1) {
                rb_put(rb, q0 + s, r);
                if constexpr (PARSE == 1)
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
            if constexpr (PARSE == 1)
                rx_store(p.rx, lo + q0 + s, hdr_slow, static_cast<uint64_t>(m[s].pkt - p.base), m[s].L, r, lane, c);
            if constexpr (PARSE == 2)
                rx_acc_put(ra, hdr_slow, (q0 + s) & 63u, static_cast<uint64_t>(m[s].pkt - p.base), m[s].L);
        }
}

// A wave owns the contiguous packet range [lo, lo + nq) and walks it in sets of S packets
// (S independent CRC chains for ILP); the loads of set t + D are issued before set t is
// processed (a D-deep register ring), keeping ~D*S packets in flight per wave against the
// ~3 us loaded HBM latency.  Results leave 64 at a time as coalesced stores.
// TABLE: the table image is not in LDS yet.  The wave issues its first (offset, length) block
// (ragged batches), its share of the table image (into `tv`) and its first sets' row loads before
// it waits for the table share, so that the three memory latencies overlap (a small batch, one
// packet per wave, is made of little else); then every wave, with or without packets, writes its
// share to LDS and joins the barrier.
// SM: a ragged batch's (offset, length) by scalar loads one set ahead of the row loads (the long-
// packet half's dense walk, whose waves hold hundreds of packets) instead of 64-packet vector
// blocks read back lane by lane.
template <int MODE, int S, int D, class A, int PARSE = 0, bool LONG = false, bool TRAILER = false, bool TABLE = false,
          bool SM = false>
__device__ __forceinline__ void run_pipelined(const BatchParams &p, const char *lds, const LaneConsts &c,
                                              uint32_t lane, uint32_t lo, uint32_t nq, TableShare *tv = nullptr) {
    constexpr int B = D + 1;
    static_assert(64 % S == 0, "sets must not straddle a 64-packet result block");
    if (!TABLE && nq == 0) return;
    const uint32_t nsets = (nq + S - 1) / S;
    const bool ragged = p.off != nullptr || p.len != nullptr;
    MetaBlock mb;
    mb.block = -1;
    mb.off_lo = mb.off_hi = mb.len = 0;
    ResultBuf rb;
    rb.v = 0;
    rb.valid = 0;
    HeadMasks hm;
    head_masks_init(hm);
    RxAcc ra;
    if constexpr (PARSE == 2) rx_acc_init(ra);
    SlotMeta m[B][S];
    uint32_t u[B][S][ring_words<MODE>()];
    // (SM, ragged batches) the (offset, length) of one set's slots by scalar loads, issued one
    // set before its row loads need them
    const bool smeta = SM && ragged;
    uint64_t nm_off[S];
    uint32_t nm_len[S];
    auto smeta_load = [&](uint32_t set) __attribute__((always_inline)) {
        typedef __attribute__((address_space(4))) const uint64_t c_u64;
        typedef __attribute__((address_space(4))) const uint32_t c_u32;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t q = set * S + static_cast<uint32_t>(s);
            const uint32_t i = lo + q;
            nm_off[s] = 0;
            nm_len[s] = 0;
            if (q < nq) {  // uniform: past the range nothing is read
                nm_off[s] = p.off ? ((c_u64 *)p.off)[i] : static_cast<uint64_t>(i) * p.stride;
                nm_len[s] = p.len ? ((c_u32 *)p.len)[i] : p.ulen;
            }
        }
    };
    auto smeta_slot = [&](uint32_t set, int s, SlotMeta &sm) __attribute__((always_inline)) {
        sm.kind = 0;
        sm.R = 0;
        sm.k0 = 0;
        sm.pkt = p.base;
        sm.L = 0;
        if (set * S + static_cast<uint32_t>(s) < nq) slot_classify<MODE, LONG>(p, nm_off[s], nm_len[s], sm);
    };
    if constexpr (TABLE) {
        if (ragged && nq != 0 && !smeta) meta_fetch(p, mb, lo, lo + nq, 0, lane);
        table_fetch(*tv, p.table);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        // TABLE: unconditional (an empty slot's loads are out of range), so that the wait for the
        // table share below counts exactly these loads behind it
        if (TABLE || static_cast<uint32_t>(d) < nsets) {
            if (smeta) smeta_load(static_cast<uint32_t>(d));
#pragma unroll
            for (int s = 0; s < S; ++s) {
                if (smeta) smeta_slot(static_cast<uint32_t>(d), s, m[d][s]);
                else slot_meta<MODE, LONG>(p, mb, ragged, lo, d * S + s, nq, lane, m[d][s]);
                slot_load<A, MODE, TRAILER>(m[d][s], lane, u[d][s]);
            }
        }
    }
    if (smeta) smeta_load(static_cast<uint32_t>(D));
    if constexpr (TABLE) {
        table_store(*tv, const_cast<uint4 *>(reinterpret_cast<const uint4 *>(lds)));
        if (nq == 0) return;
    }
    for (uint32_t t = 0; t < nsets; t += B) {
        const bool cont = static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            constexpr int bp = (b + D) % B;
            const uint32_t ts = t + b;
            if (ts >= nsets) return false;
            const uint32_t tp = ts + D;
            // unconditional: past the end slot_meta yields kind 0 (zero-size descriptor).  The burst
            // runs at raised wave priority, so the loads leave ahead of the other waves' row steps
            // (scripts/overlapbench.hip: the C1 walk 0.667 -> 0.648 ms against 0.638 loads-only).
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(3);
#pragma unroll
            for (int s = 0; s < S; ++s) {
                if (smeta) smeta_slot(tp, s, m[bp][s]);
                else slot_meta<MODE, LONG>(p, mb, ragged, lo, tp * S + s, nq, lane, m[bp][s]);
                slot_load<A, MODE, TRAILER>(m[bp][s], lane, u[bp][s]);
            }
            if (smeta) smeta_load(tp + 1u);
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(0);
            const uint32_t q0 = ts * S;
            process_set<MODE, S, A, PARSE, TRAILER>(p, lds, c, lane, m[b], u[b], q0, rb, hm, ra, lo);
            const uint32_t qn = q0 + S;  // next unprocessed
            if ((qn & 63u) == 0 || qn >= nq) {
                if constexpr (PARSE == 2) rx_acc_flush(p, ra, lo + ((q0 >> 6) << 6), rb.v, lane);
                // !A::kStores (A/B): only the chunk's last block is stored (its lanes depend on every
                // earlier packet through rb_put's selects, so nothing is dead code)
                if constexpr (A::kStores) rb_flush<MODE, A::kSysStores>(p, rb, lo + ((q0 >> 6) << 6), lane);
                else if (qn >= nq) rb_flush<MODE, A::kSysStores>(p, rb, lo + ((q0 >> 6) << 6), lane);
            }
            return true;
        });
        if (!cont) return;
    }
}

// ---- long packets of a ragged batch (hybrid dispatch) ------------------------------------------
// The one-packet pipeline (S = 1, D-deep prefetch) over only the packets with L >= p.split_len;
// the oct kernel (icrc_oct.hip) takes the shorter ones, whose per-packet costs it divides by
// eight.  Long packets stay here because one contiguous 256-byte row per wave instruction
// streams from HBM faster than several packets per instruction (profiles/r01_membench.json,
// patterns D and E; profiles/r02_shortbench.jsonl).  The walk skips short packets with the
// ballot of each 64-packet meta block; results are kept per block and stored 64 at a time.
// Packets in flight ahead of the one being stepped (3 measured the same on C2: the long half's
// tail is the CUs freeing up from the short-packet kernel, not the walk's latency).
constexpr int kLongWalkDepth = 1;
// PARSE 2 (the ragged one-pass receive's long half): each long packet's descriptor collected as in
// the fused small-batch receive (RxAcc) and stored with its block's ok bytes.
template <int MODE, int D, class A, bool TRAILER, int PARSE = 0>
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
    HeadMasks hm;
    head_masks_init(hm);
    RxAcc ra;  // PARSE 2: the current result block's descriptors
    if constexpr (PARSE == 2) rx_acc_init(ra);
    SlotMeta m[B][1];
    uint32_t qs[B];
    uint32_t u[B][1][ring_words<MODE>()];
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
                const int N = static_cast<int>(stream_words<MODE>(L));
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
        slot_load<A, MODE, TRAILER>(m[d][0], lane, u[d][0]);
        if (m[d][0].kind) inflight += 1;
    }
    for (;;) {
        static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            constexpr int bp = (b + D) % B;
            next(m[bp][0], qs[bp]);
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(3);
            slot_load<A, MODE, TRAILER>(m[bp][0], lane, u[bp][0]);
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(0);
            if (m[bp][0].kind) inflight += 1;
            if (m[b][0].kind) {
                const int blk = static_cast<int>(qs[b] >> 6);
                if (blk != rb_block) {
                    if (rb.valid) {
                        if constexpr (PARSE == 2) rx_acc_flush(p, ra, lo + static_cast<uint32_t>(rb_block) * 64u, rb.v, lane);
                        rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
                    }
                    rb_block = blk;
                }
                process_set<MODE, 1, A, PARSE, TRAILER>(p, lds, c, lane, m[b], u[b], qs[b], rb, hm, ra, lo);
                inflight -= 1;
            }
            return true;
        });
        if (qn >= nq && inflight == 0) break;
    }
    if (rb.valid) {
        if constexpr (PARSE == 2) rx_acc_flush(p, ra, lo + static_cast<uint32_t>(rb_block) * 64u, rb.v, lane);
        rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
    }
}

// A sparse long-packet walk tried in round 6 (A/B only, see long_walk_masked below).
// run_pipelined_long above fetches each 64-packet block's
// (offset, length) when its walk reaches the block and waits for it there, so every block costs a
// memory round trip with the ring drained (a conditional load: vmcnt(0)); on configs[2] (1.4 % long
// packets) that is about one round trip per long packet.  Here the wave scans its range for long
// packets 1024 at a time (16 vector loads of 64 lengths issued together, one wait; lane j of two
// VGPRs = the long-packet mask of block j of the group), and each long packet's (offset, length)
// comes by a vector load issued one packet ahead, before that packet's row loads, every step
// (out of range when there is none), so no wait in the ring is for more than the loads already
// behind it.
template <int MODE, class A, bool TRAILER, int PARSE = 0>
__device__ __forceinline__ void run_walk_masked(const BatchParams &p, const char *lds, const LaneConsts &c,
                                                uint32_t lane, uint32_t lo, uint32_t nq) {
    constexpr int B = 2;  // one packet's rows in flight while the previous one is stepped
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    if (nq == 0) return;
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t *>(p.len ? p.len + lo : nullptr), 0, p.len ? static_cast<int>(nq * 4u) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t *>(p.off ? p.off + lo : nullptr), 0, p.off ? static_cast<int>(nq * 8u) : 0, 0x00020000);
    uint32_t gm_lo = 0, gm_hi = 0;  // lane j < 16: the long packets of block 16 grp + j
    int grp = -1;
    uint32_t qn = 0;  // next candidate
    auto find = [&]() __attribute__((always_inline)) -> uint32_t {
        while (qn < nq) {
            const uint32_t blk = qn >> 6, g = blk >> 4;
            if (static_cast<int>(g) != grp) {  // a new group of 16 blocks: one round trip for all of them
                uint32_t lv[16];
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    lv[j] = p.len ? __builtin_amdgcn_raw_buffer_load_b32(rl, static_cast<int>(((g * 16u + j) * 64u + lane) * 4u), 0, 0)
                                  : ((g * 16u + j) * 64u + lane < nq ? p.ulen : 0u);
                uint32_t mlo = 0, mhi = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint64_t m = __ballot(lv[j] >= p.split_len);
                    mlo = lane == static_cast<uint32_t>(j) ? static_cast<uint32_t>(m) : mlo;
                    mhi = lane == static_cast<uint32_t>(j) ? static_cast<uint32_t>(m >> 32) : mhi;
                }
                gm_lo = mlo;
                gm_hi = mhi;
                grp = static_cast<int>(g);
            }
            const int j = static_cast<int>(blk & 15u);
            const uint64_t m = ((static_cast<uint64_t>(readlane_u32(gm_hi, j)) << 32) | readlane_u32(gm_lo, j)) &
                               (~0ull << (qn & 63u));
            if (m == 0ull) {
                qn = (blk + 1u) * 64u;
                continue;
            }
            const uint32_t q = blk * 64u + static_cast<uint32_t>(__builtin_ctzll(m));
            qn = q + 1u;
            return q;
        }
        return kNone;
    };
    // the pending packet: its index and (lane 0) its (offset, length), loaded one packet ahead
    uint32_t pq = find();
    uint32_t pv_lo = 0, pv_hi = 0, pv_len = 0;
    auto pload = [&]() __attribute__((always_inline)) {  // unconditional: out of range when there is none
        const bool have = pq != kNone && lane == 0u;
        const auto o = __builtin_amdgcn_raw_buffer_load_b64(ro, have ? static_cast<int>(pq * 8u) : static_cast<int>(0x80000000u), 0, 0);
        pv_lo = o[0];
        pv_hi = o[1];
        pv_len = __builtin_amdgcn_raw_buffer_load_b32(rl, have ? static_cast<int>(pq * 4u) : static_cast<int>(0x80000000u), 0, 0);
    };
    pload();
    auto next = [&](SlotMeta &sm, uint32_t &q) __attribute__((always_inline)) {
        sm.kind = 0;
        sm.R = 0;
        sm.k0 = 0;
        sm.pkt = p.base;
        sm.L = 0;
        q = pq;
        if (pq == kNone) {
            pload();  // (the same loads every step)
            return;
        }
        const uint64_t off = p.off ? ((static_cast<uint64_t>(readlane_u32(pv_hi, 0)) << 32) | readlane_u32(pv_lo, 0))
                                   : static_cast<uint64_t>(lo + pq) * p.stride;
        const uint32_t L = p.len ? readlane_u32(pv_len, 0) : p.ulen;
        pq = find();
        pload();
        sm.pkt = p.base + off;
        sm.L = L;
        sm.kind = 2;
        if (((reinterpret_cast<uintptr_t>(sm.pkt) | static_cast<uintptr_t>(L)) & 3u) == 0) {
            const int N = static_cast<int>(stream_words<MODE>(L));
            const int R = (N + 63) >> 6;
            if (R <= kRows) {
                sm.kind = 1;
                sm.R = R;
                sm.k0 = N - 64 * R;
            }
        }
    };

    ResultBuf rb;
    rb.v = 0;
    rb.valid = 0;
    int rb_block = -1;
    HeadMasks hm;
    head_masks_init(hm);
    RxAcc ra;
    if constexpr (PARSE == 2) rx_acc_init(ra);
    SlotMeta m[B][1];
    uint32_t qs[B];
    uint32_t u[B][1][ring_words<MODE>()];
    int inflight = 0;
    next(m[0][0], qs[0]);
    slot_load<A, MODE, TRAILER>(m[0][0], lane, u[0][0]);
    if (m[0][0].kind) inflight += 1;
    for (;;) {
        static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            constexpr int bp = (b + 1) % B;
            next(m[bp][0], qs[bp]);
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(3);
            slot_load<A, MODE, TRAILER>(m[bp][0], lane, u[bp][0]);
            if constexpr (A::kPrio) __builtin_amdgcn_s_setprio(0);
            if (m[bp][0].kind) inflight += 1;
            if (m[b][0].kind) {
                const int blk = static_cast<int>(qs[b] >> 6);
                if (blk != rb_block) {
                    if (rb.valid) {
                        if constexpr (PARSE == 2) rx_acc_flush(p, ra, lo + static_cast<uint32_t>(rb_block) * 64u, rb.v, lane);
                        rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
                    }
                    rb_block = blk;
                }
                process_set<MODE, 1, A, PARSE, TRAILER>(p, lds, c, lane, m[b], u[b], qs[b], rb, hm, ra, lo);
                inflight -= 1;
            }
            return true;
        });
        if (pq == kNone && inflight == 0) break;
    }
    if (rb.valid) {
        if constexpr (PARSE == 2) rx_acc_flush(p, ra, lo + static_cast<uint32_t>(rb_block) * 64u, rb.v, lane);
        rb_flush<MODE>(p, rb, lo + static_cast<uint32_t>(rb_block) * 64u, lane);
    }
}

// (A/B only, ICRC_AB_LONG_WALK=1) run_walk_masked instead of run_pipelined_long.  Measured and
// rejected: configs[2] compute 0.428-0.436 ms against 0.425-0.430, receive 0.515-0.525 against
// 0.511, identical results (scripts/probe_long_walk.py, profiles/r06/c2/long_walk_ab.jsonl): the
// walk's meta round trips were not what the long half waits for.
__device__ __forceinline__ bool long_walk_masked(const BatchParams &p) {
#ifdef ICRC_AB_BUILD
    return p.ab_long_walk != 0;
#else
    (void)p;
    return false;
#endif
}

// Default (COMPACT = false): per wave, the C1 pipeline (S = 2 chains, D = 1) over the wave's whole
// chunk with short packets left as empty slots when long packets are dense — on an all-long ragged
// batch it runs at the strided rate (1 Mi x 4156 B: 0.75 ms split vs 0.80-0.87 with the walker) —
// and the compacting S = 1 walker above when they are sparse (on a mixed-MTU batch the dense walk
// costs 1.32 ms against 0.49).  COMPACT = true: the walker always (A/B: variant 200 + q).
// Split batches (hybrid dispatch): whether any packet in [g0, end) is short (SHORT: L < split_len)
// or long (!SHORT).  Every thread of the workgroup calls it; the waves scan 1024-packet strides
// and stop as soon as one of them has found such a packet (a flag in LDS word 0, which the caller
// overwrites with its tables only after the last barrier here).
template <bool SHORT>
__device__ __forceinline__ bool wg_any_split(const BatchParams &p, uint4 *lds4, uint64_t g0, uint64_t end) {
    volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(lds4);
    if (threadIdx.x == 0) *flag = 0u;
    __syncthreads();
    for (uint64_t b = g0; b < end; b += kThreadsPerGroup) {
        const uint64_t i = b + threadIdx.x;
        if (__ballot(i < end && (p.len[i] < p.split_len) == SHORT) != 0ull) {
            *flag = 1u;
            break;
        }
        if (__builtin_amdgcn_readfirstlane(static_cast<int>(*flag)) != 0) break;
    }
    __syncthreads();
    const bool go = *flag != 0u;
    __syncthreads();  // every wave has read the flag before the caller's table load overwrites it
    return go;
}

// The long-packet kernel's work for workgroup `bid` of `nblk` (its own kernel, or the long-packet
// workgroups of the fused hybrid kernel, icrc_oct.hip).
// PARSE 2: the ragged one-pass receive's long half (descriptors of the long packets, RxAcc).
template <int MODE, bool COMPACT, bool TRAILER, class LA = Ring<kStreamAux>, int PARSE = 0>
__device__ __forceinline__ void long_body(const BatchParams &p, uint4 *lds4, uint32_t bid, uint32_t nblk) {
    if (p.split_len != 0 && p.len != nullptr) {
        // A workgroup whose packets are all the oct kernel's exits before its 160 KiB table load.
        const uint64_t per = static_cast<uint64_t>(kWavesPerGroup) * wave_chunk(p.n, nblk * kWavesPerGroup);
        const uint64_t g0 = static_cast<uint64_t>(bid) * per, g1 = g0 + per < p.n ? g0 + per : p.n;
        if (!wg_any_split<false>(p, lds4, g0, g1)) return;
    }
    table_fill(lds4, p.table);
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t tw = nblk * kWavesPerGroup;
    const uint32_t chunk = wave_chunk(p.n, tw);
    const uint64_t g0 = static_cast<uint64_t>(bid) * kWavesPerGroup * chunk;
    // The waves' shares: skewed by age as in the batch kernel (p.skew's long half) when the
    // workgroup's range is dense with long packets, equal otherwise — on sparse ranges (C2) a skew
    // measured slower (profiles/r03_probe_skew_long.jsonl; dense: profiles/r04_ab_long_dense_skew.jsonl).
    // The sample: 64 lengths spread evenly over the whole range (the same in every wave), so a range
    // that turns sparse after its first packets does not take the dense range's skew.
    uint32_t skew = 0u;
    if (!COMPACT && p.len != nullptr && g0 < p.n) {
        const uint64_t span = (p.n - g0 < static_cast<uint64_t>(kWavesPerGroup) * chunk)
                                  ? p.n - g0 : static_cast<uint64_t>(kWavesPerGroup) * chunk;
        const uint64_t step = span > 64u ? span / 64u : 1u;
        const uint64_t i = g0 + lane * step;
        const uint64_t dm = __ballot(i < p.n && lane < span && p.len[i] >= p.split_len);
        const uint32_t ns = span < 64u ? static_cast<uint32_t>(span) : 64u;
        if (4u * static_cast<uint32_t>(__builtin_popcountll(dm)) >= 3u * ns) skew = p.skew >> 16;
    }
    uint64_t lo64, hi64;
    wave_range(g0, chunk, wave, skew, lo64, hi64);
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = static_cast<uint32_t>((hi64 < p.n ? hi64 : p.n) - lo64);
    if constexpr (COMPACT) {
        run_pipelined_long<MODE, kLongWalkDepth, Ring<kStreamAux>, TRAILER, PARSE>(p, lds, c, lane, lo, nq);
    } else {
        // Per wave, by the density of long packets in its first 64-packet block: dense (>= 3/4,
        // e.g. a 4 KiB WRITE stream) -> the C1 pipeline with short packets as empty slots; sparse
        // (a mixed-MTU batch: ~1.5 % long) -> the compacting walker, which visits long packets only.
        const uint32_t L0 = lane < nq ? (p.len ? p.len[lo + lane] : p.ulen) : 0u;
        const uint64_t lm = __ballot(lane < nq && L0 >= p.split_len);
        const uint32_t nb = nq < 64u ? nq : 64u;
        if (4u * static_cast<uint32_t>(__builtin_popcountll(lm)) >= 3u * nb) {
            // (PARSE: a dense range's descriptors are the sweep's -- stored inside this ring they cost
            // 786 K x 4156 B 0.608 ms against 0.540, the fused pass's old finding -- so the wave only
            // raises the call's second sweep flag, and the sweep takes every long packet)
            run_pipelined<MODE, 2, 1, LA, 0, true, TRAILER, false, LA::kScalarMeta>(p, lds, c, lane, lo, nq);
            if (PARSE && p.rx_flag && lane == 0) atomicMax(p.rx_flag + 1, p.rx_gen);
        } else if (long_walk_masked(p))
            run_walk_masked<MODE, Ring<kStreamAux>, TRAILER, PARSE>(p, lds, c, lane, lo, nq);
        else
            run_pipelined_long<MODE, kLongWalkDepth, Ring<kStreamAux>, TRAILER, PARSE>(p, lds, c, lane, lo, nq);
    }
}

}  // namespace
}  // namespace icrc
