// icrc_oct.hip — the short-packet ICRC kernel (variant 40, the default for ragged batches and for
// strided batches of short packets): eight packets per wavefront, each packet's rows in 10-row
// FRAMES, frames chained for longer packets (L <= 1088 here; longer ones belong to the long-packet
// kernel of the hybrid dispatch).  Bit-exact with compute_icrc / is_icrc_valid
// (blue-rdma-device/src/third_party/net/packet_processor.rs:275-301, 341-353); the algorithm is
// described at the top of icrc_kernels.hip.
//
// Mapping.  Lanes 8g .. 8g+7 carry one packet; a packet row is 8 stream words (one
// buffer_load_dword per lane: 32 contiguous bytes per packet, 256 B per wave instruction).  The
// stream (N words) is front-padded with z = -N mod 8 zero words (free leading zeros), so its rows
// are aligned to BOTH ends: lane c of row r holds word 8 r + c - z.  Hence
//  * the header masks (stream words 0..9) always fall in rows 0..2 — three OR masks per set, read
//    with ds_bpermute from one register that holds the mask of word k in lane k;
//  * the column multiplier M^(8 - c) depends only on the lane (the oct table image);
//  * a packet of R rows simply stops after its row R - 1: a set of packets with different row
//    counts freezes each lane's accumulator past its own last row (one select per row, only in
//    such sets), and no set ever carries leading empty rows.
//
// Frames.  A ring slot is one frame: the 10 row loads of one set of eight packets (rows 10 f ..
// 10 f + 9), what the process side needs, and uniform flags (first / last frame of its set).
// Every slot issues exactly the same loads, unconditionally (absent lanes: an out-of-range
// offset; rows past a packet's end read what follows it, within the block, and are skipped), so
// the compiler's vmcnt waits stay exact; the accumulator carries from frame to frame.  (A uniform
// branch between two load sequences, tried, made it wait for all but the newest frame.)  The row loads take their row
// offsets from the instruction's immediate field (no per-row address arithmetic; the register
// offset is never negative, see the packetizer note in icrc_kernels.hip).
//
// Why (measured, profiles/r02_shortbench.jsonl, r02_probe_short_oct_ablation.jsonl): the access
// shape itself (8 packets per instruction, 32-B rows, default cache policy) streams at 5.96
// TB/s on 316- and 1084-byte packets, as fast as one packet per wave; the previous kernels lost
// to per-set instruction count (their loads-only build ran within 4 % of the full one).
//
// Per 64-packet block the packets this kernel takes (44 <= L <= 1088, 4-byte aligned, L % 4
// == 0, within [-1 GiB, +1 GiB) of the block's first one) are sorted by row count (a radix sort
// over the lanes, skipped when already sorted), so most sets are uniform.  The rest go to a
// per-packet tail loop.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "icrc_device.h"
#include "icrc_internal.h"
#include "icrc_long.h"

namespace icrc {
namespace {

constexpr uint32_t kOctOOR = 0x80000000u;       // buffer offset out of range: the load returns 0
constexpr uint32_t kOctFar = 0x7FFF0000u;       // an absent lane's row offset: out of range, and
                                                // + the immediate row offset never wraps
constexpr uint32_t kOctRelLimit = 0x7F000000u;  // packet offset in its block + L stay below
constexpr uint32_t kOctNotMine = 63u;           // sort key (>> 6) of a packet this kernel skips
constexpr int kOctK = 10;                       // rows per frame (320 bytes of a packet)
constexpr bool kOctPrio = true;
constexpr bool kOctClampRows = true;            // a set's rows past its last one re-load that row
constexpr int kOctPairs = 2;                    // ring positions of two frames: one pair in flight
constexpr uint32_t kOctMaxL = 1088u;            // 34 rows, 4 frames: longer packets are the long kernel's
// Block results are held in registers and stored kOctRes blocks at a time (and after the ring):
// a store inside the ring sits in the same in-order vmcnt queue as the row loads, so every load
// behind it waits for its write acknowledgement (scripts/shortbench.hip: one store per 8 sets
// costs 19 % of the short-packet stream; this buffer: C2 -1.5-2.5 %, same-box A/B).
constexpr int kOctRes = 8;

// Frame descriptor (one per frame of a block, lane t of OctBlock::ftab; also the slot flags):
constexpr uint32_t kFdSet = 7u;             // bits 0-2: the set (sorted positions 8 s .. 8 s + 7)
constexpr uint32_t kOctFirst = 1u << 3;     // first frame of its set
constexpr uint32_t kOctLast = 1u << 4;      // last frame of its set
constexpr uint32_t kOctUni = 1u << 5;       // every packet of the set has the same row count
constexpr uint32_t kOctFull = 1u << 6;      // the set's longest packet fills all rows of this frame
constexpr uint32_t kOctBlockLast = 1u << 7; // last frame of the block: its results leave
constexpr uint32_t kOctHave = 1u << 8;      // (slot flags) the slot holds a frame
// bits 16-23: frame index f in the set; bits 24-31: rows of the set's longest packet from the
// frame's row 0 (rrem)

// A prepared block of 64 packets.  key / vrel / len are indexed by SORTED position (lane p);
// pos by original index (lane i); ftab by frame (lane t).
struct OctBlock {
    uint32_t key;   // R << 6 | original index (R = kOctNotMine: not this kernel's)
    uint32_t vrel;  // packet offset - boff
    uint32_t len;   // L
    uint32_t pos;   // sorted position of packet i
    uint32_t ftab;  // frame descriptors
    uint64_t mine;  // original indices this kernel computes
    uint64_t boff;  // block base (byte offset from p.base): the packets' offsets are boff + vrel
    uint32_t bend;  // highest (offset - boff + L) of those packets: the loads' record count
    int nfr;        // frames
    int block;
};

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t readfirstlane_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v)));
}

// Maximum over the 64 lanes (DPP within 16-lane rows, then the four rows on the scalar unit).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = umax32(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0xB1, 0xF, 0xF, true)));
    x = umax32(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x4E, 0xF, 0xF, true)));
    x = umax32(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x124, 0xF, 0xF, true)));
    x = umax32(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x128, 0xF, 0xF, true)));
    const uint32_t m = umax32(umax32(readlane_u32(x, 0), readlane_u32(x, 16)), umax32(readlane_u32(x, 32), readlane_u32(x, 48)));
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m)));  // keep it scalar
}

// Lanes below this one whose bit is set in m.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

constexpr uint64_t kOctBaseSlack = 1ull << 30;  // block base: 1 GiB below its first packet

// Classify block b from this lane's (offset, L): which packets are this kernel's, their row
// counts, the block's base offset and extent; sort by row count.  Returns the ballot of packets
// that are neither this kernel's nor the long-packet kernel's (the tail loop's).
template <int MODE>
__device__ __forceinline__ uint64_t oct_block(const BatchParams &p, OctBlock &B, uint64_t off, uint32_t L, bool valid,
                                              uint32_t lo, int b, uint32_t lane) {
    const bool foreign = valid && p.split_len != 0 && L >= p.split_len;  // the long-packet kernel's
    bool mine = valid && !foreign && L >= ICRC_MIN_PACKET && L <= kOctMaxL &&
                ((reinterpret_cast<uintptr_t>(p.base + off) | L) & 3u) == 0;
    uint64_t boff;
    if (p.off == nullptr) {
        boff = static_cast<uint64_t>(lo + static_cast<uint32_t>(b) * 64u) * p.stride;
    } else {  // 1 GiB below the first candidate's offset (packets further apart: the tail loop)
        const uint64_t cand = __ballot(mine);
        const int f = cand ? __builtin_ctzll(cand) : 0;
        const uint64_t o0 = static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off), f)) |
                            (static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off >> 32), f)) << 32);
        boff = o0 > kOctBaseSlack ? o0 - kOctBaseSlack : 0ull;
    }
    mine = mine && off >= boff && (off - boff) + L <= kOctRelLimit;
    const uint32_t vrel = static_cast<uint32_t>(off - boff);
    const uint32_t R = mine ? (stream_words<MODE>(L) + 7u) >> 3 : kOctNotMine;
    // sort (R << 6 | index) ascending: LSD radix over the bits of R that vary, one ballot and one
    // ds_permute per bit (skipped when the block is already in order)
    uint32_t key = (R << 6) | lane;
    const uint32_t nxt = bperm((lane + 1u) & 63u, key);
    if (__ballot(lane == 63u || key <= nxt) != ~0ull) {
#pragma unroll
        for (int bit = 6; bit < 12; ++bit) {
            const uint64_t ones = __ballot((key >> bit) & 1u);
            if (ones != 0ull && ones != ~0ull) {
                const uint32_t r1 = lanes_below(ones);
                const uint32_t nzero = 64u - static_cast<uint32_t>(__popcll(ones));
                const uint32_t dst = ((key >> bit) & 1u) ? nzero + r1 : lane - r1;
                key = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(static_cast<int>(dst << 2), static_cast<int>(key)));
            }
        }
    }
    const uint32_t idx = key & 63u;
    B.key = key;
    B.vrel = bperm(idx, vrel);
    B.len = bperm(idx, L);
    B.pos = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(static_cast<int>(idx << 2), static_cast<int>(lane)));
    B.pos = mine ? B.pos : 0xFFu;
    B.mine = __ballot(mine);
    B.boff = boff;
    B.bend = wave_max_u32(mine ? vrel + L : 0u);
    B.block = b;
    // The frame schedule.  Lane s < nsets: set s's longest / shortest row count and frame count
    // (ceil(R / 10) as a multiply-shift, exact below 2000), and its first frame (a DPP prefix sum
    // over lanes 0..7); then every frame lane t finds its set through a scattered start mark.
    const int nmine = __popcll(B.mine);
    const uint32_t nsets = static_cast<uint32_t>((nmine + 7) >> 3);
    const uint32_t s8 = (lane & 7u) * 8u;
    const uint32_t plast = s8 + 7u < static_cast<uint32_t>(nmine - 1) ? s8 + 7u : static_cast<uint32_t>(nmine - 1);
    const uint32_t rmax = bperm(plast & 63u, key) >> 6;
    const uint32_t rmin = bperm(s8, key) >> 6;
    const bool live_set = lane < nsets;
    const uint32_t nf = live_set ? ((rmax + 9u) * 6554u) >> 16 : 0u;
    uint32_t inc = nf;  // inclusive prefix sum within the first DPP row (lanes 0..15)
    inc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(inc), 0x111, 0xF, 0xF, true));
    inc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(inc), 0x112, 0xF, 0xF, true));
    inc += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(inc), 0x114, 0xF, 0xF, true));
    const uint32_t start = inc - nf;
    B.nfr = nsets ? static_cast<int>(readlane_u32(inc, 7)) : 0;
    const uint32_t sinfo = start | (nf << 8) | (rmax << 16) | (rmin == rmax ? 1u << 24 : 0u);
    const uint32_t mark = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(static_cast<int>((live_set ? start : 63u) << 2),
                                                                            static_cast<int>(live_set ? 1u : 0u)));
    const uint64_t starts = __ballot(mark != 0u);
    const uint32_t st = lanes_below(starts) + static_cast<uint32_t>((starts >> lane) & 1ull) - 1u;  // this frame's set
    const uint32_t si = bperm(st & 7u, sinfo);
    const uint32_t f = lane - (si & 0xFFu);
    const uint32_t rrem = ((si >> 16) & 0xFFu) - static_cast<uint32_t>(kOctK) * f;
    B.ftab = (st & kFdSet) | (f == 0u ? kOctFirst : 0u) | (f + 1u == ((si >> 8) & 0xFFu) ? kOctLast : 0u) |
             ((si >> 24) ? kOctUni : 0u) | (rrem >= static_cast<uint32_t>(kOctK) ? kOctFull : 0u) |
             (static_cast<int>(lane) + 1 == B.nfr ? kOctBlockLast : 0u) | kOctHave | (f << 16) |
             ((rrem < 255u ? rrem : 255u) << 24);
    return __ballot(valid && !mine && !foreign);
}

// The tail loop's classification (reads (offset, L) from the batch arrays).
template <int MODE>
__device__ __forceinline__ uint64_t oct_classify(const BatchParams &p, uint32_t lo, uint32_t nq, int b, uint32_t lane,
                                                 uint64_t &off, uint32_t &L) {
    const uint32_t q = static_cast<uint32_t>(b) * 64u + lane;
    const bool valid = q < nq;
    const uint32_t i = lo + q;
    off = 0;
    L = 0;
    if (valid) {
        off = p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride;
        L = p.len ? p.len[i] : p.ulen;
    }
    OctBlock B;
    return oct_block<MODE>(p, B, off, L, valid, lo, b, lane);
}

// One ring slot = one frame of one set (per-lane values in VGPRs, the frame descriptor in an SGPR).
template <int MODE, bool TRAILER>
struct OctSlot {
    uint32_t u[kOctK];  // frame rows (verify: the trailer is the stream's last word, kIcrcResidue)
    int kf;        // stream word of this lane in the set's row 0 (header masks), first frame
    int rl;        // rows of this lane's packet from this frame's row 0 (generic sets: the freeze)
    uint32_t rt;   // routing: lane i of the block takes the result of lane rt (0xFF: none), last frame
    uint32_t rq;   // the block (bits 0-30); bit 31: lane i of the block is not this kernel's packet
    uint32_t tro;  // trailer offset from the block base (lane 8g of a packet, last frame), else OOR
    uint64_t boff; // uniform (TRAILER only)
    uint32_t fl;   // uniform: the frame descriptor (kOct* flags, rrem in bits 24-31), 0 if empty
};

// The row steps of one frame.  FIRST: rows 0..2 carry the header masks and row 0 starts the
// accumulators; UNI: no per-lane freeze; FULL: all K rows (else rows past S.rrem are skipped, a
// uniform branch per row).
// A slot's rows from its row 0 (the freeze count): OctSlot::rl, or (PK, the receive kernel) bits
// 16-23 of OctSlot::kf, signed -- one register fewer per slot.
template <bool PK, int MODE, bool TRAILER>
__device__ __forceinline__ int slot_rows(const OctSlot<MODE, TRAILER> &S) {
    return PK ? __builtin_amdgcn_sbfe(S.kf, 16, 8) : S.rl;
}

template <bool FIRST, bool UNI, bool FULL, int MODE, bool TRAILER, bool PK = false>
__device__ __forceinline__ uint32_t oct_rows(const OctSlot<MODE, TRAILER> &S, uint32_t acc, uint32_t hm,
                                             const char *lds, const LaneConsts &c) {
    uint32_t m0 = 0, m1 = 0, m2 = 0;
    if constexpr (FIRST) {
        const uint32_t k = static_cast<uint32_t>(S.kf) & 63u;  // negative k wraps to lanes 57..63 (mask 0)
        m0 = bperm(k, hm);
        m1 = bperm((k + 8u) & 63u, hm);
        m2 = bperm((k + 16u) & 63u, hm);
    }
#pragma unroll
    for (int j = 0; j < kOctK; ++j) {
        if (!FULL && j > 0 && j >= static_cast<int>(S.fl >> 24)) break;
        uint32_t u = S.u[j];
        if constexpr (FIRST) {
            if (j == 0) u |= m0;
            if (j == 1) u |= m1;
            if (j == 2) u |= m2;
        }
        const uint32_t nv = (FIRST && j == 0) ? u : step_m64(lds, acc, u, c);
        if constexpr (UNI) acc = nv;
        else acc = j < slot_rows<PK>(S) ? nv : acc;
    }
    return acc;
}

// One frame's rows, dispatched on its (uniform) flags.
template <int MODE, bool TRAILER, class D, bool PK = false>
__device__ __forceinline__ uint32_t oct_frame(const OctSlot<MODE, TRAILER> &S, uint32_t acc, uint32_t hm, const char *lds,
                                              const LaneConsts &c) {
    if constexpr (!D::kRows) {
#pragma unroll
        for (int j = 0; j < kOctK; ++j) acc ^= S.u[j];
        return acc;
    } else {
        switch (S.fl & (kOctFirst | kOctUni | kOctFull)) {
        case kOctFirst | kOctUni | kOctFull: return oct_rows<true, true, true, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        case kOctFirst | kOctFull: return oct_rows<true, false, true, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        case kOctUni | kOctFull: return oct_rows<false, true, true, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        case kOctFull: return oct_rows<false, false, true, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        case kOctFirst | kOctUni:
        case kOctFirst: return oct_rows<true, false, false, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        default: return oct_rows<false, false, false, MODE, TRAILER, PK>(S, acc, hm, lds, c);
        }
    }
}

// Two independent frames stepped interleaved (two accumulator chains: each row step waits on
// LDS lookups, and the other chain's step fills that wait).  Both frames are full and uniform;
// B is the first frame of its set, A the first (FA) or a later one.
template <bool FA, int MODE, bool TRAILER>
__device__ __forceinline__ void oct_rows2(const OctSlot<MODE, TRAILER> &A, const OctSlot<MODE, TRAILER> &B, uint32_t &accA,
                                          uint32_t &accB, uint32_t hm, const char *lds, const LaneConsts &c) {
    uint32_t a0 = 0, a1 = 0, a2 = 0;
    if constexpr (FA) {
        const uint32_t k = static_cast<uint32_t>(A.kf) & 63u;
        a0 = bperm(k, hm);
        a1 = bperm((k + 8u) & 63u, hm);
        a2 = bperm((k + 16u) & 63u, hm);
    }
    const uint32_t kb = static_cast<uint32_t>(B.kf) & 63u;
    const uint32_t b0 = bperm(kb, hm), b1 = bperm((kb + 8u) & 63u, hm), b2 = bperm((kb + 16u) & 63u, hm);
    uint32_t xa = accA, xb = 0;
#pragma unroll
    for (int j = 0; j < kOctK; ++j) {
        uint32_t ua = A.u[j], ub = B.u[j];
        if constexpr (FA) {
            if (j == 0) ua |= a0;
            if (j == 1) ua |= a1;
            if (j == 2) ua |= a2;
        }
        if (j == 0) ub |= b0;
        if (j == 1) ub |= b1;
        if (j == 2) ub |= b2;
        xa = (FA && j == 0) ? ua : step_m64(lds, xa, ua, c);
        xb = j == 0 ? ub : step_m64(lds, xb, ub, c);
    }
    accA = xa;
    accB = xb;
}

// The kernel's measurement policy.  The product instantiates OctProduct: every step real.  The
// A/B library (ICRC_AB_BUILD) also instantiates OctAblation<X> (variants 41-53), each switching
// one part off or replacing it, so that a part's cost can be measured on the same build
// (results wrong by design except 48, 49, 51-53).
struct OctProduct {
    static constexpr bool kLoads = true;       // the row loads (else: synthetic rows, no memory)
    static constexpr bool kRows = true;        // the row steps (else: the rows XOR-folded)
    static constexpr bool kFinal = true;       // the final products M^(8 - c)
    static constexpr bool kStores = true;      // result and trailer stores
    static constexpr bool kSetPerm = true;     // a set's per-lane packet data from the sorted block entries
    static constexpr bool kArithSetup = false; // ... or computed from the index (strided batches only)
    static constexpr bool kPrio = true;        // raised wave priority over a frame's setup and loads
    static constexpr bool kReusePrep = false;  // the first block's preparation reused (strided, full blocks)
    static constexpr bool kStamp = false;      // each wave stamps start / end times over its first results
    static constexpr bool kRxDeposit = true;   // RX: header words into the record
    static constexpr bool kRxDecode = true;    // RX: the block decode and its stores
    static constexpr bool kRxStoreOOR = false; // RX: ... its global stores issued out of range (dropped)
    static constexpr bool kRxWrBarrier = true; // RX: a scheduling barrier after each record write of the decode
    static constexpr bool kRxX4 = false;       // RX: the descriptors leave as 16-byte stores (else dword stores)
    static constexpr int kRxStoreAux = kStreamAux;  // RX: the descriptor stores' cache policy (nt: -2.5 %, rx_oct_ab)
    static constexpr bool kRxDefer = false;    // RX: the descriptor stores after the next pair's loads
};
#ifdef ICRC_AB_BUILD
// 41 loads only; 42 row steps, no loads; 43 control and final products; 44 control only; 45 = 41
// without stores; 46 the full kernel without stores; 47 without final products; 48 each set's
// packet data from the lane's own block entry; 49 / 50 the full kernel / loads only with the
// packet data computed from the index; 51 without the raised priority; 52 the block preparation
// reused; 53 with start / end stamps (scripts/probe_oct_balance.py).
template <int X>
struct OctAblation : OctProduct {
    static constexpr bool kLoads = !(X == 2 || X == 3 || X == 4);
    static constexpr bool kRows = !(X == 1 || X == 3 || X == 4 || X == 5 || X == 10);
    static constexpr bool kFinal = !(X == 1 || X == 4 || X == 5 || X == 7 || X == 10);
    static constexpr bool kStores = !(X == 5 || X == 6);
    static constexpr bool kSetPerm = X != 8;
    static constexpr bool kArithSetup = X == 9 || X == 10;
    static constexpr bool kPrio = X != 11;
    static constexpr bool kReusePrep = X == 12;
    static constexpr bool kStamp = X == 13;
};
// The receive kernel's cuts and alternatives (ICRC_AB_RX_OCT=2..8): 2 no record writes, 3 no block
// decode / stores, 4 neither (the 16-copy verify alone), 5 the decode with every global store out
// of range; 6 the descriptor stores without the non-temporal hint, 7 (= the product), 8 16-byte
// non-temporal descriptor stores; 9 the descriptor stores deferred past the next pair's loads.
template <int X>
struct OctRxAblation : OctProduct {
    static constexpr bool kRxDeposit = !(X == 2 || X == 4);
    static constexpr bool kRxDecode = !(X == 3 || X == 4);
    static constexpr bool kRxStoreOOR = X == 5;
    static constexpr bool kRxX4 = X == 8;
    static constexpr bool kRxDefer = X == 9;
    static constexpr int kRxStoreAux = (X == 6 || X == 5) ? 0 : kStreamAux;
};
#endif

// ---- the fused receive (RX: verify + strip + parse in the oct kernel, icrc_oct_rx_kernel) ------
// The two-pass receive re-reads every packet's header lines after the verify (~1.4 128-B lines per
// 316-B packet: 0.18 of its 0.45 ms on 4 Mi x 316 B).  Here the verify waves keep what they load:
// a set's first frame holds packet words 7..17 (BTH and extension headers) in rows 1..3, and each
// lane writes its words into the wave's LDS block record; when a block's last set is done the wave
// decodes its 64 packets lane = packet (rx_decode's fields) IN the record, then stores the 64
// descriptors (4608 contiguous bytes) as 18 coalesced dword stores.  (Stored lane = packet, 72 B
// apart, the same descriptors made the pass 2.4x slower than the verify, 16-byte stores 1.6x:
// profiles/r05/rx_oct_ab.jsonl.)
//
// LDS map of the receive kernel: the bulk tables with 16 bank copies in the lower halves of the
// 512 table rows of 256 B (scripts/stepbench.hip: no slower than 32 copies on the oct shape), the
// final tables of lanes 0..31 in the upper halves of rows 0..127 (c.fin = 128 + (lane & 31) * 4,
// final_mul unchanged; lanes l and l + 32 share a bank), and per wave a record of 19 rows of 64
// packets (row stride 512 B, packets 32..63 256 B on): waves 0..9 in the upper halves of table
// rows 128..507, waves 10..15 two by two in the old final-table region.  Row k = dword k of the
// packets' descriptors; before the decode, header word w sits in the row of the dword formed from
// it (kRxHdrRows), so the decode reads and writes each row in place; row 18 takes a deposit lane's
// unused writes (entries 0..31) and, ragged batches, the base offsets of the wave's last eight
// prepared blocks (entries 32..47, written when a block is prepared, read by its decode; at most
// six blocks lie between the two).  Ragged batches also deposit each packet's offset from its
// block's base and its length into rows 4 and 6 (dwords computed from them, rewritten last).  One record per wave: a block's words are written when its sets' first frames are
// consumed, decoded and stored when its last frame is, and the next block's first frame is
// consumed after that (consume orders deposit / finish / stores per slot).
constexpr uint32_t kRxRows = 19u, kRxRecRow = 512u, kRxDummyRow = 18u;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// header word 7 + i -> record row: nibble i (7->15 8->12 9->13 10->14 11->0 12->7 13->8 14->11
// 15->2 16->9 17->10)
constexpr uint64_t kRxHdrRows = 0xA92B870EDCFull;
__device__ __forceinline__ uint32_t rx_wave_base(uint32_t w) {
    return w < 10u ? (128u + 38u * w) * 256u + 128u
                   : kFinalBase + ((w - 10u) >> 1) * (kRxRows * kRxRecRow) + ((w - 10u) & 1u) * 128u;
}
// Packet i of record row k, rotated by 2 k within its 32-packet half: the decode (lane = packet, one
// row) reads 32 banks either way, and the transposing read-back -- whose 32 lanes take ~18 rows of
// two packets -- hits ~2 lanes per bank instead of ~18 (68 LDS cycles over its 18 reads against 640).
// v, opaque to the optimiser: values derived from it inside the ring loop are recomputed there
// instead of being hoisted out of it and held (the receive ring has no registers to spare: a held
// lane constant spills, and a reload in the ring waits for every load before it).
__device__ __forceinline__ uint32_t rx_opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t rx_ent(uint32_t i, uint32_t k) {
    return k * kRxRecRow + ((i >> 5) << 8) + (((i + 2u * k) & 31u) << 2);
}

template <int MODE, bool RAGGED, bool TRAILER, class D, bool RX = false>
__device__ __forceinline__ void run_oct(const BatchParams &p, const char *lds, const LaneConsts &c, uint32_t lane,
                                        uint32_t lo, uint32_t nq) {
    constexpr bool kPrio = kOctPrio && D::kPrio;
    constexpr int K = kOctK;
    constexpr int P = kOctPairs;  // ring positions, two frames (slots 2 p, 2 p + 1) each
    constexpr int B = 2 * P;
    if (nq == 0) return;
    const uint64_t t_start = D::kStamp ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const int nblocks = static_cast<int>((nq + 63u) >> 6);
    const uint32_t grp = lane >> 3;
    const int col = static_cast<int>(lane & 7u);
    const uint32_t hm = head_mask(static_cast<int>(lane));  // lane k: the mask of stream word k
    bool irregular = false;

    // next block NB, prepared at the top of a ring cycle from the (offset, len) loaded the cycle before
    OctBlock NB;
    int nb_next = 0, mblk = -1;
    bool nb_ready = false;
    uint32_t m_lo = 0, m_hi = 0, m_len = 0;

    // load side: the block being issued (LB), its next frame (lt of lnfr) and the current set's
    // per-lane data (set up at the set's first frame)
    OctBlock LB;
    LB.nfr = 0;
    LB.block = 0;
    LB.boff = 0;
    LB.bend = 0;
    LB.pos = 0xFFu;
    int lt = 0, lnfr = 0;
    bool lreal = false, ldone = false;
    int lkf = 0, lr = 0;
    uint32_t lvrow0 = 0, ltr = kOctOOR;
    uint32_t lidx = 0;  // RX: the packet's index in its block, | 64 if real
    int inflight = 0;
    // RX: the wave's record
    const uint32_t rx_wb = RX ? rx_wave_base(readfirstlane_u32(threadIdx.x >> 6)) : 0u;
    const uint32_t lane_ = lane;  // (the block preparation's lane, opaque there under RX)

    OctSlot<MODE, TRAILER> sl[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {  // every slot's stores run from the first cycle: all out of range
        sl[b].fl = 0u;
        sl[b].rq = kOctOOR;
        sl[b].tro = kOctOOR;
        sl[b].rt = 0xFFu;
        sl[b].boff = 0;
    }

    uint32_t acc_c = 0;  // accumulator carried from frame to frame
    uint32_t rbv = 0;    // the block result register (lane i = packet i of the block)
    // finished blocks' results, not yet stored: entry e in rres[e] (the newest in rres[kOctRes -
    // 1]), bit e of rown set where this lane's packet of entry e is this kernel's, lane e of rblk
    // the entry's block; nres entries held
    uint32_t rres[kOctRes];
#pragma unroll
    for (int e = 0; e < kOctRes; ++e) rres[e] = 0;
    uint32_t rown = 0, rblk = 0;
    int nres = 0;
    // store entries [kOctRes - nres, kOctRes)
    auto flush = [&]() __attribute__((always_inline)) {
        if constexpr (!D::kStores) return;
        const int e0 = kOctRes - nres;
        const __amdgpu_buffer_rsrc_t os =
            MODE == kCompute
                ? __builtin_amdgcn_make_buffer_rsrc(p.out ? p.out + lo : nullptr, 0, p.out ? static_cast<int>(nq * 4u) : 0, 0x00020000)
                : __builtin_amdgcn_make_buffer_rsrc(p.ok ? p.ok + lo : nullptr, 0, p.ok ? static_cast<int>(nq) : 0, 0x00020000);
#pragma unroll
        for (int e = 0; e < kOctRes; ++e) {
            if (e >= e0) {
                const uint32_t q = readlane_u32(rblk, e) * 64u + lane;
                const uint32_t o = ((rown >> e) & 1u) ? q * (MODE == kCompute ? 4u : 1u) : kOctOOR;
                if constexpr (MODE == kCompute) __builtin_amdgcn_raw_buffer_store_b32(rres[e], os, static_cast<int>(o), 0, 0);
                else __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(rres[e]), os, static_cast<int>(o), 0, 0);
            }
        }
    };

    auto issue = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        OctSlot<MODE, TRAILER> &S = sl[b];
        if constexpr (kPrio) __builtin_amdgcn_s_setprio(3);  // the frame's setup gates its loads
        if (lt >= lnfr) {  // the block is issued: the next one, if prepared
            if (nb_ready) {
                LB = NB;
                nb_ready = false;
                lt = 0;
                lnfr = LB.nfr;
            } else if (nb_next >= nblocks) {
                ldone = true;
            }  // else a stall: the next block is prepared at the top of the next cycle
        }
        const bool have = lt < lnfr;
        const uint32_t fd = have ? readfirstlane_u32(readlane_u32(LB.ftab, lt)) : 0u;
        const uint32_t set = fd & kFdSet;
        if (fd & kOctFirst) {  // set setup: this lane's packet is sorted position 8 set + grp
            const uint32_t ps = 8u * set + grp;
            uint32_t key, vrel, L;
            if constexpr (D::kArithSetup) {
                L = p.ulen;
                key = (((stream_words<MODE>(L) + 7u) >> 3) << 6) | ps;
                vrel = ps * static_cast<uint32_t>(p.stride);
            } else {
                key = D::kSetPerm ? bperm(ps, LB.key) : LB.key;
                vrel = D::kSetPerm ? bperm(ps, LB.vrel) : LB.vrel;
                L = D::kSetPerm ? bperm(ps, LB.len) : LB.len;
            }
            lreal = ps < static_cast<uint32_t>(__popcll(LB.mine));
            const uint32_t N = stream_words<MODE>(L);
            const int z = static_cast<int>((8u - (N & 7u)) & 7u);
            lr = static_cast<int>(key >> 6);
            lkf = col - z;
            lvrow0 = vrel + 4u * static_cast<uint32_t>(lkf - 1);
            ltr = (lreal && col == 0) ? vrel + L - 4u : kOctOOR;
            if constexpr (RX) lidx = (key & 63u) | (lreal ? 64u : 0u);
        }
        const uint32_t lf = (fd >> 16) & 0xFFu;
        const uint32_t fo = 32u * K * lf;
        // (Rows past a shorter packet's end in a set of mixed row counts re-read the bytes after it:
        // those are the block's next packets, which the same wave reads soon after, so the
        // over-read acts as their L2 prefetch — skipping the frames past a lane's own packet
        // measured no faster, profiles/r04_ab_oct_frame_skip_rejected.jsonl.)
        const bool live = have && lreal;
        const uint32_t o0 = (live && lkf + 8 * K * static_cast<int>(lf) >= 1) ? lvrow0 + fo : kOctOOR;
        const uint32_t o1 = live ? lvrow0 + 32u + fo : kOctFar;  // rows >= 1: + 32 (j - 1) immediate
        // (readfirstlane: the block fields are uniform, but hipcc's divergence analysis loses track
        // of them through the ring's phis and wraps every load in a waterfall loop otherwise)
        const uint64_t boff = static_cast<uint64_t>(readfirstlane_u32(static_cast<uint32_t>(LB.boff))) |
                              (static_cast<uint64_t>(readfirstlane_u32(static_cast<uint32_t>(LB.boff >> 32))) << 32);
        uint8_t *bb = p.base + boff;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(bb, 0, static_cast<int>(readfirstlane_u32(LB.bend)), 0x00020000);
        if constexpr (!D::kLoads) {
#pragma unroll
            for (int j = 0; j < K; ++j) S.u[j] = (o1 + 32u * j) * 0x9E3779B1u;
        } else {
            // Rows past the set's last row (the tail frame of a set whose rows are not a multiple
            // of K) are never stepped: they re-load the last real row instead of the bytes after
            // the packet.  The row step rides in the scalar offset, clamped on the scalar unit
            // (rrem is uniform), so the loads stay unconditional and the clamp costs no VALU;
            // before, those rows fetched the next packets' lines again (C2 FETCH 1.21x the
            // algorithmic bytes, the 1 KiB class 1.26x: profiles/r03_pmc_c2_fetch.txt).
            const uint32_t rrem = fd >> 24;
            const uint32_t cap = 32u * (rrem > 2u ? rrem : 2u) - 64u;  // rows 1..rrem-1 real (no select chain)
            S.u[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(o0), 0, 0);
#pragma unroll
            for (int j = 1; j < K; ++j) {
                const uint32_t so = kOctClampRows ? (32u * (j - 1) < cap ? 32u * (j - 1) : cap) : 32u * (j - 1);
                S.u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(o1), static_cast<int>(so), 0);
            }
            if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
        }
        const bool last = (fd & kOctLast) != 0u;
        // (RX: the packet's block index in bits 8-13, bit 14 set for a real packet, the rows from this
        // frame's row 0 in bits 16-23 (slot_rows); readers mask & 63)
        if constexpr (RX) {
            const uint32_t rl = static_cast<uint32_t>(lr - K * static_cast<int>(lf)) & 0xFFu;
            S.kf = static_cast<int>((static_cast<uint32_t>(lkf) & 63u) | (lidx << 8) | (rl << 16));
        } else {
            S.kf = lkf;
            S.rl = lr - K * static_cast<int>(lf);
        }
        if constexpr (!RX) S.tro = last ? ltr : kOctOOR;  // (RX: the block's trailers are zeroed with its descriptors)
        else if constexpr (RAGGED) S.tro = lvrow0 + 4u - 4u * static_cast<uint32_t>(lkf);  // RX: the packet's offset from boff
        // routing: packet i of the block (pos_i = its sorted position, 0xFF if not this kernel's)
        // takes group (pos_i & 7)'s result at the last frame of set pos_i >> 3
        const uint32_t pi = LB.pos;
        S.rt = (last && (pi >> 3) == set) ? (pi & 7u) << 3 : 0xFFu;
        // the block (uniform) in bits 0-30, bit 31: this lane's packet is not this kernel's
        S.rq = static_cast<uint32_t>(LB.block) | (pi != 0xFFu ? 0u : kOctOOR);
        if constexpr (TRAILER) S.boff = boff;
        S.fl = fd;
        lt += have ? 1 : 0;
        inflight += have ? 1 : 0;
    };

    // RX: a set's first frame -> its packets' words 7..17 (raw, before the header masks) into the
    // wave's record.  Lane c of row j holds stream word 8 j + kf = packet word 8 j + kf - 1; it is
    // written when that is one of 7..17 and not the trailer or past it (row index 8 j + c below
    // 8 R - 1).  Every lane writes (a lane with nothing to write: its dummy entry), no branch
    // around an LDS store.
    auto deposit = [&](const OctSlot<MODE, TRAILER> &S) __attribute__((always_inline)) {
        if constexpr (RX && D::kRxDeposit) {
            if (!(S.fl & kOctFirst)) return;
            char *rec = const_cast<char *>(lds);
            const uint32_t kx = static_cast<uint32_t>(S.kf);
            const int kf = static_cast<int>((kx & 63u) ^ 32u) - 32;
            const uint32_t idx = (kx >> 8) & 63u;
            const bool real = (kx >> 14) & 1u;
            const uint32_t ln = rx_opaque(lane);
            const uint32_t dummy = rx_wb + rx_ent(ln & 31u, kRxDummyRow);
            const int rows8 = 8 * slot_rows<true>(S);
#pragma unroll
            for (int j = 1; j <= 3; ++j) {
                const int pw = 8 * j + kf - 1;
                const bool w = real && pw >= 7 && pw <= 17 && 8 * j + col + 1 < rows8;
                const uint32_t row = static_cast<uint32_t>(kRxHdrRows >> (4u * (static_cast<uint32_t>(pw - 7) & 15u))) & 15u;
                *reinterpret_cast<uint32_t *>(rec + (w ? rx_wb + rx_ent(idx, row) : dummy)) = S.u[j];
            }
            if constexpr (RAGGED) {  // lane 8 g: the offset from boff (row 4); 8 g + 1: L = 4 (N - 1), N = 8 R - c + kf
                const uint32_t Lp = 4u * static_cast<uint32_t>(rows8 - col + kf) - 4u;
                const bool w = real && col < 2;
                *reinterpret_cast<uint32_t *>(rec + (w ? rx_wb + rx_ent(idx, col == 0 ? 4u : 6u) : dummy)) = col == 0 ? S.tro : Lp;
            }
        }
    };
    // RX: the block's descriptors, decoded lane = packet in the record (rx_decode's fields; ok = the
    // verify result finish left in row 17; each row read before it is rewritten), then transposed on the way out:
    // dword g = 64 t + lane of the block's 4608 bytes is dword g % 18 of packet g / 18.  The ok
    // bytes (and, zero_trailer, the zeroed trailers) leave with them.
    // RX: the read-back of a decoded block (packets base .. base + cnt - 1): dword g = 64 t + lane of
    // its 4608 bytes is dword g % 18 of packet g / 18; 18 coalesced stores.
    uint32_t rx_pbase = 0, rx_pcnt = 0;
    bool rx_pend = false;
    auto rx_readback = [&](uint32_t base, uint32_t cnt) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<uint8_t *>(p.rx + base), 0, D::kRxStoreOOR ? 0 : static_cast<int>(cnt * 72u), 0x00020000);
        if constexpr (D::kRxX4) {
            // chunk c = 64 t + lane (16 bytes, dwords 4 c .. 4 c + 3 of the block) per store
            uint32_t pk = (4u * lane * 3641u) >> 16, kk = 4u * lane - 18u * pk;  // 4 lane / 18, 4 lane % 18
            asm volatile("" : "+v"(pk), "+v"(kk));
#pragma clang loop unroll(disable)
            for (uint32_t t = 0; t < 5; ++t) {
                u32x4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = lds_at(lds, rx_wb + rx_ent(pk, kk));
                    ++kk;
                    pk += kk == 18u ? 1u : 0u;
                    kk = kk == 18u ? 0u : kk;
                }
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, static_cast<int>((64u * t + lane) * 16u), 0, D::kRxStoreAux);
                pk += 14u;  // + 256 dwords = 18 x 14 + 4 (the 4 stepped above)
            }
        } else {
            uint32_t pk = (lane * 3641u) >> 16, kk = lane - 18u * pk;  // lane / 18 (exact below 64), lane % 18
            // (opaque here: otherwise the 18 addresses, which depend on the lane alone, are hoisted out of
            // the ring loop and held in 18 registers)
            asm volatile("" : "+v"(pk), "+v"(kk));
            // (a loop, not unrolled: this runs four times inlined in the ring, whose code already
            // fills most of the instruction cache)
#pragma clang loop unroll(disable)
            for (uint32_t t = 0; t < 18; ++t) {
                const uint32_t v = lds_at(lds, rx_wb + rx_ent(pk, kk));
                __builtin_amdgcn_raw_buffer_store_b32(v, rs, static_cast<int>((64u * t + lane) * 4u), 0, D::kRxStoreAux);
                kk += 10u;  // g + 64 = 18 (pk + 3) + kk + 10
                pk += 3u;
                pk += kk >= 18u ? 1u : 0u;
                kk -= kk >= 18u ? 18u : 0u;
            }
        }
    };
    auto rx_block = [&](const OctSlot<MODE, TRAILER> &S, bool can_defer) __attribute__((always_inline)) {
        if constexpr (RX && D::kRxDecode) {
            char *rec = const_cast<char *>(lds);
            const uint32_t blk = S.rq & 0x7FFFFFFFu;
            const bool mine = (S.rq >> 31) == 0u;
            const uint32_t base = lo + blk * 64u;
            const uint32_t cnt = nq - blk * 64u < 64u ? nq - blk * 64u : 64u;  // (strided: all of them this kernel's)
            const uint32_t ln = rx_opaque(lane);
            auto rd = [&](uint32_t r) __attribute__((always_inline)) { return lds_at(lds, rx_wb + rx_ent(ln, r)); };
            auto wr = [&](uint32_t r, uint32_t v) __attribute__((always_inline)) {  // (sched_barrier: few live registers)
                *reinterpret_cast<uint32_t *>(rec + rx_wb + rx_ent(ln, r)) = v;
                if constexpr (D::kRxWrBarrier) __builtin_amdgcn_sched_barrier(0);
            };
            // the packet's length (ragged: record row 6, read again where needed: short live ranges)
            auto len = [&]() __attribute__((always_inline)) { return RAGGED ? rd(6) : p.ulen; };
            // Per lane, one register: hs (bits 0-5), pad (8-9), status (16-17), and which fields
            // the packet has (bits 24-28: ok, RETH, secondary RETH, immediate, AETH); the selects
            // are bit-field masks, not lane masks (the ring leaves few SGPRs).
            uint32_t meta;
            {
                const uint32_t w7 = rd(15);
                const uint32_t op = w7 & 0x1Fu, tran = (w7 >> 5) & 7u, pad = (w7 >> 13) & 3u;
                const uint32_t hs = (op == 0x09u || op == 0x0Bu) ? 32u
                                  : (op == 0x0Cu)                 ? 44u
                                  : (op == 0x11u)                 ? 16u
                                  : (op >= 0x06u && op <= 0x10u)  ? 28u
                                                                  : 0u;
                const uint32_t status = (hs == 0u)           ? ICRC_RX_INVALID_OPCODE
                                      : (tran > 6u)          ? ICRC_RX_INVALID_TRANS_TYPE
                                      : (len() - 32u < hs + pad) ? ICRC_RX_TRUNCATED
                                                                 : ICRC_RX_OK;  // (L >= 44: this kernel's packets)
                const uint32_t okb = status == ICRC_RX_OK ? 1u : 0u;
                const uint32_t cls = okb | (hs != 16u ? 2u : 16u) | (hs == 44u ? 4u : 0u) | (hs == 32u ? 8u : 0u);
                meta = hs | (pad << 8) | (status << 16) | ((okb ? cls : 0u) << 24);
            }
            auto keep = [&](int bit, uint32_t v) __attribute__((always_inline)) {  // v if the packet has field `bit`
                return v & static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(meta), 24 + bit, 1));
            };
            const uint32_t hs = meta & 63u, pad = (meta >> 8) & 3u;
            {   // the dwords formed from words 7, 9, 10 first (rows 13-15 are rewritten here)
                const uint32_t w7 = rd(15), w9 = rd(13), w10 = rd(14);
                const uint32_t fl = (w7 >> 8) & 0xFFu;
                const bool ack = hs == 16u;
                const uint32_t flags = ((fl & 0x80u) ? ICRC_RX_SOLICITED : 0u) | ((w9 & 0x80u) ? ICRC_RX_ACK_REQ : 0u) |
                                       (ack ? ICRC_RX_ACKNOWLEDGE : 0u) | (hs == 32u ? ICRC_RX_HAS_IMM : 0u) |
                                       (hs == 44u ? ICRC_RX_HAS_SECONDARY_RETH : 0u);
                const uint32_t code = ack ? (w10 >> 5) & 3u : 0u, value = ack ? w10 & 0x1Fu : 0u;
                wr(16, keep(0, flags | (pad << 8) | (code << 16) | (value << 24)));
                wr(1, keep(1, bswap32(w10)));                                   // RETH va high: word 10
                wr(14, keep(4, bswap32(w10) & 0xFFFFFFu));                       // AETH msn
                wr(13, keep(0, bswap32(w9) & 0xFFFFFFu));                        // psn
                wr(15, keep(0, bswap16(w7 >> 16) | ((w7 & 0x1Fu) << 16) | (((w7 >> 5) & 7u) << 24)));  // pkey, opcode, transport
            }
            wr(17, (rd(17) & 0xFFu) | (meta & 0x30000u) >> 8);  // icrc_ok (finish left it there), status
            wr(0, keep(1, bswap32(rd(0))));   // RETH va low: word 11
            wr(2, keep(2, bswap32(rd(2))));   // secondary RETH va (bytes 56-63): words 15, 14
            wr(3, keep(2, bswap32(rd(11))));
            wr(11, keep(3, bswap32(rd(11))));  // immediate: word 14
            wr(7, keep(1, bswap32(rd(7))));    // rkey, dlen: words 12, 13
            wr(8, keep(1, bswap32(rd(8))));
            wr(9, keep(2, bswap32(rd(9))));    // secondary rkey, dlen: words 16, 17
            wr(10, keep(2, bswap32(rd(10))));
            wr(12, keep(0, bswap32(rd(12)) & 0xFFFFFFu));  // dqpn: word 8
            uint64_t boff = 0;  // ragged: the block's base offset (the ring in row 18) + record row 4
            if constexpr (RAGGED) {
                const uint32_t e = rx_wb + rx_ent(32u + 2u * (blk & 7u), kRxDummyRow);
                boff = static_cast<uint64_t>(readfirstlane_u32(lds_at(lds, e))) |
                       (static_cast<uint64_t>(readfirstlane_u32(lds_at(lds, e + 4u))) << 32);
            }
            if constexpr (TRAILER) {  // is_icrc_valid zeroes the trailer (strided: stride <= 16 MiB, offsets below 1 GiB)
                const __amdgpu_buffer_rsrc_t ts = __builtin_amdgcn_make_buffer_rsrc(
                    p.base + (RAGGED ? boff : static_cast<uint64_t>(base) * p.stride), 0, static_cast<int>(kOctOOR), 0x00020000);
                const uint32_t to = (RAGGED ? rd(4) : ln * static_cast<uint32_t>(p.stride)) + len() - 4u;
                __builtin_amdgcn_raw_buffer_store_b32(0u, ts, static_cast<int>(mine ? to : kOctOOR), 0, 0);
            }
            wr(6, keep(0, len() - 32u - hs - pad));  // (ragged: row 6 held L until here)
            {
                const uint64_t poff = (RAGGED ? boff + rd(4) : static_cast<uint64_t>(base + ln) * p.stride) + 28u + hs;
                wr(4, keep(0, static_cast<uint32_t>(poff)));
                wr(5, keep(0, static_cast<uint32_t>(poff >> 32)));
            }
            const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(
                p.ok ? p.ok + lo : nullptr, 0, p.ok && !D::kRxStoreOOR ? static_cast<int>(nq) : 0, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(rd(17)), os, static_cast<int>(mine ? blk * 64u + ln : kOctOOR), 0, 0);
            // The descriptor stores now, or (D::kRxDefer) at the start of the next consume, after the
            // next pair's loads: a store sits in the load queue, and there it must complete one ring
            // step later instead of at the next wait.  Deferred only when no deposit follows in this
            // consume (the record is read back before it is rewritten).
            if (D::kRxDefer && can_defer) {
                rx_pend = true;
                rx_pbase = base;
                rx_pcnt = cnt;
            } else {
                rx_readback(base, cnt);
            }
        }
    };

    // the result of a slot's set (its last frame): ICRC / verify result, routed into rbv
    auto finish = [&](const OctSlot<MODE, TRAILER> &S, uint32_t crc) __attribute__((always_inline)) {
        uint32_t r;
        if constexpr (MODE == kCompute) r = crc;
        else r = crc == kIcrcResidue ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH;  // over the trailer too
        if constexpr (RX) {  // lane 8 g: into record row 17 of its packet (the block's decode reads it there)
            const uint32_t kx = static_cast<uint32_t>(S.kf);
            const bool w = ((kx >> 14) & 1u) && col == 0;
            const uint32_t a = rx_wb + (w ? rx_ent((kx >> 8) & 63u, 17u) : rx_ent(rx_opaque(lane) & 31u, kRxDummyRow));
            *reinterpret_cast<uint32_t *>(const_cast<char *>(lds) + a) = r;
        } else {
            const uint32_t v = bperm(S.rt & 63u, r);
            rbv = S.rt != 0xFFu ? v : rbv;
        }
    };
    // a slot's stores, issued whether or not it holds a frame (out of range otherwise: no branch
    // around a store in the ring)
    auto stores = [&](const OctSlot<MODE, TRAILER> &S, uint32_t crc, bool can_defer) __attribute__((always_inline)) {
        if constexpr (!D::kStores) return;
        if (TRAILER && !RX && (S.fl & kOctLast)) {  // PacketWriter stores the ICRC / is_icrc_valid zeroes it
            const __amdgpu_buffer_rsrc_t ts =
                __builtin_amdgcn_make_buffer_rsrc(p.base + S.boff, 0, static_cast<int>(kOctOOR), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(MODE == kCompute ? crc : 0u, ts, static_cast<int>(S.tro), 0, 0);
        }
        // the block's results are complete after its last set: into the register buffer, which
        // is stored when full (and after the ring)
        if (!(S.fl & kOctBlockLast)) return;
        if constexpr (RX) {  // the ok bytes leave with the block's descriptors (no result buffer)
            rx_block(S, can_defer);
            return;
        }
#pragma unroll
        for (int e = 0; e + 1 < kOctRes; ++e) rres[e] = rres[e + 1];
        rres[kOctRes - 1] = rbv;
        rown = (rown >> 1) | ((S.rq >> 31) ? 0u : 1u << (kOctRes - 1));
        // lane e <- lane e + 1 (DPP wave_shl:1), the new entry's block in lane kOctRes - 1
        rblk = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(rblk), 0x130, 0xF, 0xF, false));
        rblk = lane == kOctRes - 1 ? (S.rq & 0x7FFFFFFFu) : rblk;
        if (++nres == kOctRes) {
            flush();
            nres = 0;
        }
    };

    // Consume slots a (older) and a + 1.  If the second starts a new set the two frames are
    // independent and, when both are full and uniform, stepped interleaved.
    auto consume = [&](auto ac) __attribute__((always_inline)) {
        constexpr int a = decltype(ac)::value;
        if constexpr (RX && D::kRxDefer) {
            if (rx_pend) {
                rx_readback(rx_pbase, rx_pcnt);
                rx_pend = false;
            }
        }
        OctSlot<MODE, TRAILER> &SA = sl[a];
        OctSlot<MODE, TRAILER> &SB = sl[a + 1];
        const uint32_t fa = SA.fl, fb = SB.fl;
        constexpr uint32_t kFast = kOctHave | kOctUni | kOctFull;
        uint32_t accA = acc_c, accB = 0;
        if (D::kRows && (fa & kFast) == kFast && (fb & (kFast | kOctFirst)) == (kFast | kOctFirst)) {
            if (fa & kOctFirst) oct_rows2<true>(SA, SB, accA, accB, hm, lds, c);
            else oct_rows2<false>(SA, SB, accA, accB, hm, lds, c);
        } else {
            if (fa & kOctHave) accA = oct_frame<MODE, TRAILER, D, RX>(SA, accA, hm, lds, c);
            if (fb & kOctHave) accB = oct_frame<MODE, TRAILER, D, RX>(SB, (fb & kOctFirst) ? 0u : accA, hm, lds, c);
        }
        acc_c = (fb & kOctHave) ? accB : accA;
        uint32_t crcA = 0, crcB = 0;
        if (fa & fb & kOctLast) {  // both sets end here: the two final products interleave
            crcA = ~group_xor<8>(D::kFinal ? final_mul(lds, accA, c.fin) : accA);
            crcB = ~group_xor<8>(D::kFinal ? final_mul(lds, accB, c.fin) : accB);
        } else if (fa & kOctLast) {
            crcA = ~group_xor<8>(D::kFinal ? final_mul(lds, accA, c.fin) : accA);
        } else if (fb & kOctLast) {
            crcB = ~group_xor<8>(D::kFinal ? final_mul(lds, accB, c.fin) : accB);
        }
        inflight -= ((fa & kOctHave) ? 1 : 0) + ((fb & kOctHave) ? 1 : 0);
        // A's results (and its block's result store) before B's routing touches rbv: B may hold
        // the next block's first set
        // (RX: a slot's words reach the record before its block's decode, and B's -- possibly the next
        // block's first set -- only after A's decode)
        deposit(SA);
        if (fa & kOctLast) finish(SA, crcA);
        stores(SA, crcA, !(fb & kOctFirst));
        deposit(SB);
        if (fb & kOctLast) finish(SB, crcB);
        stores(SB, crcB, true);
    };

    int cycles = 0;
    bool bailed = false;
    for (;;) {
        // top of the cycle: prepare the next block, then fetch the (offset, len) of the one after
        if (!nb_ready && nb_next < nblocks && (!RAGGED || mblk == nb_next)) {
            const uint32_t lane = RX ? rx_opaque(lane_) : lane_;  // (RX: rx_opaque)
            const uint32_t q = static_cast<uint32_t>(nb_next) * 64u + lane;
            const bool valid = q < nq;
            uint64_t off = 0;
            uint32_t L = 0;
            if (valid) {
                off = p.off ? (static_cast<uint64_t>(m_lo) | (static_cast<uint64_t>(m_hi) << 32))
                            : static_cast<uint64_t>(lo + q) * p.stride;
                L = p.len ? m_len : p.ulen;
            }
            if (D::kReusePrep && !RAGGED && nb_next > 0 && (nb_next + 1) * 64 <= static_cast<int>(nq)) {
                // (A/B, strided full blocks) the first block's preparation reused, only its
                // position moved (what a free block schedule would leave)
                NB.block = nb_next;
                NB.boff = static_cast<uint64_t>(lo + static_cast<uint32_t>(nb_next) * 64u) * p.stride;
            } else if (oct_block<MODE>(p, NB, off, L, valid, lo, nb_next, lane) != 0) {
                irregular = true;
            }
            if constexpr (RX && RAGGED) {  // the block's base offset into the record's ring (row 18, entries 32..47)
                const uint32_t e = rx_wb + rx_ent(32u + 2u * (static_cast<uint32_t>(nb_next) & 7u) + (lane & 1u), kRxDummyRow);
                const uint32_t v = (lane & 1u) ? static_cast<uint32_t>(NB.boff >> 32) : static_cast<uint32_t>(NB.boff);
                if (lane < 2u) *reinterpret_cast<uint32_t *>(const_cast<char *>(lds) + e) = v;
            }
            nb_next += 1;
            nb_ready = NB.nfr > 0;
        }
        if constexpr (RAGGED) {  // unconditional: one load pair per cycle keeps vmcnt exact
            const uint32_t q = static_cast<uint32_t>(nb_next) * 64u + lane;
            const __amdgpu_buffer_rsrc_t rs_off = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint64_t *>(p.off ? p.off + lo : nullptr), 0, p.off ? static_cast<int>(nq * 8u) : 0, 0x00020000);
            const __amdgpu_buffer_rsrc_t rs_len = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t *>(p.len ? p.len + lo : nullptr), 0, p.len ? static_cast<int>(nq * 4u) : 0, 0x00020000);
            const auto o = __builtin_amdgcn_raw_buffer_load_b64(rs_off, static_cast<int>(q * 8u), 0, 0);
            m_lo = o[0];
            m_hi = o[1];
            m_len = __builtin_amdgcn_raw_buffer_load_b32(rs_len, static_cast<int>(q * 4u), 0, 0);
            mblk = nb_next;
        }
        static_for<P>([&](auto pc) __attribute__((always_inline)) -> bool {
            constexpr int q = decltype(pc)::value;
            constexpr int n = (q + P - 1) % P;  // the pair issued now is consumed P - 1 positions later
            issue(IntC<2 * n>{});
            issue(IntC<2 * n + 1>{});
            consume(IntC<2 * q>{});
            return true;
        });
        if (ldone && inflight == 0) break;
        // Safety net: a block needs at most 32 frames (8 cycles of 2 P slots) plus a stall cycle;
        // a bookkeeping bug must end in flagged results, never in waves that do not finish.
        if (++cycles > 12 * nblocks + 16) {
            bailed = true;
            break;
        }
    }
    if (nres) flush();
    if (RX && rx_pend) rx_readback(rx_pbase, rx_pcnt);
    // (ragged receive) packets left to the tail loop below: their descriptors are the sweep's
    if (RX && RAGGED && irregular && p.rx_flag && lane == 0) atomicMax(p.rx_flag, p.rx_gen);
    if (bailed) {  // never reached by correct bookkeeping: make it loud, not silent
        for (uint32_t i = lane; i < nq; i += 64u) store_result<MODE>(p, lo + i, MODE == kCompute ? 0u : ICRC_VERIFY_BADLEN);
        if (p.nerr && lane == 0) atomicAdd(p.nerr, nq);
        return;
    }

    if (irregular) {  // L < 44, misaligned, L % 4 != 0, far-apart offsets: per packet
        for (int b = 0; b < nblocks; ++b) {
            uint64_t off;
            uint32_t L;
            uint64_t m = oct_classify<MODE>(p, lo, nq, b, lane, off, L);
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t o = static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off), l)) |
                                   (static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off >> 32), l)) << 32);
                const uint32_t Ll = readlane_u32(L, l);
                const uint32_t r = group_slow_packet<MODE, 8>(p, p.base + o, Ll, lds, c, lane);
                if (lane == 0) store_result<MODE>(p, lo + static_cast<uint32_t>(b) * 64u + static_cast<uint32_t>(l), r);
            }
        }
    }
    if constexpr (D::kStamp && MODE == kCompute) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const __amdgpu_buffer_rsrc_t os =
            __builtin_amdgcn_make_buffer_rsrc(p.out ? p.out + lo : nullptr, 0, p.out ? static_cast<int>(nq * 4u) : 0, 0x00020000);
        const uint32_t v = lane == 0 ? static_cast<uint32_t>(t_start) : lane == 1 ? static_cast<uint32_t>(t_start >> 32)
                         : lane == 2 ? static_cast<uint32_t>(t_end) : static_cast<uint32_t>(t_end >> 32);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_raw_buffer_store_b32(v, os, static_cast<int>(lane < 4u ? lane * 4u : kOctOOR), 0, 0);
    }
}

// The oct kernel's work for workgroup `bid` of `nblk` (its own kernel, or the short-packet
// workgroups of the fused hybrid kernel below).
template <int MODE, bool RAGGED, bool TRAILER, class D>
__device__ __forceinline__ void oct_body(const BatchParams &p, uint4 *lds4, uint32_t bid, uint32_t nblk) {
    const uint32_t tw = nblk * kWavesPerGroup;
    // chunks of whole 64-packet blocks (whole-line result stores) unless that idles waves
    uint32_t chunk = (p.n + tw - 1) / tw;
    chunk = chunk > 32u ? (chunk + 63u) & ~63u : (chunk + 7u) & ~7u;
    if (RAGGED && p.split_len != 0 && p.len != nullptr) {
        // Split batch: a workgroup whose packets are all the long-packet kernel's exits before
        // its 160 KiB table load.
        const uint64_t g0 = static_cast<uint64_t>(bid) * kWavesPerGroup * chunk;
        const uint64_t g1 = g0 + static_cast<uint64_t>(kWavesPerGroup) * chunk;
        const uint64_t end = g1 < p.n ? g1 : p.n;
        if (!wg_any_split<true>(p, lds4, g0, end)) return;
    }
    table_fill(lds4, p.table_oct);
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    uint64_t lo64, hi64;
    wave_range(static_cast<uint64_t>(bid) * kWavesPerGroup * chunk, chunk, wave, p.skew & 0xFFFFu, lo64, hi64);
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = static_cast<uint32_t>((hi64 < p.n ? hi64 : p.n) - lo64);
    run_oct<MODE, RAGGED, TRAILER, D>(p, lds, c, lane, lo, nq);
}

template <int MODE, bool RAGGED, bool TRAILER, class D>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_oct_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    oct_body<MODE, RAGGED, TRAILER, D>(p, lds4, blockIdx.x, gridDim.x);
}

// The hybrid dispatch in ONE launch: workgroups [0, g_oct) are the oct kernel's (L < split_len),
// the rest the long-packet kernel's (L >= split_len).  Each loads its own table image.  Workgroups
// are dispatched in index order, so the long-packet ones take each CU as its oct workgroup
// retires — the overlap the two-stream fork / join gave, without its cross-queue wait (~19 us per
// call, profiles/r02_hybrid_fused.jsonl) or the second launch.
template <int MODE, bool TRAILER, bool COMPACT, class LA = Ring<kStreamAux>>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_hybrid_kernel(BatchParams p, uint32_t g_oct) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    if (blockIdx.x < g_oct) oct_body<MODE, true, TRAILER, OctProduct>(p, lds4, blockIdx.x, g_oct);
    else long_body<MODE, COMPACT, TRAILER, LA>(p, lds4, blockIdx.x - g_oct, gridDim.x - g_oct);
}
// The default ragged dispatch (round 5): ONE set of #CUs workgroups; each runs its oct range, then
// reloads LDS with the W = 64 image and walks the long packets of the same range itself.  Against
// the two sets above (the long-packet workgroups taking CUs as the oct ones retire): configs[2]
// -1.5 %, C1's packets as a ragged batch -0.6 %, identical results (scripts/probe_long_self.py,
// profiles/r05/c2/long_self_ab.jsonl): no second dispatch of 160 KiB workgroups, no tail of them.
template <int MODE, bool TRAILER, bool COMPACT>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_hybrid_self_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    oct_body<MODE, true, TRAILER, OctProduct>(p, lds4, blockIdx.x, gridDim.x);
    __syncthreads();  // every wave is done with the oct image before the long body rewrites LDS
    long_body<MODE, COMPACT, TRAILER>(p, lds4, blockIdx.x, gridDim.x);
}
// The fused receive of strided batches of short packets (icrc_rx_parse_device's default for them):
// the oct verify on the receive kernel's LDS map (above run_oct): bulk entry (b, x) at row
// (b >> 1) * 256 + x, the even table at slot (lane & 15) * 4, the odd one 64 bytes on (thread t
// writes entry t's 16 copies as four 16-byte stores, the k-th at chunk (k + x) & 3).
// The oct half of a receive kernel on workgroup blockIdx.x: the receive image, then run_oct (RX) on
// this wave's range [lo, lo + nq); false if the wave has no range.
template <bool TRAILER, class D, bool RAGGED>
__device__ __forceinline__ bool rx_oct_part(const BatchParams &p, uint4 *lds4, uint32_t &lo, uint32_t &nq) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * kWavesPerGroup;
    uint32_t chunk = (p.n + tw - 1) / tw;
    chunk = chunk > 32u ? (chunk + 63u) & ~63u : (chunk + 7u) & ~7u;
    uint64_t lo64, hi64;
    wave_range(static_cast<uint64_t>(blockIdx.x) * kWavesPerGroup * chunk, chunk, wave, p.skew & 0xFFFFu, lo64, hi64);
    const bool mine = lo64 < p.n;
    lo = mine ? static_cast<uint32_t>(lo64) : 0u;
    nq = mine ? static_cast<uint32_t>((hi64 < p.n ? hi64 : p.n) - lo64) : 0u;
    if (RAGGED && p.split_len != 0 && p.len != nullptr) {
        // A workgroup whose packets are all long skips the ring (and its table image): the sweep
        // takes every packet.
        const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * kWavesPerGroup * chunk;
        const uint64_t g1 = g0 + static_cast<uint64_t>(kWavesPerGroup) * chunk;
        if (!wg_any_split<true>(p, lds4, g0, g1 < p.n ? g1 : p.n)) return mine;
    }
    {   // thread t: bulk entry t's 16 copies (lower half of its table row) and 16 bytes of the final
        // tables (row t >> 3, lanes 4 (t & 7) .. + 3 of the compact form's 64-lane rows)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(p.table_oct + kLdsWords), 0, static_cast<int>(kCompactWords * 4u), 0x00020000);
        const uint32_t bulk = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(4u * threadIdx.x), 0, 0);
        const uint32_t r = threadIdx.x >> 3, q = threadIdx.x & 7u;
        const auto f = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(4096u + r * 256u + q * 16u), 0, 0);
        const uint32_t b = threadIdx.x >> 8, x = threadIdx.x & 255u;
        const uint32_t row = ((b >> 1) * 65536u + x * 256u + (b & 1u) * 64u) / 16u;
        const uint4 v = make_uint4(bulk, bulk, bulk, bulk);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) lds4[row + ((k + x) & 3u)] = v;
        lds4[(r * 256u + 128u + q * 16u) / 16u] = make_uint4(f[0], f[1], f[2], f[3]);
        __syncthreads();
    }
    const char *lds = reinterpret_cast<const char *>(lds4);
    LaneConsts c;
    c.pc = ((lane & 15u) * 4u) | (((lane & 15u) * 4u + 64u) << 8) | (1u << 16);
    c.fin = 128u + (lane & 31u) * 4u;
    if (!mine) return false;
    run_oct<kVerify, RAGGED, TRAILER, D, true>(p, lds, c, lane, lo, nq);
    return true;
}

template <bool TRAILER, class D = OctProduct>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_oct_rx_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    uint32_t lo, nq;
    rx_oct_part<TRAILER, D, false>(p, lds4, lo, nq);
}

// The ragged one-pass receive, launch 1 of 2: the oct ring (RX) on the workgroup's packets with L <
// split_len (a workgroup with none skips it), then long_body's verify of the rest.
template <bool TRAILER>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_hybrid_rx_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    uint32_t lo, nq;
    rx_oct_part<TRAILER, OctProduct, true>(p, lds4, lo, nq);
    __syncthreads();  // every wave is done with the receive image before the long body rewrites LDS
    long_body<kVerify, false, TRAILER, Ring<kStreamAux>, 2>(p, lds4, blockIdx.x, gridDim.x);  // + their descriptors
}

// Launch 2: descriptors for the short packets the ring did not take (L < 44, misaligned, far apart:
// the ring's tail loop) and for the long packets of dense ranges, from their header words and the
// ok bytes those paths left in p.ok, in the descriptor pass's shape (rx_desc_block); a call with
// neither (p.rx_flag[0..1] below p.rx_gen) returns at once.  The long packets of sparse ranges
// have their descriptors from long_body's walk (PARSE 2, round 6: on configs[2] this launch took
// 69 us for them, 12 % of the receive).  The ring's
// blocks are whole, 64-aligned blocks of the batch (the dispatch guarantees more than 32 packets
// per wave), so classifying each block here again (oct_block) finds exactly the ring's packets.
// (In the first launch, after long_body, this measured slower: that kernel's registers are sized
// for its rings.)
__global__ __launch_bounds__(256) void icrc_rx_sweep_kernel(BatchParams p) {
    __shared__ uint32_t sh_all[4 * 64 * kRxStride];
    // rx_flag[0]: the ring's tail loop left short packets; rx_flag[1]: a dense long-packet range left
    // its long packets (long_body; a sparse range's long packets have their descriptors already, and
    // writing them again here writes the same bytes)
    bool all_long = true;
    if (p.rx_flag) {
        const bool tail = *reinterpret_cast<volatile const uint32_t *>(p.rx_flag) >= p.rx_gen;
        all_long = *reinterpret_cast<volatile const uint32_t *>(p.rx_flag + 1) >= p.rx_gen;
        if (!tail && !all_long) return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *sh = sh_all + wave * 64u * kRxStride;
    const uint32_t tw = gridDim.x * 4u;
    for (uint32_t base = (blockIdx.x * 4u + wave) * 64u; base < p.n; base += tw * 64u) {
        const uint32_t i = base + lane;
        const bool valid = i < p.n;
        const uint64_t off = valid ? (p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride) : 0u;
        const uint32_t L = valid ? (p.len ? p.len[i] : p.ulen) : 0u;
        OctBlock B;
        oct_block<kVerify>(p, B, off, L, valid, base, 0, lane);
        const uint64_t need = __ballot(valid && (all_long || L < p.split_len)) & ~B.mine;
        if (need != 0ull) rx_desc_block(p, sh, base, p.n - base < 64u ? p.n - base : 64u, need, lane);
    }
}

#ifdef ICRC_AB_BUILD
// A/B (ICRC_AB_HYBRID_STAMP=1, compute): the hybrid kernel with each workgroup's start and end
// (s_memrealtime, 100 MHz) and kind stored in g_hybrid_stamps, entry b = {start lo, start hi, end
// lo, end hi, 0 = oct / 1 = long} of workgroup b, read back by icrc_ab_hybrid_stamps: when the
// long-packet workgroups start and end against the oct ones' ends (scripts/probe_hybrid_timeline.py).
constexpr uint32_t kStampGroups = 8192;
__device__ uint32_t g_hybrid_stamps[5 * kStampGroups];
template <bool COMPACT>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_hybrid_stamp_kernel(BatchParams p, uint32_t g_oct) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < g_oct) oct_body<kCompute, true, false, OctProduct>(p, lds4, blockIdx.x, g_oct);
    else long_body<kCompute, COMPACT, false>(p, lds4, blockIdx.x - g_oct, gridDim.x - g_oct);
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < kStampGroups) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        uint32_t *e = g_hybrid_stamps + 5u * blockIdx.x;
        e[0] = static_cast<uint32_t>(t0);
        e[1] = static_cast<uint32_t>(t0 >> 32);
        e[2] = static_cast<uint32_t>(t1);
        e[3] = static_cast<uint32_t>(t1 >> 32);
        e[4] = blockIdx.x < g_oct ? 0u : 1u;
    }
}
#endif

}  // namespace

// Variant 40 (the default short-packet kernel): packets of at most 1088 bytes.
uint32_t oct_max_len() { return kOctMaxL; }

int launch_oct(int mode, const BatchParams &p, int grid, void *stream, int diag) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool ragged = p.off != nullptr || p.len != nullptr;
#define ICRC_O(M, R, T, D) hipLaunchKernelGGL((icrc_oct_kernel<M, R, T, D>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p)
#ifdef ICRC_AB_BUILD  // the ablations (wrong results by design): the A/B library only
#define ICRC_OD(M, R)                                                \
    do {                                                             \
        switch (diag) {                                              \
        case 1: ICRC_O(M, R, false, OctAblation<1>); break;          \
        case 2: ICRC_O(M, R, false, OctAblation<2>); break;          \
        case 3: ICRC_O(M, R, false, OctAblation<3>); break;          \
        case 4: ICRC_O(M, R, false, OctAblation<4>); break;          \
        case 5: ICRC_O(M, R, false, OctAblation<5>); break;          \
        case 6: ICRC_O(M, R, false, OctAblation<6>); break;          \
        case 7: ICRC_O(M, R, false, OctAblation<7>); break;          \
        case 9: ICRC_O(M, R, false, OctAblation<9>); break;          \
        case 10: ICRC_O(M, R, false, OctAblation<10>); break;        \
        case 11: ICRC_O(M, R, false, OctAblation<11>); break;        \
        case 12: ICRC_O(M, R, false, OctAblation<12>); break;        \
        case 13: ICRC_O(M, R, false, OctAblation<13>); break;        \
        default: ICRC_O(M, R, false, OctAblation<8>); break;         \
        }                                                            \
    } while (0)
#define ICRC_OM_DIAG(M)                                              \
        if (diag != 0 && M == kCompute && !p.trailer) {              \
            if (ragged) ICRC_OD(M, true);                            \
            else ICRC_OD(M, false);                                  \
        } else
#else
#define ICRC_OM_DIAG(M) (void)diag;
#endif
#define ICRC_OM(M)                                                   \
    do {                                                             \
        ICRC_OM_DIAG(M)                                              \
        if (ragged) {                                                \
            if (p.trailer) ICRC_O(M, true, true, OctProduct);        \
            else ICRC_O(M, true, false, OctProduct);                 \
        } else {                                                     \
            if (p.trailer) ICRC_O(M, false, true, OctProduct);       \
            else ICRC_O(M, false, false, OctProduct);                \
        }                                                            \
    } while (0)
    if (mode == kCompute) ICRC_OM(kCompute);
    else ICRC_OM(kVerify);
#undef ICRC_OM
#undef ICRC_OM_DIAG
#ifdef ICRC_AB_BUILD
#undef ICRC_OD
#endif
#undef ICRC_O
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_oct_rx(const BatchParams &p, int grid, void *stream, int diag) {
    hipStream_t s = static_cast<hipStream_t>(stream);
#ifdef ICRC_AB_BUILD
    if (diag >= 2 && diag <= 9 && !p.trailer) {
        switch (diag) {
        case 2: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<2>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 3: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<3>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 4: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<4>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 5: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<5>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 6: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<6>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 7: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<7>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        case 8: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<8>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        default: hipLaunchKernelGGL((icrc_oct_rx_kernel<false, OctRxAblation<9>>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p); break;
        }
        return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
    }
#else
    (void)diag;
#endif
    if (p.trailer) hipLaunchKernelGGL((icrc_oct_rx_kernel<true>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    else hipLaunchKernelGGL((icrc_oct_rx_kernel<false>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_hybrid_rx(const BatchParams &p, int grid, int num_cu, void *stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (p.trailer) hipLaunchKernelGGL((icrc_hybrid_rx_kernel<true>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    else hipLaunchKernelGGL((icrc_hybrid_rx_kernel<false>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p);
    if (hipGetLastError() != hipSuccess) return ICRC_EDEVICE;
    // 16 workgroups per CU: a sweep with nothing to do returns at once (4.6-4.9 us); 8 per CU saved ~1
    // us there but cost a sweep with work 13 us (786 K x 4156 B: 50 against 37 us, profiles/r06/final/)
    const uint64_t want = (static_cast<uint64_t>(p.n) + 255u) / 256u;
    const uint64_t cap = static_cast<uint64_t>(num_cu > 0 ? num_cu : 1) * 16u;
    hipLaunchKernelGGL(icrc_rx_sweep_kernel, dim3(static_cast<uint32_t>(want < cap ? want : cap)), dim3(256), 0, s, p);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

int launch_hybrid(int mode, const BatchParams &p, int grid_oct, int grid_long, void *stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 g(static_cast<uint32_t>(grid_oct + grid_long));
    const uint32_t go = static_cast<uint32_t>(grid_oct);
    if (grid_long == 0) {  // the default: each workgroup both halves of its range (icrc_hybrid_self_kernel)
        if (mode == kCompute) {
            if (p.trailer) hipLaunchKernelGGL((icrc_hybrid_self_kernel<kCompute, true, false>), dim3(go), dim3(kThreadsPerGroup), 0, s, p);
            else hipLaunchKernelGGL((icrc_hybrid_self_kernel<kCompute, false, false>), dim3(go), dim3(kThreadsPerGroup), 0, s, p);
        } else {
            if (p.trailer) hipLaunchKernelGGL((icrc_hybrid_self_kernel<kVerify, true, false>), dim3(go), dim3(kThreadsPerGroup), 0, s, p);
            else hipLaunchKernelGGL((icrc_hybrid_self_kernel<kVerify, false, false>), dim3(go), dim3(kThreadsPerGroup), 0, s, p);
        }
        return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
    }
#define ICRC_H(M, T, C) hipLaunchKernelGGL((icrc_hybrid_kernel<M, T, C>), g, dim3(kThreadsPerGroup), 0, s, p, go)
#define ICRC_HM(M)                                    \
    do {                                              \
        if (p.long_variant == 1) {                    \
            if (p.trailer) ICRC_H(M, true, true);     \
            else ICRC_H(M, false, true);              \
        } else {                                      \
            if (p.trailer) ICRC_H(M, true, false);    \
            else ICRC_H(M, false, false);             \
        }                                             \
    } while (0)
#ifdef ICRC_AB_BUILD
    // ICRC_AB_LONG_VMETA=1: the long half's dense walk with vector (offset, length) blocks
    const char *vm = std::getenv("ICRC_AB_LONG_VMETA");
    if (vm && std::atoi(vm) == 1 && mode == kCompute && !p.trailer && p.long_variant != 1) {
        hipLaunchKernelGGL((icrc_hybrid_kernel<kCompute, false, false, RingVectorMeta>), g, dim3(kThreadsPerGroup), 0, s, p, go);
        return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
    }
    const char *st = std::getenv("ICRC_AB_HYBRID_STAMP");
    if (st && std::atoi(st) == 1 && mode == kCompute && !p.trailer) {
        if (p.long_variant == 1) hipLaunchKernelGGL((icrc_hybrid_stamp_kernel<true>), g, dim3(kThreadsPerGroup), 0, s, p, go);
        else hipLaunchKernelGGL((icrc_hybrid_stamp_kernel<false>), g, dim3(kThreadsPerGroup), 0, s, p, go);
        return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
    }
#endif
    if (mode == kCompute) ICRC_HM(kCompute);
    else ICRC_HM(kVerify);
#undef ICRC_HM
#undef ICRC_H
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc

#ifdef ICRC_AB_BUILD
// A/B library only (not in include/icrc.h): copy the last stamp launch's n_groups x 5 words.
extern "C" int icrc_ab_hybrid_stamps(uint32_t *dst, uint32_t n_groups) {
    if (n_groups > icrc::kStampGroups) n_groups = icrc::kStampGroups;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(icrc::g_hybrid_stamps), 5u * n_groups * sizeof(uint32_t), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
