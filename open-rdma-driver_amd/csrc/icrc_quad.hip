// icrc_quad.hip — the four-packets-per-wavefront ICRC kernel (variants 19-21, the default for
// ragged batches).  Bit-exact with compute_icrc / is_icrc_valid
// (blue-rdma-device/src/third_party/net/packet_processor.rs:275-301, 341-353); the algorithm is
// described at the top of icrc_kernels.hip, the quad mapping below.
#include <hip/hip_runtime.h>

#include "icrc_device.h"
#include "icrc_internal.h"

namespace icrc {
namespace {

// ---- quad path: four packets per wavefront ------------------------------------------------
// Lanes 16g .. 16g+15 (group g = lane >> 4, column c = lane & 15) carry one packet.  A packet
// row is 16 stream words (one buffer_load_dword per lane: 64 contiguous bytes per group, 256 B
// per wave instruction); rows are end-aligned as in the one-packet path, so the column
// multiplier M^(16-c) depends only on the lane.  Tables: the quad image (M^16 bulk, M^(16-c)
// final; build_table_image_quad).  Against one packet per wavefront this divides every
// per-packet cost (final multiply, reduction, result handling) by four and cuts the padding
// of short packets from up to 63 words to up to 15: the mixed-MTU batch is dominated by
// 316-byte packets (79 stream words: 5 quad rows, 80 slots, against 2 x 64 = 128).
//
// A wave walks its chunk in blocks of 64 packets.  Each block is sorted by row count (bitonic
// sort of (R << 6 | index) across the lanes), and consecutive sorted packets form sets of 4
// processed in lockstep; a shorter packet in a set is END-aligned to the longest by leading
// zero rows, which leave a zero accumulator at zero, so no guards are needed.  Packets
// outside the fast path (L < 44, misaligned, L % 4 != 0, offsets too far apart for 32-bit
// buffer offsets) are done by a tail loop.
constexpr uint32_t kQuadOOR = 0x80000000u;        // voffset past the range: the load returns 0
constexpr uint32_t kQuadRelLimit = 0x7F000000u;   // packet offset in its block + L stay below
constexpr uint32_t kQuadIrregular = 0x3FFFFFFu;   // sort key (>> 6) of a non-fast-path slot
constexpr int kQuadEmptyE = -(1 << 30);          // word index of a group with no packet
// Row loads use the default cache policy: a 128-byte line here is read by two or more load
// instructions (64 bytes per packet group each), and non-temporal loads re-fetch it every time:
// four packets per wave read 3.7 TB/s with nt, 6.2 TB/s without (profiles/r01_membench_policy.json).
constexpr int kQuadAux = 0;

// Geometry of a W-lane packet group: G = 64 / W packets per wavefront.
template <int W>
struct Geo {
    static constexpr int G = 64 / W;
    static constexpr int LW = W == 16 ? 4 : 3;
    static constexpr int LG = W == 16 ? 2 : 3;
    static constexpr int HR = 1 + (9 + W - 1) / W;  // packet rows that can hold masked header words
};

struct QuadBlock {
    uint32_t key;   // per lane p (sorted position): R << 6 | block index of the packet
    uint32_t vrel;  // per lane p: packet offset relative to the block's buffer base
    uint32_t len;   // per lane p: L
    uint32_t pos;   // per lane i (block index): sorted position of packet i
    uint64_t regmask;  // uniform: block indices of fast-path packets
    uint64_t boff;     // uniform: buffer base (byte offset from p.base)
    int block;         // uniform
    int nsets;         // uniform
};

struct QuadSet {
    uint32_t vb;  // per lane: byte offset of this lane's word in set row 0 (mod 2^32)
    int e;        // per lane: packet word index at set row 0 (< 0: before the packet)
    int rows;     // uniform: rows of the longest packet in the set
    int hrows;    // uniform: rows that may hold header words (head masks / OOR selects)
};

// Fast-path classification of block b's packets (off, L of this lane's packet) and the block's
// buffer base.  Returns the ballot of the valid packets that are NOT on the fast path.
__device__ __forceinline__ uint64_t quad_classify_from(const BatchParams &p, uint64_t off, uint32_t L, bool valid,
                                                       uint32_t lo, int b, uint32_t lane, bool &reg, uint64_t &boff) {
    const bool foreign = valid && p.split_len != 0 && L >= p.split_len;  // the long-packet kernel's
    reg = valid && !foreign && L >= ICRC_MIN_PACKET && ((reinterpret_cast<uintptr_t>(p.base + off) | L) & 3u) == 0;
    if (p.off == nullptr) {
        boff = static_cast<uint64_t>(lo + static_cast<uint32_t>(b) * 64u) * p.stride;
    } else {  // minimum offset over the fast-path packets (64-bit butterfly)
        uint64_t m = reg ? off : ~0ull;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint32_t pl = lane ^ static_cast<uint32_t>(s);
            const uint64_t o = static_cast<uint64_t>(bperm(pl, static_cast<uint32_t>(m))) |
                               (static_cast<uint64_t>(bperm(pl, static_cast<uint32_t>(m >> 32))) << 32);
            m = o < m ? o : m;
        }
        boff = static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(m), 0)) |
               (static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(m >> 32), 0)) << 32);
    }
    reg = reg && (off - boff) + L <= kQuadRelLimit;
    return __ballot(valid && !reg && !foreign);
}

// The same, reading (offset, L) from the batch arrays (tail loop).
__device__ __forceinline__ uint64_t quad_classify(const BatchParams &p, uint32_t lo, uint32_t nq, int b,
                                                  uint32_t lane, uint64_t &off, uint32_t &L, bool &reg,
                                                  uint64_t &boff) {
    const uint32_t q = static_cast<uint32_t>(b) * 64u + lane;
    const bool valid = q < nq;
    const uint32_t i = lo + q;
    off = 0;
    L = 0;
    if (valid) {
        off = p.off ? p.off[i] : static_cast<uint64_t>(i) * p.stride;
        L = p.len ? p.len[i] : p.ulen;
    }
    return quad_classify_from(p, off, L, valid, lo, b, lane, reg, boff);
}

// Block b: classification, then the fast-path packets sorted by row count (bitonic sort of
// R << 6 | index across the lanes; skipped when already sorted).
template <int W>
__device__ __forceinline__ void quad_block_from(const BatchParams &p, QuadBlock &B, uint64_t off, uint32_t L,
                                                bool valid, uint32_t lo, int b, uint32_t lane, bool &irregular) {
    using Gm = Geo<W>;
    uint64_t boff;
    bool reg;
    if (quad_classify_from(p, off, L, valid, lo, b, lane, reg, boff) != 0) irregular = true;
    const uint32_t R = reg ? (1u + ((L - 4u) >> 2) + (W - 1u)) >> Gm::LW : kQuadIrregular;
    uint32_t key = (R << 6) | lane;
    const uint32_t nxt = bperm((lane + 1u) & 63u, key);
    if (__ballot(lane == 63u || key <= nxt) != ~0ull) {
#pragma unroll
        for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
                const uint32_t other = bperm(lane ^ static_cast<uint32_t>(j), key);
                const bool up = (lane & static_cast<uint32_t>(k)) == 0u;
                const bool lower = (lane & static_cast<uint32_t>(j)) == 0u;
                const uint32_t mn = key < other ? key : other;
                const uint32_t mx = key < other ? other : key;
                key = (lower == up) ? mn : mx;
            }
        }
    }
    const uint32_t idx = key & 63u;
    B.key = key;
    B.vrel = bperm(idx, static_cast<uint32_t>(off - boff));
    B.len = bperm(idx, L);
    B.pos = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(static_cast<int>(idx << 2), static_cast<int>(lane)));
    B.regmask = __ballot(reg);
    B.boff = boff;
    B.block = b;
    B.nsets = (__popcll(B.regmask) + Gm::G - 1) >> Gm::LG;
}

template <int W>
__device__ __forceinline__ void quad_set(const QuadBlock &B, int s, uint32_t lane, QuadSet &S) {
    using Gm = Geo<W>;
    constexpr int G = Gm::G;
    const int nreg = __popcll(B.regmask);
    const uint32_t ps = static_cast<uint32_t>(G * s) + (lane >> Gm::LW);
    const uint32_t key = bperm(ps & 63u, B.key);
    const uint32_t vrel = bperm(ps & 63u, B.vrel);
    const uint32_t L = bperm(ps & 63u, B.len);
    const int last = (G * s + G - 1 < nreg) ? G * s + G - 1 : nreg - 1;
    const int Rmax = static_cast<int>(readlane_u32(B.key, last) >> 6);
    const int Rmin = static_cast<int>(readlane_u32(B.key, G * s) >> 6);
    const int R = static_cast<int>(key >> 6);
    const int N = 1 + static_cast<int>((L - 4u) >> 2);
    const int k0 = N - W * R;
    const bool valid = static_cast<int>(ps) < nreg;
    S.e = valid ? k0 - 1 + static_cast<int>(lane & (W - 1u)) - W * (Rmax - R) : kQuadEmptyE;
    S.vb = vrel + 4u * static_cast<uint32_t>(S.e);
    S.rows = Rmax;
    const int full = G * s + G - 1 < nreg;
    S.hrows = full ? (Rmax - Rmin + Gm::HR < Rmax ? Rmax - Rmin + Gm::HR : Rmax) : Rmax + 1;
}

// Chunk pipeline.  A set's rows (end-aligned, see above) are cut into chunks of K rows, the
// first chunk padded in front with rows that load nothing (leading zeros: free), so every
// chunk is K straight-line loads and K straight-line steps.  A ring of B = D + 1 chunk buffers
// keeps D chunks in flight per wavefront; every buffer carries the metadata the process side
// needs (word index for head masks, last-chunk flag, trailer offset, result routing, block),
// so the process side holds no block state however far the load side has run ahead.  Every
// ring position issues exactly the same loads (absent rows have an out-of-range offset), and
// a ragged batch's next-block (offset, len) is loaded once per ring cycle, unconditionally:
// the compiler's vmcnt accounting stays exact and no wait drains the ring.

template <int W, int MODE, int K, int D, bool RAGGED, bool TRAILER, int ABLATE = 0>
__device__ __forceinline__ void run_quad(const BatchParams &p, const char *lds, const LaneConsts &c, uint32_t lane,
                                         uint32_t lo, uint32_t nq) {
    using Gm = Geo<W>;
    constexpr uint32_t RB = 4u * W;  // bytes per packet row
    constexpr int B = D + 1;
    constexpr int KT = MODE == kVerify ? K + 1 : K;  // verify: + the stored trailers
    if (nq == 0) return;
    const int nblocks = static_cast<int>((nq + 63u) >> 6);
    const uint32_t grp = lane >> Gm::LW;
    const uint32_t col = lane & (W - 1u);
    bool irregular = false;

    // Next block NB, prepared at the top of a ring cycle (one copy of the sort, not B), from
    // the (offset, len) registers loaded at the top of the cycle before (ragged batches).
    QuadBlock NB;
    int nb_next = 0, mblk = -1;
    bool nb_ready = false;
    uint32_t m_lo = 0, m_hi = 0, m_len = 0;

    // load side
    QuadBlock LB;
    QuadSet LS;
    int lblk = -1, lset = 0, f = 0;
    bool lhave = false, ldone = false;
    int inflight = 0;

    // ring: data and carried metadata
    uint32_t u[B][KT];
    uint32_t ce[B];   // per lane: (word index at chunk row 0, clamped) << 8 | result route (0xFF none)
    uint32_t ctr[B];  // per lane: trailer offset (TRAILER only)
    int cflags[B];    // uniform: bit 31 valid, bit 30 last chunk of its set, bits 0..7 head rows
    int cblk[B];
    uint64_t cboff[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        cflags[b] = 0;
        cblk[b] = -1;
        cboff[b] = 0;
        ce[b] = 0xFFu;
        ctr[b] = kQuadOOR;
#pragma unroll
        for (int j = 0; j < KT; ++j) u[b][j] = 0;
    }

    // process side
    uint32_t acc = 0, rbv = 0;
    bool got = false;
    int rb_block = -1;

    // load side of one ring position: the next chunk (or nothing) into buffer b
    auto l_issue = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        if (!lhave && !ldone) {  // next set: in this block, else the prepared next block
            bool ok = false;
            if (lblk >= 0 && lset + 1 < LB.nsets) {
                lset += 1;
                ok = true;
            } else if (nb_ready) {
                LB = NB;
                nb_ready = false;
                lblk = LB.block;
                lset = 0;
                ok = true;
            } else if (nb_next >= nblocks) {
                ldone = true;
            }  // else a stall: the next block is prepared at the top of the next cycle
            if (ok) {
                quad_set<W>(LB, lset, lane, LS);
                f = LS.rows - ((LS.rows + K - 1) / K) * K;
                lhave = true;
            }
        }
        int fl = 0;
        uint32_t vb = 0;
        if (lhave) {
            vb = LS.vb + RB * static_cast<uint32_t>(f);
            // chunk rows [js, je) may hold header words: set rows [0, hrows) sit at chunk rows - f
            const int js = f < 0 ? -f : 0;
            int je = LS.hrows - f;
            je = je > K ? K : je;
            fl = (1 << 31) | (je > js ? (js << 8) | je : 0);
            const bool last = f + K >= LS.rows;
            if (last) fl |= 1 << 30;
            const uint32_t ps = LB.pos;
            const bool mine = last && ((LB.regmask >> lane) & 1ull) && static_cast<int>(ps >> Gm::LG) == lset;
            const int e = LS.e + W * f;
            ce[b] = (static_cast<uint32_t>(e < -(1 << 20) ? -(1 << 20) : e) << 8) |
                    (mine ? (ps & (Gm::G - 1u)) << Gm::LW : 0xFFu);
            if constexpr (TRAILER) {
                ctr[b] = (col == 0u && LS.e != kQuadEmptyE) ? LS.vb + RB * static_cast<uint32_t>(LS.rows) : kQuadOOR;
            }
            cblk[b] = lblk;
            cboff[b] = LB.boff;
        }
        const __amdgpu_buffer_rsrc_t lrs =
            __builtin_amdgcn_make_buffer_rsrc(p.base + LB.boff, 0, static_cast<int>(kQuadOOR), 0x00020000);
        // Row j holds packet word e0 + W j of this lane: absent (before the packet, a pad row, an
        // empty group, no chunk) exactly when that is negative.  One compare + select per row.
        const int e0 = lhave ? LS.e + W * f : kQuadEmptyE;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t vo = e0 >= -W * j ? vb : kQuadOOR;
            if constexpr (ABLATE >= 2) u[b][j] = vo ^ static_cast<uint32_t>(j);  // diagnostic: no loads (2..5)
            else
                u[b][j] = __builtin_amdgcn_raw_buffer_load_b32(lrs, static_cast<int>(vo + RB * static_cast<uint32_t>(j)), 0,
                                                               kQuadAux);
        }
        if constexpr (MODE == kVerify) {  // lane W g: packet g's stored ICRC (the set's last chunk)
            const bool t = lhave && (fl & (1 << 30)) && col == 0u && LS.e != kQuadEmptyE;
            const uint32_t vo = t ? LS.vb + RB * static_cast<uint32_t>(LS.rows) : kQuadOOR;
            u[b][K] = __builtin_amdgcn_raw_buffer_load_b32(lrs, static_cast<int>(vo), 0, kQuadAux);
        }
        cflags[b] = fl;
        if (lhave) {
            inflight += 1;
            f += K;
            if (f >= LS.rows) lhave = false;
        }
    };

    // process side of one ring position: buffer b
    // process side: header masks of buffer b (stream word k = e + W j + 1 of row j; the masked
    // words k <= 9 are W apart in a column, so a lane has at most one (W = 16) or two (W = 8):
    // rows jh, jh + 1, masks hm, hm2.  They lie in chunk rows [js, je) (uniform).  When a set
    // of equal row counts starts the chunk (js = 0: no pad rows, e.g. 316-byte packets in
    // chunks of 10 rows) that is rows 0 .. HR - 1, and the other rows cost nothing; any other
    // window masks every row.)
    auto p_masks = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        const int fl = cflags[b];
        const int js = (fl >> 8) & 0xFF, je = fl & 0xFF;
        if (je > js) {
            const int k0 = (static_cast<int>(ce[b]) >> 8) + 1;
            const int jh = k0 >= 0 ? 0 : (W - 1 - k0) >> Gm::LW;
            const uint32_t hm = head_mask(k0 + W * jh);
            const uint32_t hm2 = W < 16 ? head_mask(k0 + W * (jh + 1)) : 0u;
            if (js == 0 && je <= Gm::HR) {  // the set starts the chunk: rows 0 .. HR - 1
#pragma unroll
                for (int j = 0; j < (Gm::HR < K ? Gm::HR : K); ++j)
                    u[b][j] |= (jh == j ? hm : 0u) | (W < 16 && jh + 1 == j ? hm2 : 0u);
            } else {
#pragma unroll
                for (int j = 0; j < K; ++j) u[b][j] |= (jh == j ? hm : 0u) | (W < 16 && jh + 1 == j ? hm2 : 0u);
            }
        }
    };

    // process side: the ICRC of the set whose last chunk is buffer b, from the final products
    // fm (final_mul of its accumulator): result, trailer store, routing to the packet's lane
    auto p_finish = [&](auto bc, uint32_t fm) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        const uint32_t crc = ~group_xor<W>(fm);
        uint32_t r;
        if constexpr (MODE == kCompute) r = crc;
        else r = bperm(grp << Gm::LW, u[b][K]) == crc ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH;
        if constexpr (TRAILER) {  // PacketWriter stores the ICRC / is_icrc_valid zeroes it
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(p.base + cboff[b], 0, static_cast<int>(kQuadOOR), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(MODE == kCompute ? crc : 0u, rs, static_cast<int>(ctr[b]), 0, 0);
        }
        if (cblk[b] != rb_block) {
            if (rb_block >= 0 && got) store_result<MODE>(p, lo + static_cast<uint32_t>(rb_block) * 64u + lane, rbv);
            got = false;
            rb_block = cblk[b];
        }
        const uint32_t rt = ce[b] & 0xFFu;
        const uint32_t v = bperm(rt & 63u, r);
        if (rt != 0xFFu) {
            rbv = v;
            got = true;
        }
    };

    // process side of one ring position: buffer b
    auto p_consume = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        const int fl = cflags[b];
        if (!(fl & (1 << 31))) return;
        if constexpr (ABLATE != 5) p_masks(bc);  // diagnostic 5: no header masks
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if constexpr (ABLATE == 1 || ABLATE >= 3) acc ^= u[b][j];  // diagnostic: loads only / overhead only
            else acc = step_m64(lds, acc, u[b][j], c);
        }
        inflight -= 1;
        if (fl & (1 << 30)) {
            if constexpr (ABLATE == 4) {  // diagnostic 4: no final products / routing
                rbv ^= acc;
                got = true;
                rb_block = cblk[b];
            } else if constexpr (ABLATE == 6) {
                p_finish(bc, acc);  // diagnostic 6: no final products
            } else {
                p_finish(bc, final_mul(lds, acc, c.fin));
            }
            acc = 0;
        }
    };

    for (;;) {
        // top of the cycle: prepare the next block, then fetch the (offset, len) of the one after
        if (!nb_ready && nb_next < nblocks && (!RAGGED || mblk == nb_next)) {
            const uint32_t q = static_cast<uint32_t>(nb_next) * 64u + lane;
            const bool valid = q < nq;
            uint64_t off = 0;
            uint32_t L = 0;
            if (valid) {
                off = p.off ? (static_cast<uint64_t>(m_lo) | (static_cast<uint64_t>(m_hi) << 32))
                            : static_cast<uint64_t>(lo + q) * p.stride;
                L = p.len ? m_len : p.ulen;
            }
            quad_block_from<W>(p, NB, off, L, valid, lo, nb_next, lane, irregular);
            nb_next += 1;
            nb_ready = NB.nsets > 0;
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
        static_for<B>([&](auto bc) __attribute__((always_inline)) -> bool {
            constexpr int b = decltype(bc)::value;
            l_issue(IntC<(b + D) % B>{});
            p_consume(bc);
            return true;
        });
        if (ldone && inflight == 0) break;
    }
    if (rb_block >= 0 && got) store_result<MODE>(p, lo + static_cast<uint32_t>(rb_block) * 64u + lane, rbv);

    if (irregular) {  // L < 44, misaligned, L % 4 != 0, far-apart offsets: per packet
        for (int b = 0; b < nblocks; ++b) {
            uint64_t off, boff;
            uint32_t L;
            bool reg;
            uint64_t m = quad_classify(p, lo, nq, b, lane, off, L, reg, boff);
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t o = static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off), l)) |
                                   (static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off >> 32), l)) << 32);
                const uint32_t Ll = readlane_u32(L, l);
                const uint32_t r = quad_slow_packet<MODE, W>(p, p.base + o, Ll, lds, c, lane);
                if (lane == 0) store_result<MODE>(p, lo + static_cast<uint32_t>(b) * 64u + static_cast<uint32_t>(l), r);
            }
        }
    }
}

template <int W, int MODE, int K, int D, bool RAGGED, bool TRAILER, int ABLATE = 0, int NT = kThreadsPerGroup>
__global__ __launch_bounds__(NT) void icrc_quad_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    const uint32_t tw = gridDim.x * (NT / 64);
    // chunks of whole 64-packet blocks (whole-line result stores) unless that idles waves
    uint32_t chunk = (p.n + tw - 1) / tw;
    chunk = chunk > 32u ? (chunk + 63u) & ~63u : (chunk + (64u / W - 1u)) & ~(64u / W - 1u);
    if (RAGGED && p.split_len != 0 && p.len != nullptr) {
        // Split batch: a workgroup whose packets are all the long-packet kernel's exits before
        // its 160 KiB table load (an all-long ragged batch costs this kernel a length scan only).
        const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * (NT / 64) * chunk;
        const uint64_t g1 = g0 + static_cast<uint64_t>(NT / 64) * chunk;
        const uint64_t end = g1 < p.n ? g1 : p.n;
        bool any_short = false;
        for (uint64_t i = g0 + threadIdx.x; i < end; i += NT) any_short |= p.len[i] < p.split_len;
        // OR across the workgroup through the (not yet loaded) table space: the tables fill the
        // whole LDS, so __syncthreads_or's own LDS word does not fit
        volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(lds4);
        if (threadIdx.x == 0) *flag = 0u;
        __syncthreads();
        if (any_short) *flag = 1u;
        __syncthreads();
        const bool go = *flag != 0u;
        __syncthreads();  // every wave has read the flag before the table load overwrites it
        if (!go) return;
    }
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(W == 16 ? p.table_quad : p.table_oct);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += NT) lds4[i] = src[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t gw = blockIdx.x * (NT / 64) + wave;
    const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
    run_quad<W, MODE, K, D, RAGGED, TRAILER, ABLATE>(p, lds, c, lane, lo, nq);
}

}  // namespace

// Quad (W = 16): variant 20: K = 6 rows per chunk, D = 4 chunks in flight.  Oct (W = 8): 24 (the
// default for short packets): K = 10, D = 3; 25: K = 8, D = 4; 26: K = 5, D = 6.  Diagnostics of 24
// (wrong results by design): 31 loads only (ragged), 32 no loads (ragged), 35 no loads and no row
// steps (strided: what is left is per-set control).
int launch_quad(int mode, int variant, const BatchParams &p, int grid, void *stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool ragged = p.off != nullptr || p.len != nullptr;
#define ICRC_L(W, M, K, D, R, T, ...) \
    hipLaunchKernelGGL((icrc_quad_kernel<W, M, K, D, R, T, ##__VA_ARGS__>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p)
#define ICRC_Q(W, M, K, D)                                      \
    do {                                                        \
        if (ragged) {                                           \
            if (p.trailer) ICRC_L(W, M, K, D, true, true);      \
            else ICRC_L(W, M, K, D, true, false);               \
        } else {                                                \
            if (p.trailer) ICRC_L(W, M, K, D, false, true);     \
            else ICRC_L(W, M, K, D, false, false);              \
        }                                                       \
    } while (0)
#define ICRC_QV(M)                                  \
    do {                                            \
        switch (variant) {                          \
        case 20: ICRC_Q(16, M, 6, 4); break;        \
        case 25: ICRC_Q(8, M, 8, 4); break;         \
        case 26: ICRC_Q(8, M, 5, 6); break;         \
        default: ICRC_Q(8, M, 10, 3); break;        \
        }                                           \
    } while (0)
    if (variant == 31 || variant == 32 || variant == 35) {
        if (variant == 31) ICRC_L(8, kCompute, 10, 3, true, false, 1);
        else if (variant == 32) ICRC_L(8, kCompute, 10, 3, true, false, 2);
        else ICRC_L(8, kCompute, 10, 3, false, false, 3);
        return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
    }
    if (mode == kCompute) ICRC_QV(kCompute);
    else ICRC_QV(kVerify);
#undef ICRC_QV
#undef ICRC_Q
#undef ICRC_L
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc
