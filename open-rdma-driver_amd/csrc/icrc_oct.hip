// icrc_oct.hip — the short-packet ICRC kernel: eight packets per wavefront, one FIXED frame of K
// rows per set of eight (the default for packets of at most 32 K bytes; K = 10: L <= 320, the
// 256-byte-MTU packets that dominate a mixed-MTU batch).  Bit-exact with compute_icrc /
// is_icrc_valid (blue-rdma-device/src/third_party/net/packet_processor.rs:275-301, 341-353); the
// algorithm is described at the top of icrc_kernels.hip.
//
// Mapping.  Lanes 8g .. 8g+7 carry one packet; a packet row is 8 stream words (one
// buffer_load_dword per lane: 32 contiguous bytes per packet, 256 B per wave instruction); the
// packet is END-aligned in the K-row frame, so a shorter packet has leading zero rows (a zero
// accumulator stays zero) and the column multiplier M^(8 - c) depends only on the lane (the oct
// table image: M^8 bulk, M^(8 - (l & 7)) final tables).
//
// Why a fixed frame.  The previous short-packet kernel (icrc_quad.hip, kept as A/B variant 24) cut
// each set's rows into chunks that straddle sets and blocks, so every chunk carried its own
// bookkeeping (word index, head-mask window, last-chunk flag, trailer offset, routing) and two
// thirds of its time on 316-byte packets went to that control.  Here a ring slot IS a set: its
// schedule (addresses, head masks, result routing) is computed once on the load side, the process
// side is K straight-line row steps, one final product, one group XOR and one routed result.
//
// Per 64-packet block the packets this kernel takes (44 <= L <= 32 K, 4-byte aligned, L % 4
// == 0, within 2 GiB of the block's lowest) are sorted by row count (bitonic over the lanes), so
// the sets are mostly uniform; a set whose packets all fill the frame masks only its first three
// rows, any other set takes the generic per-lane mask rows.  Longer packets belong to the long-
// packet kernel (hybrid dispatch, p.split_len); the rest go to a per-packet tail loop.
#include <hip/hip_runtime.h>

#include "icrc_device.h"
#include "icrc_internal.h"

namespace icrc {
namespace {

constexpr uint32_t kOctOOR = 0x80000000u;       // buffer offset out of range: the load returns 0
constexpr uint32_t kOctRelLimit = 0x7F000000u;  // packet offset in its block + L stay below
constexpr uint32_t kOctNotMine = 63u;           // sort key (>> 6) of a packet this phase skips
constexpr int kOctK1 = 10, kOctK2 = 34;          // frame rows of the two phases
constexpr uint32_t kOctMaxL = 32u * kOctK2;      // 1088: longer packets are the long-packet kernel's

// A prepared block of 64 packets.  key / vrel / len are indexed by SORTED position (lane p);
// pos by original index (lane i).
struct OctBlock {
    uint32_t key;   // R << 6 | original index (R = kOctNotMine: not this kernel's)
    uint32_t vrel;  // packet offset - boff
    uint32_t len;   // L
    uint32_t pos;   // sorted position of packet i
    uint64_t mine;  // original indices this kernel computes
    uint64_t boff;  // lowest offset of those packets (byte offset from p.base)
    int nsets;
    int block;
};

// Classify block b from this lane's (offset, L): which packets are this kernel's, their row
// counts, the block's base offset; sort by row count.  Returns the ballot of packets that are
// neither this kernel's nor the long-packet kernel's (the tail loop's).
// A phase takes the fast-path packets with LMIN < L <= 32 K (N = 1 + (L - 4) / 4 <= 8 K); the
// fast path of the whole kernel is 44 <= L <= kOctMaxL, so both phases agree on which packets are
// the tail loop's (and on the block base).
template <int K, uint32_t LMIN>
__device__ __forceinline__ uint64_t oct_block(const BatchParams &p, OctBlock &B, uint64_t off, uint32_t L,
                                              bool valid, uint32_t lo, int b, uint32_t lane) {
    constexpr uint32_t kMaxL = 32u * K;
    const bool foreign = valid && p.split_len != 0 && L >= p.split_len;  // the long-packet kernel's
    bool fast = valid && !foreign && L >= ICRC_MIN_PACKET && L <= kOctMaxL &&
                ((reinterpret_cast<uintptr_t>(p.base + off) | L) & 3u) == 0;
    uint64_t boff;
    if (p.off == nullptr) {
        boff = static_cast<uint64_t>(lo + static_cast<uint32_t>(b) * 64u) * p.stride;
    } else {  // minimum offset over this kernel's packets (64-bit butterfly)
        uint64_t m = fast ? off : ~0ull;
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
    fast = fast && (off - boff) + L <= kOctRelLimit;
    const bool mine = fast && L > LMIN && L <= kMaxL;
    const uint32_t R = mine ? (1u + ((L - 4u) >> 2) + 7u) >> 3 : kOctNotMine;
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
    B.mine = __ballot(mine);
    B.boff = boff;
    B.block = b;
    B.nsets = (__popcll(B.mine) + 7) >> 3;
    return __ballot(valid && !fast && !foreign);
}

// The tail loop's classification (reads (offset, L) from the batch arrays).
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
    return oct_block<kOctK2, 0>(p, B, off, L, valid, lo, b, lane);
}

// One ring slot: the loads of one set and what its process side needs (per-lane values in VGPRs;
// only two uniform flags and, with trailer stores, the block base in SGPRs).
template <int K, int MODE, bool TRAILER>
struct OctSlot {
    uint32_t u[MODE == kVerify ? K + 1 : K];  // frame rows (+ the stored trailer, lane 8g)
    int kf;        // stream word of this lane at frame row 0 (head masks: words 0..9)
    uint32_t rt;   // routing: lane i of the block takes the result of lane rt (0xFF: none)
    uint32_t tro;  // trailer offset from the block base (lane 8g of a packet), else kOctOOR
    uint32_t rq;   // result store index (the block's packet i, after the block's last set), else kOctOOR
    uint64_t boff; // uniform (TRAILER only)
    bool have;     // uniform: the slot holds a set
    bool full;     // uniform: every packet of the set fills the frame (head masks on rows 0..2)
};

// DIAG (ablation builds, variants 41 / 42): 1 = the loads without the row steps and final
// products, 2 = the row steps without the loads.
template <int MODE, int K, int D, bool RAGGED, bool TRAILER, uint32_t LMIN, bool TAIL, int DIAG>
__device__ __forceinline__ void run_oct(const BatchParams &p, const char *lds, const LaneConsts &c, uint32_t lane,
                                        uint32_t lo, uint32_t nq) {
    constexpr int B = D + 1;
    if (nq == 0) return;
    const int nblocks = static_cast<int>((nq + 63u) >> 6);
    const uint32_t grp = lane >> 3;
    const uint32_t col = lane & 7u;
    bool irregular = false;

    // next block NB, prepared at the top of a ring cycle from the (offset, len) loaded the cycle before
    OctBlock NB;
    int nb_next = 0, mblk = -1;
    bool nb_ready = false;
    uint32_t m_lo = 0, m_hi = 0, m_len = 0;

    // load side: the block being issued and its next set
    OctBlock LB;
    LB.nsets = 0;
    LB.block = -1;
    int lset = 0;
    bool ldone = false;
    int inflight = 0;

    OctSlot<K, MODE, TRAILER> sl[B];
#pragma unroll
    for (int b = 0; b < B; ++b) sl[b].have = false;

    // process side: the block result register (lane i = packet i of the block)
    uint32_t rbv = 0;

    auto issue = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        OctSlot<K, MODE, TRAILER> &S = sl[b];
        bool have = false;
        if (!ldone) {
            if (LB.block >= 0 && lset + 1 < LB.nsets) {
                lset += 1;
                have = true;
            } else if (nb_ready) {
                LB = NB;
                nb_ready = false;
                lset = 0;
                have = true;
            } else if (nb_next >= nblocks) {
                ldone = true;
            }  // else a stall: the next block is prepared at the top of the next cycle
        }
        // this lane's packet of the set: sorted position 8 lset + grp
        const int nmine = __popcll(LB.mine);
        const uint32_t ps = 8u * static_cast<uint32_t>(lset) + grp;
        const uint32_t key = bperm(ps & 63u, LB.key);
        const uint32_t vrel = bperm(ps & 63u, LB.vrel);
        const uint32_t L = bperm(ps & 63u, LB.len);
        const bool real = have && static_cast<int>(ps) < nmine;
        const int R = static_cast<int>(key >> 6);
        const int k0 = 1 + static_cast<int>((L - 4u) >> 2) - 8 * R;  // stream word of lane 0, packet row 0
        const int kf = k0 + static_cast<int>(col) - 8 * (K - R);      // stream word of this lane, frame row 0
        const int vb = static_cast<int>(vrel) + 4 * (kf - 1);         // its packet word's byte offset
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(p.base + LB.boff, 0, static_cast<int>(kOctOOR), 0x00020000);
#pragma unroll
        for (int j = 0; j < K; ++j) {
            // the full offset formed in the VGPR (no immediate offset on a lane that is out of range)
            const int o = vb + 32 * j;
            if constexpr (DIAG == 2) S.u[j] = static_cast<uint32_t>(o) * 0x9E3779B1u;
            else S.u[j] = __builtin_amdgcn_raw_buffer_load_b32(
                rs, (real && kf + 8 * j >= 1) ? o : static_cast<int>(kOctOOR), 0, 0);
        }
        const uint32_t tr = (real && col == 0u) ? vrel + L - 4u : kOctOOR;
        if constexpr (MODE == kVerify) S.u[K] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(tr), 0, 0);
        S.tro = tr;
        S.kf = real ? kf : -(1 << 20);
        // routing: packet i of the block takes group (pos_i & 7)'s result when pos_i is in this set
        const uint32_t pi = LB.pos;
        const bool mine_i = ((LB.mine >> lane) & 1ull) != 0;
        const bool take = have && mine_i && (pi >> 3) == static_cast<uint32_t>(lset);
        S.rt = take ? (pi & 7u) << 3 : 0xFFu;
        const bool last = have && lset + 1 == LB.nsets;
        S.rq = (last && mine_i) ? static_cast<uint32_t>(LB.block) * 64u + lane : kOctOOR;
        if constexpr (TRAILER) S.boff = LB.boff;
        S.have = have;
        const uint32_t rfirst = readlane_u32(LB.key, (8 * lset) & 63) >> 6;  // sorted: the set's fewest rows
        S.full = have && rfirst == static_cast<uint32_t>(K);
        if (have) inflight += 1;
    };

    auto consume = [&](auto bc) __attribute__((always_inline)) {
        constexpr int b = decltype(bc)::value;
        OctSlot<K, MODE, TRAILER> &S = sl[b];
        if (!S.have) return;
        uint32_t acc = 0;
        if constexpr (DIAG == 1) {
#pragma unroll
            for (int j = 0; j < K; ++j) acc ^= S.u[j] | head_mask(S.kf + 8 * j);
        } else if (S.full) {  // every packet fills the frame: stream words 0..9 lie in rows 0..2
            const uint32_t m0 = head_mask(S.kf), m1 = head_mask(S.kf + 8), m2 = head_mask(S.kf + 16);
#pragma unroll
            for (int j = 0; j < K; ++j) {
                uint32_t u = S.u[j];
                if (j == 0) u |= m0;
                if (j == 1) u |= m1;
                if (j == 2) u |= m2;
                acc = j == 0 ? u : step_m64(lds, acc, u, c);
            }
        } else {  // head masks wherever this lane's stream words 0..9 fall (branch-free, every row)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t u = S.u[j] | head_mask(S.kf + 8 * j);
                acc = j == 0 ? u : step_m64(lds, acc, u, c);
            }
        }
        const uint32_t crc = ~group_xor<8>(DIAG == 1 ? acc : final_mul(lds, acc, c.fin));
        uint32_t r;
        if constexpr (MODE == kCompute) r = crc;
        else r = bperm(grp << 3, S.u[K]) == crc ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH;
        if constexpr (TRAILER) {  // PacketWriter stores the ICRC / is_icrc_valid zeroes it
            const __amdgpu_buffer_rsrc_t ts =
                __builtin_amdgcn_make_buffer_rsrc(p.base + S.boff, 0, static_cast<int>(kOctOOR), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(MODE == kCompute ? crc : 0u, ts, static_cast<int>(S.tro), 0, 0);
        }
        const uint32_t v = bperm(S.rt & 63u, r);
        rbv = S.rt != 0xFFu ? v : rbv;
        // the block's results leave after its last set, as one store every set issues (out of range
        // otherwise: no branch around a store in the ring)
        if constexpr (MODE == kCompute) {
            const __amdgpu_buffer_rsrc_t os =
                __builtin_amdgcn_make_buffer_rsrc(p.out ? p.out + lo : nullptr, 0, p.out ? static_cast<int>(nq * 4u) : 0,
                                                  0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(rbv, os, static_cast<int>(S.rq == kOctOOR ? kOctOOR : 4u * S.rq), 0, 0);
        } else {
            const __amdgpu_buffer_rsrc_t os =
                __builtin_amdgcn_make_buffer_rsrc(p.ok ? p.ok + lo : nullptr, 0, p.ok ? static_cast<int>(nq) : 0, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(rbv), os, static_cast<int>(S.rq), 0, 0);
        }
        inflight -= 1;
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
            if (oct_block<K, LMIN>(p, NB, off, L, valid, lo, nb_next, lane) != 0) irregular = true;
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
            issue(IntC<(b + D) % B>{});
            consume(bc);
            return true;
        });
        if (ldone && inflight == 0) break;
    }

    if (TAIL && irregular) {  // L < 44, misaligned, L % 4 != 0, far-apart offsets: per packet
        for (int b = 0; b < nblocks; ++b) {
            uint64_t off;
            uint32_t L;
            uint64_t m = oct_classify(p, lo, nq, b, lane, off, L);
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t o = static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off), l)) |
                                   (static_cast<uint64_t>(readlane_u32(static_cast<uint32_t>(off >> 32), l)) << 32);
                const uint32_t Ll = readlane_u32(L, l);
                const uint32_t r = quad_slow_packet<MODE, 8>(p, p.base + o, Ll, lds, c, lane);
                if (lane == 0) store_result<MODE>(p, lo + static_cast<uint32_t>(b) * 64u + static_cast<uint32_t>(l), r);
            }
        }
    }
}

template <int MODE, bool RAGGED, bool TRAILER, int DIAG>
__global__ __launch_bounds__(kThreadsPerGroup) void icrc_oct_kernel(BatchParams p) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    const uint32_t tw = gridDim.x * kWavesPerGroup;
    // chunks of whole 64-packet blocks (whole-line result stores) unless that idles waves
    uint32_t chunk = (p.n + tw - 1) / tw;
    chunk = chunk > 32u ? (chunk + 63u) & ~63u : (chunk + 7u) & ~7u;
    if (RAGGED && p.split_len != 0 && p.len != nullptr) {
        // Split batch: a workgroup whose packets are all the long-packet kernel's exits before
        // its 160 KiB table load.
        const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * kWavesPerGroup * chunk;
        const uint64_t g1 = g0 + static_cast<uint64_t>(kWavesPerGroup) * chunk;
        const uint64_t end = g1 < p.n ? g1 : p.n;
        bool any_short = false;
        for (uint64_t i = g0 + threadIdx.x; i < end; i += kThreadsPerGroup) any_short |= p.len[i] < p.split_len;
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
        const uint4 *src = reinterpret_cast<const uint4 *>(p.table_oct);
        for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += kThreadsPerGroup) lds4[i] = src[i];
    }
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
    const uint64_t lo64 = static_cast<uint64_t>(gw) * chunk;
    if (lo64 >= p.n) return;
    const uint32_t lo = static_cast<uint32_t>(lo64);
    const uint32_t nq = (p.n - lo) < chunk ? (p.n - lo) : chunk;
    // phase 1: L <= 320 in 10-row frames, 3 sets in flight; phase 2: 320 < L <= 1088 in 34-row
    // frames, its 34 loads in flight before the row steps (~7.5-8.5 KiB per wave in flight either way)
    run_oct<MODE, kOctK1, 3, RAGGED, TRAILER, 0, false, DIAG>(p, lds, c, lane, lo, nq);
    run_oct<MODE, kOctK2, 0, RAGGED, TRAILER, 32u * kOctK1, true, DIAG>(p, lds, c, lane, lo, nq);
}

}  // namespace

// Variant 40 (the default short-packet kernel): packets of at most 1088 bytes in two phases.
uint32_t oct_max_len() { return kOctMaxL; }

int launch_oct(int mode, const BatchParams &p, int grid, void *stream, int diag) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool ragged = p.off != nullptr || p.len != nullptr;
#define ICRC_O(M, R, T, G) hipLaunchKernelGGL((icrc_oct_kernel<M, R, T, G>), dim3(grid), dim3(kThreadsPerGroup), 0, s, p)
#define ICRC_OM(M)                                                   \
    do {                                                             \
        if (diag != 0 && M == kCompute && !p.trailer) {              \
            if (ragged) {                                            \
                if (diag == 1) ICRC_O(M, true, false, 1);            \
                else ICRC_O(M, true, false, 2);                      \
            } else {                                                 \
                if (diag == 1) ICRC_O(M, false, false, 1);           \
                else ICRC_O(M, false, false, 2);                     \
            }                                                        \
        } else if (ragged) {                                         \
            if (p.trailer) ICRC_O(M, true, true, 0);                 \
            else ICRC_O(M, true, false, 0);                          \
        } else {                                                     \
            if (p.trailer) ICRC_O(M, false, true, 0);                \
            else ICRC_O(M, false, false, 0);                         \
        }                                                            \
    } while (0)
    if (mode == kCompute) ICRC_OM(kCompute);
    else ICRC_OM(kVerify);
#undef ICRC_OM
#undef ICRC_O
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc
