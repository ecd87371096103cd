// icrc_internal.h — shared between the HIP kernels (icrc_kernels.hip) and the host engine.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "icrc.h"

namespace icrc {

// ---- LDS table image (identical layout in HBM and in LDS; copied linearly per workgroup) --
// Bulk tables B_b (b = 0..3): B_b[x] = M^64(x << 8b), M = "advance the reflected CRC-32
// state over 4 zero bytes".  32 copies, one per ds_read_b32 bank, so lane l always reads
// bank (l & 31):  byte address = (b >> 1) * 65536 + x * 256 + (b & 1) * 128 + (l & 31) * 4.
// Final per-lane tables F_l (l = 0..63): F_l[n][v] = M^(64-l)(v << 4n), nibble-indexed:
//   byte address = kFinalBase + (n * 16 + v) * 256 + l * 4.
constexpr uint32_t kLdsBytes = 163840;  // 160 KiB: the whole CU LDS
constexpr uint32_t kFinalBase = 131072;
constexpr uint32_t kLdsWords = kLdsBytes / 4;

// Host: fill a kLdsWords image.
void build_table_image(uint32_t *img);
// Oct image (eight packets per wavefront, 8 lanes each): M^8 bulk, M^(8 - (l & 7)) final.
void build_table_image_oct(uint32_t *img);
// Compact image, stored in HBM right after each full image (the device buffer holds
// kLdsWords + kCompactWords words): the 1024 distinct bulk entries (word b * 256 + x = B_b[x]),
// then the 32 KiB final tables exactly as at kFinalBase.  A workgroup reads these 36 KiB and
// replicates the bulk entries 32x into LDS itself (table_fill, icrc_device.h) instead of reading
// the 160 KiB image: 256 workgroups x 160 KiB = 40 MiB of table reads per launch becomes 9 MiB.
constexpr uint32_t kCompactWords = 1024u + (kLdsBytes - kFinalBase) / 4u;
constexpr uint32_t kTableBufWords = kLdsWords + kCompactWords;
void append_compact_image(uint32_t *img);  // img[kLdsWords ..] <- compact form of img[0 .. kLdsWords)
// Host reference helpers used by the table builder (exposed for unit tests).
uint32_t advance_words(uint32_t state, uint32_t nwords);  // M^nwords(state)

// ---- kernel launch parameters ------------------------------------------------------------
// Work skew of a workgroup's persistent waves, in 1/1024: the four waves of a SIMD are served by
// age (the oldest wins issue arbitration), so with equal shares the oldest finish first and the
// youngest run the tail alone (diagnostic 53: ends at 200 / 217 / 237 / 260 us on 4 Mi x 316 B,
// identical run to run).  Wave slot k (age rank a = k / 4) takes a share 1 + e (3 - 2a) / 1024;
// e for the oct kernel in bits 0-11, for the one-packet pipeline (batch and long-packet
// workgroups) in bits 16-27; bits 12-13 / 28-29: the shares' unit, 8 << that packets (the oct
// kernel counts its blocks from its own first packet, so one set will do; the one-packet pipeline
// keeps 64-packet blocks: whole-line result stores).  Units of one set measured no better than
// whole blocks for the oct kernel (profiles/r03_probe_skew_unit.jsonl).
constexpr uint32_t kWaveSkewOct = 45u | (3u << 12);  // probe_skew.py: C2 -3.6 %, 316 B -2 %, 1 KiB -3.4 %
// The batch kernel's one-packet pipeline (C1: 4 blocks per wave, too coarse for whole-block
// shares; units of 8 packets): e = 180, C1 -2.9 %, C1 verify -2 % (profiles/r03_probe_skew_long.jsonl).
// The hybrid launch's long-packet workgroups keep equal shares (long_body).  (A/B:
// ICRC_AB_SKEW_OCT / ICRC_AB_SKEW_LONG.)
constexpr uint32_t kWaveSkewLong = 180u;
constexpr uint32_t kWaveSkew = kWaveSkewOct | (kWaveSkewLong << 16);

struct BatchParams {
    uint8_t *base;
    const uint64_t *off;  // nullptr => strided (offset = i * stride)
    const uint32_t *len;  // nullptr => uniform length ulen
    uint64_t stride;
    uint32_t ulen;
    uint32_t n;
    uint32_t *out;   // compute: ICRC per packet (may be null)
    uint8_t *ok;     // verify: 1/0/0xFF per packet
    uint32_t *nerr;  // may be null
    const uint32_t *table;  // kLdsWords image in device memory
    int trailer;     // compute: write trailer; verify: zero trailer
    int variant;     // kernel variant (icrc_kernels.hip launch_mode): 0 = unpipelined, 1..5 = pipelined
    icrc_rx_desc *rx;  // receive parse (launch_rx): one descriptor per packet
    const uint32_t *table_oct;   // kLdsWords oct image (W = 8: variants 40-53)
    uint32_t split_len;  // hybrid dispatch (0 = off): the oct kernel takes L < split_len, the
                         // long-packet kernel (launch_long) L >= split_len
    int long_variant;    // launch_long: 0 = filtered S = 2 pipeline (default), 1 = compacting S = 1 walker
    int spread;          // one-packet pipeline: consecutive waves' packets on different workgroups
                         // (small host-mapped batches: more CUs issue PCIe reads at once)
    uint32_t skew = kWaveSkew;  // persistent waves' work shares by age (wave_range, icrc_device.h)
    // ragged one-pass receive: the sweep (icrc_rx_sweep_kernel) runs only when the ring found packets
    // it leaves to it (its tail loop's): the ring raises *rx_flag to rx_gen (atomicMax), the sweep
    // exits when *rx_flag < rx_gen.  rx_gen grows per call of the engine (0: no flag, always sweep).
    uint32_t *rx_flag = nullptr;
    uint32_t rx_gen = 0;
    uint32_t ab_long_walk = 0;  // (A/B library only: ICRC_AB_LONG_WALK=1, run_walk_masked)
};

constexpr int kDefaultVariant = 16;  // S=2 chains, D=1, nt row loads (A/B: profiles/r01_ab_c1_depth.json)
constexpr int kDefaultRaggedVariant = 40;  // oct, fixed 10-row frames (icrc_oct.hip): L <= 320
constexpr int kOctVariant = 40;
// 100 + q (q an oct variant): the default hybrid dispatch with q as its short-packet kernel.
constexpr int kHybridVariantBase = 100;
// 200 + q: the same with the compacting long-packet walker (A/B); 301: the fused single-pass
// receive parse (A/B against the two-pass default).
constexpr int kHybridCompactBase = 200;
constexpr int kRxVariantBase = 300;
// Variants a batch can be forced to (icrc_engine_set_kernel_variant).  The product library
// accepts only result-exact ones: 0, 13, 16, 17 (one packet per wave) and 40 (oct).  The A/B
// library (built with ICRC_AB_BUILD: _build/libicrc_amd_ab.so, for measurement scripts and the
// bench's loads-only denominator) adds the diagnostics 15, 18, 19, 21-23, 27-30, 33, 41-53, whose results are
// wrong by design (49 and 51 are exact on strided batches only / on all batches, 48, 52 and 53
// exact, but ablations all the same).
#ifdef ICRC_AB_BUILD
inline bool is_batch_variant(int v) {
    switch (v) {
    case 0: case 13: case 15: case 16: case 17: case 18: case 19: case 21: case 22: case 23:
    case 27: case 28: case 29: case 30: case 33:
    case 40: case 41: case 42: case 43: case 44: case 45: case 46: case 47: case 48: case 49: case 50: case 51: case 52: case 53:
        return true;
    default:
        return false;
    }
}
inline bool is_short_variant(int v) { return v >= 40 && v <= 53; }
#else
inline bool is_batch_variant(int v) { return v == 0 || v == 13 || v == 16 || v == 17 || v == 40; }
inline bool is_short_variant(int v) { return v == 40; }
#endif

enum Mode : int { kCompute = 0, kVerify = 1 };

constexpr int kWavesPerGroup = 16;                // 1024-thread workgroup, 1 per CU (LDS-bound)
constexpr int kThreadsPerGroup = 64 * kWavesPerGroup;

// Launch wrappers (icrc_kernels.hip).  `grid` = number of workgroups.
int launch_batch(int mode, const BatchParams &p, int grid, void *stream);
// One-packet pipeline over the packets with L >= p.split_len of a ragged batch (hybrid dispatch).
int launch_long(int mode, const BatchParams &p, int grid, void *stream);
int launch_rx(const BatchParams &p, int grid, void *stream);  // fused verify + parse (p.rx), variants 1-3
// Receive parse pass 2 (the default path): descriptors from the header words, icrc_ok read from
// p.ok where the verify pass left it.
int launch_rx_desc(const BatchParams &p, int num_cu, void *stream);
// Fixed-frame oct kernel (icrc_oct.hip), variant 40: packets of at most oct_max_len() bytes.
int launch_oct(int mode, const BatchParams &p, int grid, void *stream, int diag = 0);
uint32_t oct_max_len();
// The fused receive (icrc_oct.hip, icrc_oct_rx_kernel): verify + descriptors in one pass over a
// strided batch whose packets are all the oct kernel's (44 <= L <= oct_max_len(), 4-aligned).
// diag (A/B library only, ICRC_AB_RX_OCT=2..5): the kernel's cuts (OctRxAblation, icrc_oct.hip).
int launch_oct_rx(const BatchParams &p, int grid, void *stream, int diag = 0);
// The same for ragged batches, two launches (icrc_hybrid_rx_kernel: the oct ring on L < p.split_len,
// long_body's verify on the rest; icrc_rx_sweep_kernel: descriptors for every packet the ring did not
// take); p.ok must be set.  Workgroup ranges must be whole 64-packet blocks (more than 32 packets
// per wave of the grid).
int launch_hybrid_rx(const BatchParams &p, int grid, int num_cu, void *stream);
// The hybrid dispatch with the oct kernel as its short-packet half, in one launch (icrc_oct.hip):
// grid_oct workgroups of the oct kernel, then grid_long of the long-packet kernel.
int launch_hybrid(int mode, const BatchParams &p, int grid_oct, int grid_long, void *stream);
// The length from which the hybrid dispatch hands packets to the long-packet kernel: what the
// fixed-frame oct kernel can hold.
inline uint32_t split_len_for(int) { return oct_max_len() + 1u; }
int launch_synth(uint8_t *base, const icrc_synth_desc *desc, const uint8_t *hdr, uint32_t n,
                 void *stream);
struct PacketizeParams {
    const uint8_t *src;
    uint64_t src_bytes;
    const icrc_write_msg *msgs;
    uint32_t nmsgs;
    uint32_t npackets;
    uint8_t *wire;
    uint64_t wire_bytes;
    uint32_t *pkt_len;
    uint32_t *icrc;
    const uint32_t *table;
};
int launch_packetize(const PacketizeParams &p, int grid, void *stream);
int launch_ack(const icrc_rx_desc *desc, const icrc_ack_ctx *ctx, uint32_t n, uint8_t *out, uint32_t stride,
               uint32_t *out_len, uint32_t mode, int num_cu, void *stream);
int launch_ipv4_checksum(uint8_t *base, const uint64_t *off, uint64_t stride, uint32_t n, uint16_t *csum, int fill,
                         void *stream);

// ---- host-message submission ring (icrc_ring.cpp: host protocol; icrc_ring_kernel: service) ----
// The emulator's own call model is a doorbell and a queue its send thread drains
// (blue-rdma-device/src/queues/send/queue.rs:66-100, rust_driver/src/device/ringbuf.rs:201-209).
// Here: a resident service kernel keeps the W = 64 tables in LDS and polls a ring of job slots in
// coherent pinned host memory; a host caller fills a free slot (one message: a scalar packet or a
// host batch of at most kRingMaxPackets) and publishes it by writing the slot's cmd word last.
// Slot s is served by kRingWgPerSlot workgroups.  While idle only wave 0 of each workgroup runs: it
// polls the slot's line, and on a new job writes it into its workgroup's decision line in device
// memory; the workgroup then takes its share of the job in lockstep (a barrier before and after)
// and its wave 0 writes the cmd into the workgroup's done word, so the host sees completion without
// any atomic.  The kernel ends when the
// host sets kRingStop, or when a leader has seen no call for RingParams::idle_ticks or has run for
// life_ticks (it sets the exit flag, which every workgroup polls between jobs: one leader ends them all,
// so a half-alive kernel never holds a slot); the host relaunches it on the next call, and re-runs a job
// whose launch ended under it.
constexpr uint32_t kRingStop = 0x80000000u;  // RingSlot::cmd: every wave exits
constexpr uint32_t kRingMaxPackets = 1024u;  // packets per job (one message)
constexpr uint32_t kRingMaxSlots = 16u;
constexpr uint32_t kRingSlots = 4u;          // default: one per emulator thread (3) + one
// Default shape: 8 workgroups of 256 threads per slot, i.e. a message's loads spread over 8 CUs
// (one CU pulls host memory at ~25 GB/s, four at ~56: scripts/hostreadbench.hip), 32 CUs in all.
// 3 threads 64-65 K messages/s against 56-57 K for 2 x 1024 (profiles/r05/ring/r05i).
constexpr uint32_t kRingThreads = 256u;      // default workgroup size of the service kernel
constexpr uint32_t kRingWgPerSlot = 8u;      // default workgroups per slot (CUs reading one message)
struct alignas(64) RingSlot {  // host-written, one 64-byte line per slot
    uint32_t cmd;       // job number (bits 0-30, never 0 for a job) | kRingStop; written last
    uint32_t activity;  // the host's submission counter, copied into every slot on every call
    uint32_t n;         // packets
    uint32_t ulen;      // uniform length (packet i at base + i * stride) or 0 (off / len arrays)
    uint64_t base;      // device address of the packet bytes (mapped host memory)
    uint64_t stride;
    uint64_t off;       // device address of n u64 offsets from base (ulen == 0)
    uint64_t len;       // device address of n u32 lengths (ulen == 0)
    uint64_t out;       // device address of n u32 ICRCs (coherent mapped host memory)
    uint32_t reserved;  // 0
    uint32_t hash;      // ring_line_hash of the line, written before cmd: the kernel reads the line in
                        // one load per poll and takes its fields only when the hash matches (a read
                        // torn by the host's writes is read again)
};
static_assert(sizeof(RingSlot) == 64, "one line per slot");
#ifdef __HIPCC__
#define ICRC_HD __host__ __device__
#else
#define ICRC_HD
#endif
// Hash of a slot line's dwords 0 (cmd) and 2..14 (the job), kept in dword 15.
ICRC_HD inline uint32_t ring_line_hash(uint32_t h, uint32_t d) {
    h ^= d;
    h *= 0x85EBCA6Bu;
    return h ^ (h >> 13);
}
ICRC_HD inline uint32_t ring_line_hash(const uint32_t *w) {
    uint32_t h = ring_line_hash(0x9E3779B9u, w[0]);
    for (int k = 2; k < 15; ++k) h = ring_line_hash(h, w[k]);
    return h;
}
struct RingParams {
    const RingSlot *slots;  // device view of the slot lines (host memory)
    uint32_t *done;         // [slot][wg]: the last cmd each workgroup finished (host memory)
    uint32_t *exited;       // [slot][wg]: epoch, stored when the workgroup ends (host memory)
    uint32_t *exit_flag;    // device memory: epoch once a leader has timed out
    RingSlot *decision;     // device memory [slot][wg]: wave 0's decision (the job, or kRingStop)
    const uint32_t *table;  // W = 64 table buffer (image + compact form)
    uint32_t wg_per_slot;
    uint32_t threads;       // workgroup size, 256 / 512 / 1024: one workgroup per CU either way (the
                            // 160 KiB table image), so fewer threads spread a job over more CUs
    uint32_t epoch;         // launch number
    uint32_t idle_ticks;    // s_memrealtime ticks (100 MHz) without host activity before exiting
    uint32_t life_ticks;    // ... and since the launch: a launch ends at a job boundary after this long,
                            // so a kernel that needs every CU (the batch kernels: one 160 KiB workgroup
                            // per CU) waits at most that long for the CUs the ring holds
    uint32_t ab;            // A/B library only (ICRC_RING_AB, diagnostic cuts): 1 no acquire, 2 a
                            // release fence after the results, 4 no sleep between polls, 8 no compute; 0 in the product
    uint64_t *trace;        // A/B library only (ICRC_RING_TRACE): per slot, kRingTraceJobs records of
                            // s_memrealtime stamps {cmd seen, job decoded, results complete, done
                            // stored} by the slot's first workgroup; nullptr in the product
};
constexpr uint32_t kRingTraceJobs = 4096;
int launch_ring(const RingParams &rp, uint32_t nslots, void *stream);

// Segmentation shared by host and tests (generate_segments_from_request, common.rs:152-176).
inline uint32_t write_first_segment(uint64_t local_va, uint32_t total_len, uint32_t pmtu) {
    const uint32_t first = pmtu - static_cast<uint32_t>(local_va) % pmtu;
    return total_len < first ? total_len : first;
}

}  // namespace icrc
