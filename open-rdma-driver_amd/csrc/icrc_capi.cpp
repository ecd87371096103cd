// icrc_capi.cpp — the C-ABI of include/icrc.h: engines, scalar drop-ins, host- and
// device-resident batches.  Every CRC is computed by the HIP kernel (icrc_kernels.hip);
// this file only moves bytes and launches.  There is deliberately no CPU CRC here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "icrc_internal.h"
#include "icrc_ring.h"

namespace {

// One stage of the host-resident pipeline: device + pinned host buffers, a stream, an event.
struct Stage {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t *d_buf = nullptr;
    size_t d_cap = 0;
    uint64_t *d_off = nullptr;
    uint32_t *d_len = nullptr;
    uint32_t *d_res = nullptr;
    size_t meta_cap = 0;
    uint8_t *h_buf = nullptr;  // pinned gather buffer
    size_t h_cap = 0;
    uint64_t *h_off = nullptr;  // pinned
    uint32_t *h_len = nullptr;  // pinned
    uint32_t *h_res = nullptr;  // pinned
    // chunk in flight
    bool busy = false;
    uint32_t i0 = 0, cnt = 0;
};

// One call waiting for the combining submitter: a scalar call (icrc_compute / icrc_verify, n = 1)
// or a small host batch (one message's packets, icrc_compute_batch / icrc_verify_batch).  Always
// an ICRC computation: verify compares with the trailer on the calling thread.
struct SubmitReq {
    const uint8_t *dbase;   // device view of the packets (a thread's mapped slot or the caller's pinned buffer)
    const uint64_t *off;    // n offsets from dbase (host memory of the caller)
    const uint32_t *len;    // n lengths
    uint32_t n;
    uint32_t *res;          // n ICRCs (host memory of the caller)
    int rc = ICRC_OK;
    bool taken = false;     // in a launch (by this caller or another leader)
    bool done = false;      // results handed out
};

// One launch lane of the submitter: a stream and the mapped (offset, length, result) arrays of the
// launch it carries.  A lane is busy from the moment a leader takes it until the leader has handed
// out its results.
struct Lane {
    hipStream_t stream = nullptr;
    uint64_t *h_off = nullptr;  // pinned + mapped: packet offsets from the batch base
    uint32_t *h_len = nullptr;
    uint32_t *h_res = nullptr;
    uint64_t *d_off = nullptr;  // their device views
    uint32_t *d_len = nullptr;
    uint32_t *d_res = nullptr;
    bool busy = false;
};

// The combining submitter: concurrent calls (the emulator's send, packet-handler and receive
// threads, packet_processor.rs:260 / udp_agent.rs:99) queue here.  A caller whose call is still
// queued and who finds a free lane becomes that lane's leader: it takes the queued calls (up to cap
// packets), runs them as ONE compute launch on the lane's stream and waits for it on that stream
// alone, then hands out the results.  With kLanes lanes, up to kLanes launches are in flight at once
// (the emulator's three threads each get a lane; more callers than lanes combine into the next
// launch).  Packets are read by the kernel straight from pinned, device-mapped host memory (no copy
// engine); results come back through mapped pinned memory.
struct Combiner {
    // Four streams.  They do not own hardware queues: with GPU_MAX_HW_QUEUES = 4 HIP shares the
    // process's four queues among every stream (these, the engine's, the staging and the callers'
    // streams), so a lane's launch can queue behind another stream's kernel on the same queue.
    static constexpr int kLanes = 4;
    static constexpr uint32_t kCap = 4096;    // array capacity per lane
    std::mutex mu;
    std::condition_variable cv;
    std::vector<SubmitReq *> pending;
    Lane lanes[kLanes];
    uint32_t cap = kCap;  // packets per launch: min(kCap, #CUs x 16) keeps every launch on the one-packet
                          // pipeline, whose loads stay inside each packet (callers' buffers are unrelated
                          // host allocations; the oct kernel reads a short packet's rows up to its block end)
};

// The submission ring's device side (icrc_ring.h RingDevice): the service kernel on a stream of its
// own.  That stream is created with a CU mask (every CU) because a CU-masked stream gets a hardware
// queue of its own: a resident kernel on a queue that another stream shares would hold that stream's
// later kernels behind it.
struct RingHip final : icrc::RingDevice {
    int device = 0;
    hipStream_t stream = nullptr;
    bool dedicated = false;  // the stream was created with a CU mask
    icrc::RingParams rp{};
    uint32_t nslots = 0;
    int launch(uint32_t epoch) override;
    int ended() override;
};
struct RingState {
    RingHip dev;
    void *host = nullptr;        // the coherent mapped block (slots, done / exited words, slot arrays)
    uint8_t *d_mem = nullptr;    // device memory: exit flag | decision lines
    std::unique_ptr<icrc::HostRing> ring;
};
constexpr uint64_t kRingWatchdogUs = 2000000;  // a job not done in 2 s fails with ICRC_ETIMEDOUT
constexpr uint32_t kRingIdleTicks = 200000;    // 2 ms (s_memrealtime, 100 MHz) without a call: the kernel ends
constexpr uint32_t kRingLifeTicks = 100000;    // 1 ms after its launch a busy kernel ends between jobs

}  // namespace

struct icrc_engine {
    int device = 0;
    int num_cu = 0;
    int variant = -1;  // -1: kDefaultVariant for strided batches, kDefaultRaggedVariant otherwise
    uint32_t *d_table = nullptr;
    uint32_t *d_table_oct = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;  // the long-packet half of a split batch runs here, beside the caller's
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    std::mutex fork_mu;  // orders the fork / join event pair between threads
    std::mutex mu;  // guards the host-batch stages
    Stage st[2];
    std::mutex comb_init_mu;
    std::unique_ptr<Combiner> comb;  // scalar calls (created on first use)
    std::atomic<int> host_path{ICRC_HOST_RING};  // scalar calls and host messages: the submission ring or launches
    std::mutex ring_mu;
    std::unique_ptr<struct RingState> ring;  // the submission ring (created on first use)
    uint32_t *d_rx_flag = nullptr;          // the ragged receive's sweep flag (BatchParams::rx_flag)
    std::atomic<uint32_t> rx_gen{0};        // ... and its per-call generation
};

namespace {

using icrc::BatchParams;

// icrc_shutdown (include/icrc.h) has run: every engine is gone and no entry point makes a HIP call
// any more (DeviceGuard refuses, the scalar / default-engine paths check first).  Counted refusals are
// the teardown test's evidence (icrc_teardown_stats).
std::atomic<bool> g_shutdown{false};
std::atomic<uint64_t> g_refused_after_shutdown{0};
std::atomic<uint64_t> g_engines_torn_down{0};
std::atomic<uint64_t> g_slots_freed_at_shutdown{0};
bool shut_down() {
    if (!g_shutdown.load(std::memory_order_acquire)) return false;
    g_refused_after_shutdown.fetch_add(1, std::memory_order_relaxed);
    return true;
}

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (shut_down()) {  // no HIP call after icrc_shutdown
            ok = false;
            return;
        }
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(expr)                                  \
    do {                                               \
        if ((expr) != hipSuccess) return ICRC_EDEVICE; \
    } while (0)

int grid_for(const icrc_engine *e, uint32_t n);

// Dispatch knobs.  The product runs the defaults; the A/B library (ICRC_AB_BUILD) reads them from
// the environment on every call, so that one process can time the alternatives on one box (the
// records of each are under profiles/).
struct DispatchKnobs {
    uint32_t spread_per_wg = 1;  // ICRC_AB_SPREAD: packets per workgroup of a spread launch
    int skew = -1, skew_oct = -1, skew_long = -1;  // ICRC_AB_SKEW[_OCT|_LONG]: the waves' work skew
    uint32_t split = 0;          // ICRC_AB_SPLIT: the length split of ragged batches (0: the variant's)
    int hybrid_seq = 0;          // ICRC_AB_HYBRID_SEQ: 1 / 2 = the halves as two kernels in a row (oct / long first)
    int long_grid_mult = 1;      // ICRC_AB_LONG_GRID: long-packet workgroups per oct workgroup
    int long_cus = 0;            // ICRC_AB_LONG_CUS: CUs running long-packet workgroups from the start
    int long_self = 1;           // ICRC_AB_LONG_SELF=0: the two workgroup sets (oct, then long-packet ones)
    int self_grid_mult = 1;      // ICRC_AB_SELF_GRID: workgroups per CU of the in-place hybrid (smaller ranges)
    int long_walk = 0;           // ICRC_AB_LONG_WALK=1: run_walk_masked (icrc_long.h; measured, rejected)
    int small_ppw = 2;           // packets per wave of a small batch's grid (ICRC_AB_SMALL_PPW)
};
DispatchKnobs dispatch_knobs() {
    DispatchKnobs k;
#ifdef ICRC_AB_BUILD
    auto env = [](const char *name, int dflt) {
        const char *v = std::getenv(name);
        return v ? std::atoi(v) : dflt;
    };
    k.spread_per_wg = static_cast<uint32_t>(std::max(1, std::min(16, env("ICRC_AB_SPREAD", 1))));
    k.skew = env("ICRC_AB_SKEW", -1);
    k.skew_oct = env("ICRC_AB_SKEW_OCT", -1);
    k.skew_long = env("ICRC_AB_SKEW_LONG", -1);
    k.split = static_cast<uint32_t>(std::max(0, env("ICRC_AB_SPLIT", 0)));
    k.hybrid_seq = env("ICRC_AB_HYBRID_SEQ", 0);
    k.long_grid_mult = std::max(1, env("ICRC_AB_LONG_GRID", 1));
    k.long_cus = env("ICRC_AB_LONG_CUS", 0);
    k.long_self = env("ICRC_AB_LONG_SELF", 1);
    k.self_grid_mult = std::max(1, std::min(8, env("ICRC_AB_SELF_GRID", 1)));
    k.long_walk = env("ICRC_AB_LONG_WALK", 0);
    k.small_ppw = std::max(1, std::min(16, env("ICRC_AB_SMALL_PPW", 2)));
#endif
    return k;
}

// Launch a batch.  A variant forced on the engine runs alone.  A batch of at most one packet per
// wave runs on the one-packet pipeline alone.  Otherwise: a uniform strided
// batch runs on the one-packet pipeline (kDefaultVariant) when its packets are long, on the oct
// kernel (kDefaultRaggedVariant) when short; a ragged batch is split by length (hybrid
// dispatch): the oct kernel takes L < split (and every packet off the fast paths), the long-packet
// kernel the rest — by default one launch of the fused hybrid kernel (icrc_oct.hip), whose
// long-packet workgroups take each CU as the oct ones retire; under a forced hybrid variant (A/B)
// two kernels on the caller's stream and the engine's side stream, forked and joined by events.
int dispatch(icrc_engine *e, int mode, BatchParams p, void *stream) {
    const DispatchKnobs k = dispatch_knobs();
    // spread (small host-mapped batches): one workgroup per packet up to #CUs, so that as many CUs
    // as possible read host memory over PCIe at once
    const int grid = p.spread ? static_cast<int>(std::min<uint32_t>(std::max<uint32_t>((p.n + k.spread_per_wg - 1) / k.spread_per_wg, 1u),
                                                                    static_cast<uint32_t>(e->num_cu)))
                              : grid_for(e, p.n);
    p.split_len = 0;
    p.ab_long_walk = static_cast<uint32_t>(k.long_walk);
    if (k.skew >= 0) p.skew = static_cast<uint32_t>(k.skew) * 0x10001u;
    if (k.skew_oct >= 0) p.skew = (p.skew & 0xFFFF0000u) | (static_cast<uint32_t>(k.skew_oct) & 0xFFFFu);
    if (k.skew_long >= 0) p.skew = (p.skew & 0xFFFFu) | (static_cast<uint32_t>(k.skew_long) << 16);
    if (e->variant >= 0 && e->variant < icrc::kHybridVariantBase) {
        p.variant = e->variant;
        return icrc::launch_batch(mode, p, grid, stream);
    }
    const bool hybrid_forced = e->variant >= icrc::kHybridVariantBase && e->variant < icrc::kRxVariantBase;
    // Small batches (at most one packet per wave of the grid, e.g. a 16 MiB message = 4096 packets):
    // the one-packet pipeline alone — packing short packets eight to a wave buys nothing when
    // every packet has a wave of its own, and the split's second launch and fork / join cost more
    // than the kernels (C3 round trip 0.069 -> 0.020 ms).  Two packets per wave (one set of the
    // pipeline: both packets' rows in flight together) on half the workgroups: C3 9.9 -> 9.6 us per
    // launch (rocprof), 4 or 8 per wave 13.5 / 21 us (profiles/r06/c3/c3_grid_ppw.jsonl).
    if (!hybrid_forced && p.n <= static_cast<uint32_t>(e->num_cu) * icrc::kWavesPerGroup) {
        p.variant = icrc::kDefaultVariant;
        if (k.small_ppw > 1 && !p.spread) {
            const uint32_t per_wg = icrc::kWavesPerGroup * static_cast<uint32_t>(k.small_ppw);
            return icrc::launch_batch(mode, p, static_cast<int>(std::max<uint32_t>(1u, (p.n + per_wg - 1) / per_wg)), stream);
        }
        return icrc::launch_batch(mode, p, grid, stream);
    }
    p.long_variant = e->variant >= icrc::kHybridCompactBase && hybrid_forced ? 1 : 0;
    const int short_variant = !hybrid_forced ? icrc::kDefaultRaggedVariant
                            : e->variant - (p.long_variant ? icrc::kHybridCompactBase : icrc::kHybridVariantBase);
    const uint32_t split = icrc::split_len_for(short_variant);
    if (p.off == nullptr && p.len == nullptr) {
        p.variant = p.ulen >= split ? icrc::kDefaultVariant : short_variant;
        return icrc::launch_batch(mode, p, grid, stream);
    }
    p.variant = short_variant;
    p.split_len = k.split ? std::min(split, k.split) : split;
    // Default: both halves in one launch (the fused hybrid kernel).  A forced hybrid variant
    // (100 + q, 200 + q: A/B) keeps the two-stream fork / join below.
    if (!hybrid_forced) {
        if (k.hybrid_seq == 1 || k.hybrid_seq == 2) {
            const bool oct_first = k.hybrid_seq == 1;
            int rc = oct_first ? icrc::launch_batch(mode, p, grid, stream) : icrc::launch_long(mode, p, grid, stream);
            if (rc == ICRC_OK) rc = oct_first ? icrc::launch_long(mode, p, grid, stream) : icrc::launch_batch(mode, p, grid, stream);
            return rc;
        }
        if (k.long_cus > 0 && k.long_cus < grid) return icrc::launch_hybrid(mode, p, grid - k.long_cus, k.long_cus, stream);
        if (k.long_self) return icrc::launch_hybrid(mode, p, grid * k.self_grid_mult, 0, stream);
        return icrc::launch_hybrid(mode, p, grid, grid * k.long_grid_mult, stream);
    }
    std::lock_guard<std::mutex> g(e->fork_mu);
    HIP_TRY(hipEventRecord(e->fork_ev, static_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamWaitEvent(e->side, e->fork_ev, 0));
    int rc = icrc::launch_batch(mode, p, grid, stream);
    if (rc == ICRC_OK) rc = icrc::launch_long(mode, p, grid, e->side);
    HIP_TRY(hipEventRecord(e->join_ev, e->side));
    HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), e->join_ev, 0));
    return rc;
}

// Live rings (every engine's, with its device), never destroyed: stopped at process exit if
// icrc_shutdown never ran (ring_atexit); read by the A/B grid below.
struct RingEntry {
    int device;
    icrc::HostRing *ring;
};
std::mutex g_ring_mu;
std::vector<RingEntry> &g_rings = *new std::vector<RingEntry>();

// (A/B, ICRC_AB_RING_AWARE=1) a device batch's grid without the CUs the engine's submission ring
// holds while its service kernel is resident (one 160 KiB-LDS workgroup per CU, 32 by default).
// Measured and rejected (scripts/probe_ring_c1.py): C1 with a busy
// ring 0.78-0.80 ms on the full grid (its queued workgroups start as the ring's kernel ends, within
// its 1 ms life) against 0.84-0.86 on the smaller grid (the ring's CUs idle once its kernel ends),
// 0.72 alone.  The product keeps the full grid.
int free_cus(const icrc_engine *e) {
#ifdef ICRC_AB_BUILD
    static const bool aware = [] {
        const char *v = std::getenv("ICRC_AB_RING_AWARE");
        return v && std::atoi(v) != 0;
    }();
    if (aware) {
        int held = 0;  // any engine's ring on this device
        {
            std::lock_guard<std::mutex> lk(g_ring_mu);
            for (const RingEntry &r : g_rings)
                if (r.device == e->device && r.ring->live()) held += static_cast<int>(r.ring->workgroups());
        }
        return held < e->num_cu ? e->num_cu - held : e->num_cu;
    }
#endif
    return e->num_cu;
}

int grid_for(const icrc_engine *e, uint32_t n) {
    const uint64_t want = (static_cast<uint64_t>(n) + icrc::kWavesPerGroup - 1) / icrc::kWavesPerGroup;
    return static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(want, static_cast<uint64_t>(free_cus(e)))));
}

void stage_free(Stage &s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.d_buf) (void)hipFree(s.d_buf);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_len) (void)hipFree(s.d_len);
    if (s.d_res) (void)hipFree(s.d_res);
    if (s.h_buf) (void)hipHostFree(s.h_buf);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.h_res) (void)hipHostFree(s.h_res);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Stage{};
}

int stage_reserve(Stage &s, size_t bytes, size_t pkts, bool need_host_buf) {
    if (!s.stream) {
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return ICRC_EDEVICE;
        if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return ICRC_EDEVICE;
    }
    if (bytes > s.d_cap) {
        if (s.d_buf) (void)hipFree(s.d_buf);
        s.d_buf = nullptr;
        s.d_cap = 0;
        const size_t cap = std::max<size_t>(bytes, size_t(1) << 20);
        if (hipMalloc(&s.d_buf, cap + 64) != hipSuccess) return ICRC_ENOMEM;
        s.d_cap = cap;
    }
    if (need_host_buf && bytes > s.h_cap) {
        if (s.h_buf) (void)hipHostFree(s.h_buf);
        s.h_buf = nullptr;
        s.h_cap = 0;
        const size_t cap = std::max<size_t>(bytes, size_t(1) << 20);
        if (hipHostMalloc(&s.h_buf, cap, hipHostMallocDefault) != hipSuccess) return ICRC_ENOMEM;
        s.h_cap = cap;
    }
    if (pkts > s.meta_cap) {
        for (void *p : {static_cast<void *>(s.d_off), static_cast<void *>(s.d_len), static_cast<void *>(s.d_res)})
            if (p) (void)hipFree(p);
        for (void *p : {static_cast<void *>(s.h_off), static_cast<void *>(s.h_len), static_cast<void *>(s.h_res)})
            if (p) (void)hipHostFree(p);
        s.d_off = nullptr;
        s.d_len = nullptr;
        s.d_res = nullptr;
        s.h_off = nullptr;
        s.h_len = nullptr;
        s.h_res = nullptr;
        s.meta_cap = 0;
        const size_t cap = std::max<size_t>(pkts, 4096);
        if (hipMalloc(&s.d_off, cap * 8) != hipSuccess || hipMalloc(&s.d_len, cap * 4) != hipSuccess ||
            hipMalloc(&s.d_res, cap * 4) != hipSuccess ||
            hipHostMalloc(&s.h_off, cap * 8, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&s.h_len, cap * 4, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&s.h_res, cap * 4, hipHostMallocDefault) != hipSuccess)
            return ICRC_ENOMEM;
        s.meta_cap = cap;
    }
    return ICRC_OK;
}

bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error; clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Engine registries, never destroyed (a thread or handler running after static destruction must not
// find them gone): every live engine (icrc_engine_destroy refuses one it does not hold, so a handle
// destroyed by icrc_shutdown and then by its owner is not freed twice) and the default engines.
std::recursive_mutex g_registry_mu;  // recursive: icrc_engine_default creates under it
std::map<int, icrc_engine *> &g_default = *new std::map<int, icrc_engine *>();
std::set<icrc_engine *> &g_engines = *new std::set<icrc_engine *>();

int validate_host(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n) {
    if (n == 0) return ICRC_OK;
    if (!base || !off || !len) return ICRC_EINVAL;
    for (uint32_t i = 0; i < n; i++)
        if (len[i] < ICRC_MIN_PACKET) return ICRC_EINVAL;  // the reference panics here
    return ICRC_OK;
}

// Gathering pageable packets into pinned staging is the host-resident path's bound (one core copies
// at ~22 GiB/s, PCIe takes ~51): the copy is split over a small pool of host threads, the calling
// thread included.  Workers (ICRC_HOST_COPY_THREADS, default min(8, cores / 2), 1 = no pool) are
// started on first use and joined at exit; tasks are packet ranges taken from an atomic counter.
class CopyPool {
   public:
    static CopyPool &get() {
        static CopyPool pool;
        return pool;
    }
    // Runs fn(t) for t in [0, ntasks) on the workers and the caller; returns when all are done.
    // Each job has its own counters, so a worker still leaving an earlier job never touches this one.
    template <class F>
    void run(uint32_t ntasks, F &&fn) {
        if (th_.empty() || ntasks < 2) {
            for (uint32_t t = 0; t < ntasks; ++t) fn(t);
            return;
        }
        auto job = std::make_shared<Job>();
        job->fn = fn;
        job->n = ntasks;
        {
            std::lock_guard<std::mutex> lk(mu_);
            cur_ = job;
            ++gen_;
        }
        cv_.notify_all();
        work(*job);
        while (job->done.load(std::memory_order_acquire) < ntasks) std::this_thread::yield();
        std::lock_guard<std::mutex> lk(mu_);
        if (cur_ == job) cur_.reset();
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }

   private:
    struct Job {
        std::function<void(uint32_t)> fn;
        uint32_t n = 0;
        std::atomic<uint32_t> next{0}, done{0};
    };
    CopyPool() {
        unsigned n = std::max(1u, std::thread::hardware_concurrency() / 2u);
        n = std::min(n, 8u);
        if (const char *v = std::getenv("ICRC_HOST_COPY_THREADS")) n = static_cast<unsigned>(std::max(1, std::min(64, std::atoi(v))));
        for (unsigned i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    static void work(Job &j) {
        for (;;) {
            const uint32_t t = j.next.fetch_add(1);
            if (t >= j.n) return;
            j.fn(t);
            j.done.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (gen_ != seen && cur_); });
                if (stop_) return;
                seen = gen_;
                j = cur_;
            }
            work(*j);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::shared_ptr<Job> cur_;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Host-resident batch, pipelined over two stages: chunk c+1 is copied H2D while chunk c's
// kernel runs.  Pinned, compact batches are copied as one span per chunk (no CPU copy);
// otherwise packets are gathered into pinned staging first.  Trailers (write / zero) are
// applied to the caller's host buffer from the returned results.
constexpr size_t kChunkBytes = size_t(64) << 20;

struct HostJob {
    int mode;
    uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    uint32_t *out;
    uint8_t *ok;
    int trailer;
};

int finish_stage(icrc_engine *e, Stage &s, const HostJob &j) {
    if (!s.busy) return ICRC_OK;
    s.busy = false;
    HIP_TRY(hipEventSynchronize(s.done));
    for (uint32_t i = 0; i < s.cnt; i++) {
        const uint32_t k = s.i0 + i;
        uint8_t *t = j.base + j.off[k] + j.len[k] - 4;
        if (j.mode == icrc::kCompute) {
            const uint32_t c = s.h_res[i];
            if (j.out) j.out[k] = c;
            if (j.trailer) {
                t[0] = uint8_t(c);
                t[1] = uint8_t(c >> 8);
                t[2] = uint8_t(c >> 16);
                t[3] = uint8_t(c >> 24);
            }
        } else {
            j.ok[k] = reinterpret_cast<const uint8_t *>(s.h_res)[i];
            if (j.trailer) std::memset(t, 0, 4);
        }
    }
    (void)e;
    return ICRC_OK;
}

int message_batch(icrc_engine *e, int mode, uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                  uint32_t *out_icrc, uint8_t *ok, int trailer);

int host_batch(icrc_engine *e, int mode, uint8_t *base, const uint64_t *off, const uint32_t *len,
               uint32_t n, uint32_t *out_icrc, uint8_t *ok, int trailer) {
    if (!e) return ICRC_EINVAL;
    if (n && mode == icrc::kCompute && !out_icrc && !trailer) return ICRC_EINVAL;
    if (n && mode == icrc::kVerify && !ok) return ICRC_EINVAL;
    int vrc = validate_host(base, off, len, n);
    if (vrc) return vrc;
    if (n == 0) return ICRC_OK;
    const int mrc = message_batch(e, mode, base, off, len, n, out_icrc, ok, trailer);
    if (mrc != 1) return mrc;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    std::lock_guard<std::mutex> lk(e->mu);
    const HostJob job{mode, base, off, len, out_icrc, ok, trailer};
    const bool pinned = host_pinned(base);
    int rc = ICRC_OK;
    uint32_t i0 = 0;
    for (int c = 0; i0 < n && rc == ICRC_OK; ++c) {
        Stage &s = e->st[c & 1];
        if ((rc = finish_stage(e, s, job)) != ICRC_OK) break;
        // chunk [i0, i1): packed size <= kChunkBytes (at least one packet)
        uint32_t i1 = i0;
        size_t packed = 0;
        uint64_t smin = UINT64_MAX, smax = 0;
        while (i1 < n && (i1 == i0 || packed + len[i1] + 3 <= kChunkBytes)) {
            packed += (static_cast<size_t>(len[i1]) + 3) & ~size_t(3);
            smin = std::min<uint64_t>(smin, off[i1]);
            smax = std::max<uint64_t>(smax, off[i1] + len[i1]);
            i1++;
        }
        const uint32_t cnt = i1 - i0;
        const bool direct = pinned && (smax - smin) <= packed + packed / 4 + 4096;
        const size_t dev_bytes = direct ? static_cast<size_t>(smax - smin) : packed;
        if ((rc = stage_reserve(s, dev_bytes, cnt, !direct)) != ICRC_OK) break;
        std::memcpy(s.h_len, len + i0, cnt * sizeof(uint32_t));
        if (direct) {
            for (uint32_t i = 0; i < cnt; i++) s.h_off[i] = off[i0 + i] - smin;
            if (hipMemcpyAsync(s.d_buf, base + smin, dev_bytes, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
                rc = ICRC_EDEVICE;
                break;
            }
        } else {
            size_t pos = 0;
            for (uint32_t i = 0; i < cnt; i++) {
                s.h_off[i] = pos;
                pos += (static_cast<size_t>(len[i0 + i]) + 3) & ~size_t(3);
            }
            // the gather: packet ranges of ~1 MiB over the copy pool
            CopyPool &pool = CopyPool::get();
            const uint32_t per = static_cast<uint32_t>(std::max<size_t>(1, cnt / std::max<size_t>(1, pos >> 20)));
            const uint32_t ntasks = (cnt + per - 1) / per;
            pool.run(ntasks, [&](uint32_t t) {
                const uint32_t a = t * per, b = std::min(cnt, a + per);
                for (uint32_t i = a; i < b; i++) std::memcpy(s.h_buf + s.h_off[i], base + off[i0 + i], len[i0 + i]);
            });
            if (hipMemcpyAsync(s.d_buf, s.h_buf, pos, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
                rc = ICRC_EDEVICE;
                break;
            }
        }
        if (hipMemcpyAsync(s.d_off, s.h_off, cnt * 8, hipMemcpyHostToDevice, s.stream) != hipSuccess ||
            hipMemcpyAsync(s.d_len, s.h_len, cnt * 4, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
            rc = ICRC_EDEVICE;
            break;
        }
        BatchParams p{};
        p.base = s.d_buf;
        p.off = s.d_off;
        p.len = s.d_len;
        p.n = cnt;
        p.table = e->d_table;
        p.table_oct = e->d_table_oct;
        p.trailer = 0;  // trailers are applied to the caller's host copy in finish_stage
        if (mode == icrc::kCompute) p.out = s.d_res;
        else p.ok = reinterpret_cast<uint8_t *>(s.d_res);
        if ((rc = dispatch(e, mode, p, s.stream)) != ICRC_OK) break;
        const size_t res_bytes = mode == icrc::kCompute ? cnt * 4 : cnt;
        if (hipMemcpyAsync(s.h_res, s.d_res, res_bytes, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
            hipEventRecord(s.done, s.stream) != hipSuccess) {
            rc = ICRC_EDEVICE;
            break;
        }
        s.busy = true;
        s.i0 = i0;
        s.cnt = cnt;
        i0 = i1;
    }
    for (Stage &s : e->st) {
        const int r2 = finish_stage(e, s, job);
        if (rc == ICRC_OK) rc = r2;
    }
    return rc;
}

int device_batch(icrc_engine *e, int mode, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                 uint64_t stride, uint32_t ulen, uint32_t n, uint32_t *d_out, uint8_t *d_ok, int trailer,
                 uint32_t *d_nerr, void *stream) {
    if (!e || !d_base) return ICRC_EINVAL;
    if (mode == icrc::kVerify && !d_ok) return ICRC_EINVAL;
    if (n == 0) return ICRC_OK;
    if (!d_len && ulen < ICRC_MIN_PACKET) return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    BatchParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.ulen = ulen;
    p.n = n;
    p.out = d_out;
    p.ok = d_ok;
    p.nerr = d_nerr;
    p.table = e->d_table;
    p.table_oct = e->d_table_oct;
    p.trailer = trailer ? 1 : 0;
    return dispatch(e, mode, p, stream);
}

// ---- scalar drop-ins and one-message host batches -------------------------------------------
// Per-thread pinned, device-mapped staging: each calling thread copies its packets into a slot of
// its own (no lock around the copy); the slot outlives the call, one per (thread, engine), and
// grows to the largest call the thread has made.
// Every slot's pinned block is also listed in g_slots: icrc_shutdown frees them all (threads that
// never exit, the main thread's slot) while the runtime is alive, and a slot whose block shutdown
// already freed makes no HIP call from its thread-exit destructor.
std::mutex g_slot_mu;
std::set<void *> &g_slots = *new std::set<void *>();
void slot_block_free(void *h) {
    bool mine = false;
    {
        std::lock_guard<std::mutex> lk(g_slot_mu);
        mine = g_slots.erase(h) != 0;
    }
    if (mine) (void)hipHostFree(h);
}
struct StageSlot {
    const icrc_engine *engine = nullptr;
    uint8_t *h = nullptr;  // pinned host
    uint8_t *d = nullptr;  // device view
    size_t cap = 0;
    ~StageSlot() {
        if (h) slot_block_free(h);
    }
};
constexpr size_t kScalarSlotBytes = 65536 + 64;  // any packet the C-ABI accepts (len <= 65535)
// Host batches up to this size take the submitter (zero-copy, one launch, combinable across
// threads): one message of the emulator's (configs[0]: 64 x 4156 B) is far below it.  Larger
// batches take the staged, pipelined H2D path (host_batch).
constexpr uint32_t kMsgMaxPackets = 1024;
static_assert(kMsgMaxPackets <= Combiner::kCap, "a message must fit one lane's arrays");
constexpr size_t kMsgMaxBytes = size_t(8) << 20;
thread_local StageSlot t_slot;

int stage_slot(const icrc_engine *e, size_t bytes, uint8_t **h, uint8_t **d) {
    bytes = std::max(bytes, kScalarSlotBytes);
    if (t_slot.engine != e || !t_slot.h || t_slot.cap < bytes) {
        if (t_slot.h) slot_block_free(t_slot.h);
        t_slot.engine = nullptr;
        t_slot.h = t_slot.d = nullptr;
        t_slot.cap = 0;
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocMapped) != hipSuccess) return ICRC_ENOMEM;
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
            (void)hipHostFree(p);
            return ICRC_EDEVICE;
        }
        {
            std::lock_guard<std::mutex> lk(g_slot_mu);
            g_slots.insert(p);
        }
        t_slot.engine = e;
        t_slot.h = static_cast<uint8_t *>(p);
        t_slot.d = static_cast<uint8_t *>(dp);
        t_slot.cap = bytes;
    }
    *h = t_slot.h;
    *d = t_slot.d;
    return ICRC_OK;
}

void lane_release(Lane &l) {
    if (l.stream) {
        (void)hipStreamSynchronize(l.stream);
        (void)hipStreamDestroy(l.stream);
    }
    for (void *p : {static_cast<void *>(l.h_off), static_cast<void *>(l.h_len), static_cast<void *>(l.h_res)})
        if (p) (void)hipHostFree(p);
    l = Lane{};
}

int lane_init(Lane &l) {
    void *a = nullptr, *b = nullptr, *r = nullptr, *da = nullptr, *db = nullptr, *dr = nullptr;
    if (hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking) != hipSuccess) {
        l.stream = nullptr;
        return ICRC_EDEVICE;
    }
    if (hipHostMalloc(&a, Combiner::kCap * 8, hipHostMallocMapped) != hipSuccess) return ICRC_ENOMEM;
    l.h_off = static_cast<uint64_t *>(a);
    if (hipHostMalloc(&b, Combiner::kCap * 4, hipHostMallocMapped) != hipSuccess) return ICRC_ENOMEM;
    l.h_len = static_cast<uint32_t *>(b);
    if (hipHostMalloc(&r, Combiner::kCap * 4, hipHostMallocMapped) != hipSuccess) return ICRC_ENOMEM;
    l.h_res = static_cast<uint32_t *>(r);
    if (hipHostGetDevicePointer(&da, a, 0) != hipSuccess || hipHostGetDevicePointer(&db, b, 0) != hipSuccess ||
        hipHostGetDevicePointer(&dr, r, 0) != hipSuccess)
        return ICRC_EDEVICE;
    l.d_off = static_cast<uint64_t *>(da);
    l.d_len = static_cast<uint32_t *>(db);
    l.d_res = static_cast<uint32_t *>(dr);
    return ICRC_OK;
}

Combiner *combiner(icrc_engine *e, int *rc) {
    std::lock_guard<std::mutex> lk(e->comb_init_mu);
    if (e->comb) return e->comb.get();
    auto c = std::make_unique<Combiner>();
    c->cap = std::min<uint32_t>(Combiner::kCap, static_cast<uint32_t>(e->num_cu) * icrc::kWavesPerGroup);
    for (Lane &l : c->lanes) {
        if ((*rc = lane_init(l)) != ICRC_OK) {
            for (Lane &x : c->lanes) lane_release(x);  // a failed set-up leaves nothing behind; the next call retries
            return nullptr;
        }
    }
    *rc = ICRC_OK;
    e->comb = std::move(c);
    return e->comb.get();
}

void combiner_free(icrc_engine *e) {
    if (!e->comb) return;
    for (Lane &l : e->comb->lanes) lane_release(l);
    e->comb.reset();
}

// One compute launch over the taken calls on lane l (its leader only, outside the combiner lock).
void run_combined(icrc_engine *e, Lane &l, SubmitReq *const *reqs, uint32_t nreq) {
    uintptr_t lo = UINTPTR_MAX;
    for (uint32_t i = 0; i < nreq; i++) lo = std::min(lo, reinterpret_cast<uintptr_t>(reqs[i]->dbase));
    uint32_t k = 0;
    for (uint32_t i = 0; i < nreq; i++) {
        const uint64_t rel = reinterpret_cast<uintptr_t>(reqs[i]->dbase) - lo;
        for (uint32_t q = 0; q < reqs[i]->n; q++, k++) {
            l.h_off[k] = rel + reqs[i]->off[q];
            l.h_len[k] = reqs[i]->len[q];
        }
    }
    BatchParams p{};
    p.base = reinterpret_cast<uint8_t *>(lo);
    p.off = l.d_off;
    p.len = l.d_len;
    p.n = k;
    // A message of equal, evenly spaced packets (a WRITE's full-MTU segments, one scalar packet)
    // launches as a strided batch: the kernel computes each offset instead of fetching the
    // (offset, length) arrays from host memory first (one PCIe round trip less per call).
    const uint32_t L0 = l.h_len[0];
    const uint64_t st = k > 1 ? l.h_off[1] - l.h_off[0] : L0;
    bool uniform = k > 0 && l.h_off[1 % k] >= l.h_off[0] && st >= L0 && ((lo + l.h_off[0]) & 3u) == 0 &&
                   ((st | L0) & 3u) == 0;
    for (uint32_t i = 1; uniform && i < k; i++) uniform = l.h_len[i] == L0 && l.h_off[i] == l.h_off[0] + i * st;
    if (uniform) {
        p.base += l.h_off[0];
        p.off = nullptr;
        p.len = nullptr;
        p.stride = st;
        p.ulen = L0;
    }
    p.table = e->d_table;
    p.table_oct = e->d_table_oct;
    p.out = l.d_res;
    p.spread = 1;  // k <= cap <= #CUs x 16: one workgroup per packet up to #CUs, on the one-packet pipeline
    int rc = dispatch(e, icrc::kCompute, p, l.stream);
    if (rc == ICRC_OK && hipStreamSynchronize(l.stream) != hipSuccess) rc = ICRC_EDEVICE;
    k = 0;
    for (uint32_t i = 0; i < nreq; i++) {
        reqs[i]->rc = rc;
        std::memcpy(reqs[i]->res, l.h_res + k, reqs[i]->n * sizeof(uint32_t));
        k += reqs[i]->n;
    }
}

int submit(icrc_engine *e, Combiner *c, SubmitReq &req) {
    std::unique_lock<std::mutex> lk(c->mu);
    c->pending.push_back(&req);
    while (!req.done) {
        Lane *lane = nullptr;
        if (!req.taken)
            for (Lane &l : c->lanes)
                if (!l.busy) {
                    lane = &l;
                    break;
                }
        if (lane) {  // become this lane's leader: take queued calls up to cap packets, launch, hand out results
            lane->busy = true;
            uint32_t take = 0, pk = 0;
            while (take < c->pending.size() && (take == 0 || pk + c->pending[take]->n <= c->cap))
                pk += c->pending[take++]->n;
            std::vector<SubmitReq *> batch(c->pending.begin(), c->pending.begin() + take);
            c->pending.erase(c->pending.begin(), c->pending.begin() + take);
            for (SubmitReq *r : batch) r->taken = true;
            lk.unlock();
            run_combined(e, *lane, batch.data(), take);
            lk.lock();
            for (SubmitReq *r : batch) r->done = true;
            lane->busy = false;
            c->cv.notify_all();
        } else {
            c->cv.wait(lk);
        }
    }
    return req.rc;
}

// ---- the submission ring (icrc_ring.h): creation, the device side, shutdown -------------------------
int RingHip::launch(uint32_t epoch) {
    DeviceGuard g(device);
    if (!g.ok) return ICRC_ENODEV;
    rp.epoch = epoch;
    return icrc::launch_ring(rp, nslots, stream);
}

int RingHip::ended() {
    DeviceGuard g(device);
    const hipError_t q = hipStreamQuery(stream);
    if (q == hipSuccess) return 1;
    if (q == hipErrorNotReady) return 0;
    (void)hipGetLastError();
    return -1;
}

// Live rings, stopped at process exit: every wave ends (host memory only, no HIP call) before the
// runtime's own teardown, which registered its handlers before ours.
#ifdef ICRC_AB_BUILD
// ICRC_RING_TRACE (A/B library): per-slot job stamps from the ring kernel, summarised at exit
struct RingTrace {
    const uint64_t *rec;
    uint32_t nslots;
};
std::vector<RingTrace> g_traces;
void ring_trace_dump() {
    for (const RingTrace &t : g_traces) {
        std::vector<double> seen_dec, dec_res, res_done, gap;
        for (uint32_t s = 0; s < t.nslots; ++s) {
            const uint64_t *r = t.rec + static_cast<size_t>(s) * icrc::kRingTraceJobs * 4u;
            for (uint32_t j = 1; j < icrc::kRingTraceJobs; ++j) {  // job numbers start at 1
                const uint64_t *x = r + j * 4u;
                if (!x[3]) continue;
                seen_dec.push_back((x[1] - x[0]) * 0.01);
                dec_res.push_back((x[2] - x[1]) * 0.01);
                res_done.push_back((x[3] - x[2]) * 0.01);
                if (j > 1 && x[-1] && x[0] > x[-1] && x[0] - x[-1] < 100000u) gap.push_back((x[0] - x[-1]) * 0.01);
            }
        }
        auto med = [](std::vector<double> v) {
            if (v.empty()) return 0.0;
            std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
            return v[v.size() / 2];
        };
        std::fprintf(stderr,
                     "{\"ring_trace\": true, \"jobs\": %zu, \"seen_to_decoded_us\": %.2f, \"decoded_to_results_us\": "
                     "%.2f, \"results_to_done_us\": %.2f, \"done_to_next_seen_us\": %.2f}\n",
                     seen_dec.size(), med(seen_dec), med(dec_res), med(res_done), med(gap));
    }
}
#endif

// The last resort for a C caller that never calls icrc_shutdown: the rings' waves are stopped through
// host memory only (no HIP call).  Python's binding calls icrc_shutdown from its own atexit handler,
// before the interpreter and the HIP runtime finalise, and this then finds no ring.
void ring_atexit() {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    for (const RingEntry &r : g_rings) (void)r.ring->stop(1000000);
#ifdef ICRC_AB_BUILD
    ring_trace_dump();
#endif
}

int ring_free(icrc_engine *e) {
    std::unique_ptr<RingState> rs;
    {
        std::lock_guard<std::mutex> lk(e->ring_mu);
        rs = std::move(e->ring);
    }
    if (!rs) return ICRC_OK;
    if (rs->ring) {
        {
            std::lock_guard<std::mutex> lk(g_ring_mu);
            const icrc::HostRing *mine = rs->ring.get();
            g_rings.erase(std::remove_if(g_rings.begin(), g_rings.end(), [&](const RingEntry &x) { return x.ring == mine; }),
                          g_rings.end());
        }
        if (rs->ring->stop(1000000) != ICRC_OK) {
            // a wedged service kernel (the case in which the watchdog retired the ring): neither wait
            // for its stream nor free memory its waves may still touch.  The ring is leaked.
            std::fprintf(stderr, "icrc_amd: the submission ring's kernel did not stop within 1 s; its stream and "
                                 "memory are left in place\n");
            (void)rs.release();
            return ICRC_ETIMEDOUT;
        }
    }
    if (rs->dev.stream) {
        (void)hipStreamSynchronize(rs->dev.stream);
        (void)hipStreamDestroy(rs->dev.stream);
    }
    if (rs->d_mem) (void)hipFree(rs->d_mem);
    if (rs->host) (void)hipHostFree(rs->host);
    return ICRC_OK;
}

// The engine's ring, created on first use (nullptr, with *rc, when it cannot be: the caller falls
// back to kernel launches).
icrc::HostRing *ring_for(icrc_engine *e, int *rc) {
    std::lock_guard<std::mutex> lk(e->ring_mu);
    if (e->ring) return e->ring->ring ? e->ring->ring.get() : nullptr;
    auto rs = std::make_unique<RingState>();
    RingState *r = rs.get();
    e->ring = std::move(rs);  // kept even on failure: a failed set-up is not retried per call
    uint32_t nslots = icrc::kRingSlots, wgs = icrc::kRingWgPerSlot;
    // measurement knobs (scripts/msg_probe): the ring's shape
    if (const char *v = std::getenv("ICRC_RING_SLOTS")) nslots = static_cast<uint32_t>(std::max(1, std::min(16, std::atoi(v))));
    if (const char *v = std::getenv("ICRC_RING_WGS")) wgs = static_cast<uint32_t>(std::max(1, std::min(32, std::atoi(v))));
    uint32_t threads = icrc::kRingThreads;
    if (const char *v = std::getenv("ICRC_RING_THREADS")) {
        const int t = std::atoi(v);
        threads = (t == 256 || t == 512 || t == 1024) ? static_cast<uint32_t>(t) : threads;
    }
    wgs = std::min<uint32_t>(wgs, std::max<uint32_t>(1u, static_cast<uint32_t>(e->num_cu) / nslots));
    // one coherent, device-mapped block: slot lines | done words | exited words | per slot (off, len, res)
    const size_t words = static_cast<size_t>(nslots) * wgs;  // one done / exited word per workgroup
    const size_t o_done = nslots * sizeof(icrc::RingSlot), o_exit = o_done + words * 4u;
    const size_t o_arr = (o_exit + words * 4u + 255u) & ~size_t(255);
    const size_t per_slot = icrc::kRingMaxPackets * (8u + 4u + 4u);
    const size_t bytes = o_arr + nslots * per_slot;
    *rc = ICRC_ENOMEM;
    if (hipHostMalloc(&r->host, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        r->host = nullptr;
        return nullptr;
    }
    std::memset(r->host, 0, bytes);
    void *dv = nullptr;
    *rc = ICRC_EDEVICE;
    if (hipHostGetDevicePointer(&dv, r->host, 0) != hipSuccess) return nullptr;
    // device memory: the exit flag (its own 256-byte block), then one decision line per workgroup
    const size_t d_dec = 256;
    const size_t d_bytes = d_dec + words * sizeof(icrc::RingSlot);
    if (hipMalloc(&r->d_mem, d_bytes) != hipSuccess) {
        r->d_mem = nullptr;
        return nullptr;
    }
    if (hipMemset(r->d_mem, 0, d_bytes) != hipSuccess) return nullptr;
    std::vector<uint32_t> mask((static_cast<size_t>(e->num_cu) + 31u) / 32u, 0u);
    for (int cu = 0; cu < e->num_cu; ++cu) mask[cu / 32] |= 1u << (cu % 32);
    if (hipExtStreamCreateWithCUMask(&r->dev.stream, static_cast<uint32_t>(mask.size()), mask.data()) == hipSuccess) {
        r->dev.dedicated = true;
    } else {
        (void)hipGetLastError();
        if (hipStreamCreateWithFlags(&r->dev.stream, hipStreamNonBlocking) != hipSuccess) {
            r->dev.stream = nullptr;
            return nullptr;
        }
    }
    uint8_t *h = static_cast<uint8_t *>(r->host);
    const uint64_t d = reinterpret_cast<uint64_t>(dv);
    icrc::RingMemory mem;
    mem.slots = reinterpret_cast<icrc::RingSlot *>(h);
    mem.done = reinterpret_cast<uint32_t *>(h + o_done);
    mem.exited = reinterpret_cast<uint32_t *>(h + o_exit);
    mem.d_slots = d;
    for (uint32_t s = 0; s < nslots; ++s) {
        const size_t b = o_arr + s * per_slot;
        mem.off[s] = reinterpret_cast<uint64_t *>(h + b);
        mem.len[s] = reinterpret_cast<uint32_t *>(h + b + icrc::kRingMaxPackets * 8u);
        mem.res[s] = reinterpret_cast<uint32_t *>(h + b + icrc::kRingMaxPackets * 12u);
        mem.d_off[s] = d + b;
        mem.d_len[s] = d + b + icrc::kRingMaxPackets * 8u;
        mem.d_res[s] = d + b + icrc::kRingMaxPackets * 12u;
    }
    r->dev.device = e->device;
    r->dev.nslots = nslots;
    r->dev.rp.slots = reinterpret_cast<const icrc::RingSlot *>(d);
    r->dev.rp.done = reinterpret_cast<uint32_t *>(d + o_done);
    r->dev.rp.exited = reinterpret_cast<uint32_t *>(d + o_exit);
    r->dev.rp.exit_flag = reinterpret_cast<uint32_t *>(r->d_mem);
    r->dev.rp.decision = reinterpret_cast<icrc::RingSlot *>(r->d_mem + d_dec);
    r->dev.rp.table = e->d_table;
    r->dev.rp.wg_per_slot = wgs;
    r->dev.rp.threads = threads;
    r->dev.rp.idle_ticks = kRingIdleTicks;
    r->dev.rp.life_ticks = kRingLifeTicks;
    if (const char *v = std::getenv("ICRC_RING_LIFE_US"))  // measurement knob: 100 us .. 20 ms
        r->dev.rp.life_ticks = static_cast<uint32_t>(std::max(100, std::min(20000, std::atoi(v))) * 100);
#ifdef ICRC_AB_BUILD
    if (const char *v = std::getenv("ICRC_RING_AB")) r->dev.rp.ab = static_cast<uint32_t>(std::atoi(v));
    if (std::getenv("ICRC_RING_TRACE")) {  // never freed: read at exit
        void *tp = nullptr, *tdv = nullptr;
        const size_t tb = static_cast<size_t>(nslots) * icrc::kRingTraceJobs * 32u;
        if (hipHostMalloc(&tp, tb, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer(&tdv, tp, 0) == hipSuccess) {
            std::memset(tp, 0, tb);
            r->dev.rp.trace = static_cast<uint64_t *>(tdv);
            std::lock_guard<std::mutex> gl(g_ring_mu);
            g_traces.push_back({static_cast<const uint64_t *>(tp), nslots});
        }
    }
#endif
    uint64_t watchdog_us = kRingWatchdogUs;
    if (const char *v = std::getenv("ICRC_RING_WATCHDOG_US"))  // test knob: the watchdog's fallback path
        watchdog_us = static_cast<uint64_t>(std::max(1, std::min(2000000, std::atoi(v))));
    r->ring = std::make_unique<icrc::HostRing>(&r->dev, mem, nslots, wgs, watchdog_us);
    {
        static std::once_flag once;
        std::call_once(once, [] { std::atexit(ring_atexit); });
        std::lock_guard<std::mutex> gl(g_ring_mu);
        g_rings.push_back(RingEntry{e->device, r->ring.get()});
    }
    *rc = ICRC_OK;
    return r->ring.get();
}

// One host message (n packets at dbase, the device view of pinned host memory; off / len host
// arrays relative to dbase) -> n ICRCs into res: through the submission ring, or (host path
// ICRC_HOST_LAUNCH, or a ring that cannot run) one launch through the four-lane submitter.  A
// ring watchdog timeout retires the ring and the call runs as a launch (a GPU whose CUs
// are all held by other work would otherwise fail a valid call); a stopped ring fails the call.
int host_job(icrc_engine *e, const uint8_t *dbase, const uint64_t *off, const uint32_t *len, uint32_t n,
             uint32_t *res) {
    int rc = ICRC_OK;
    if (e->host_path.load(std::memory_order_relaxed) == ICRC_HOST_RING && n <= icrc::kRingMaxPackets) {
        icrc::HostRing *ring = ring_for(e, &rc);
        if (ring && !ring->retired()) {
            icrc::RingJob j;
            j.n = n;
            j.res = res;
            // equal, evenly spaced packets (a WRITE's full-MTU segments, one packet): strided
            const uint64_t st = n > 1 ? off[1] - off[0] : len[0];
            bool uniform = n == 1 || off[1] >= off[0];
            for (uint32_t i = 1; uniform && i < n; i++) uniform = len[i] == len[0] && off[i] == off[0] + i * st;
            if (uniform) {
                j.dbase = reinterpret_cast<uint64_t>(dbase) + off[0];
                j.stride = st;
                j.ulen = len[0];
            } else {
                j.dbase = reinterpret_cast<uint64_t>(dbase);
                j.off = off;
                j.len = len;
            }
            rc = ring->submit(j);
            if (rc == ICRC_OK) return rc;
            // a stopped ring (engine destruction, process exit): no launch either
            if (ring->stopped()) return ICRC_EDEVICE;
            // the watchdog (ICRC_ETIMEDOUT: counted in host_stats, the slot stays quarantined with its
            // own result array, the ring is retired) or a failed launch: this call runs as a launch
        } else if (ring && ring->stopped()) {
            return ICRC_EDEVICE;
        }
    }
    Combiner *c = combiner(e, &rc);
    if (!c) return rc;
    SubmitReq req{dbase, off, len, n, res};
    return submit(e, c, req);
}

int scalar_call(const uint8_t *pkt, size_t len, uint32_t *result) {
    icrc_engine *e = nullptr;
    int rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    uint8_t *h = nullptr, *d = nullptr;
    if ((rc = stage_slot(e, len, &h, &d)) != ICRC_OK) return rc;
    std::memcpy(h, pkt, len);
    const uint64_t off0 = 0;
    const uint32_t len32 = static_cast<uint32_t>(len);
    return host_job(e, d, &off0, &len32, 1, result);
}

// Device view of [base + smin, base + smax) when that whole span lies inside ONE pinned host
// allocation (hipHostMalloc / hipHostRegister), else nullptr (the caller stages the packets).
const uint8_t *pinned_device_view(uint8_t *base, uint64_t smin, uint64_t smax) {
    if (!host_pinned(base + smin)) return nullptr;
    void *d0 = nullptr;
    if (hipHostGetDevicePointer(&d0, base + smin, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    // the allocation holding the first byte must also hold the last one: both ends being pinned is
    // not enough (pageable memory may lie between two pinned allocations)
    hipDeviceptr_t abase = nullptr;
    size_t asize = 0;
    if (hipMemGetAddressRange(&abase, &asize, d0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(abase), p0 = reinterpret_cast<uintptr_t>(d0);
    if (p0 < a0 || p0 - a0 + (smax - smin) > asize) return nullptr;
    return static_cast<const uint8_t *>(d0);
}

// A host batch of at most kMsgMaxPackets / kMsgMaxBytes (one message): ICRCs through the
// submitter, zero-copy from a pinned caller buffer, else packed into this thread's mapped slot;
// then trailers written (compute) or compared and zeroed (verify) on the calling thread.
// Returns 1 when the batch is too large for this path (the caller takes host_batch).
int message_batch(icrc_engine *e, int mode, uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                  uint32_t *out_icrc, uint8_t *ok, int trailer) {
    if (n > kMsgMaxPackets) return 1;
    size_t packed = 0;
    uint64_t smin = UINT64_MAX, smax = 0;
    for (uint32_t i = 0; i < n; i++) {
        packed += (static_cast<size_t>(len[i]) + 3) & ~size_t(3);
        smin = std::min<uint64_t>(smin, off[i]);
        smax = std::max<uint64_t>(smax, off[i] + len[i]);
    }
    if (packed > kMsgMaxBytes) return 1;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    int rc = ICRC_OK;
    // the submitter's launches stay at most #CUs x 16 packets (one packet per wave)
    if (n > std::min<uint32_t>(Combiner::kCap, static_cast<uint32_t>(e->num_cu) * icrc::kWavesPerGroup)) return 1;
    thread_local std::vector<uint64_t> t_off;
    thread_local std::vector<uint32_t> t_res;
    t_off.resize(n);
    t_res.resize(n);
    // zero-copy only for a compact span of 4-byte aligned packets: a misaligned one would take the
    // kernel's byte-wise path over PCIe, slower than packing it into the staging slot
    bool aligned = true;
    for (uint32_t i = 0; aligned && i < n; i++)
        aligned = ((reinterpret_cast<uintptr_t>(base) + off[i]) & 3u) == 0 && (len[i] & 3u) == 0;
    const uint8_t *dbase =
        aligned && (smax - smin) <= packed + packed / 4 + 4096 ? pinned_device_view(base, smin, smax) : nullptr;
    if (dbase) {
        for (uint32_t i = 0; i < n; i++) t_off[i] = off[i] - smin;
    } else {
        uint8_t *h = nullptr, *d = nullptr;
        if ((rc = stage_slot(e, packed, &h, &d)) != ICRC_OK) return rc;
        size_t pos = 0;
        for (uint32_t i = 0; i < n; i++) {
            std::memcpy(h + pos, base + off[i], len[i]);
            t_off[i] = pos;
            pos += (static_cast<size_t>(len[i]) + 3) & ~size_t(3);
        }
        dbase = d;
    }
    if ((rc = host_job(e, dbase, t_off.data(), len, n, t_res.data())) != ICRC_OK) return rc;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *t = base + off[i] + len[i] - 4;
        const uint32_t crc = t_res[i];
        if (mode == icrc::kCompute) {
            if (out_icrc) out_icrc[i] = crc;
            if (trailer) {  // PacketWriter::write stores the ICRC LE (packet_processor.rs:260-263)
                t[0] = uint8_t(crc);
                t[1] = uint8_t(crc >> 8);
                t[2] = uint8_t(crc >> 16);
                t[3] = uint8_t(crc >> 24);
            }
        } else {  // is_icrc_valid (packet_processor.rs:341-353)
            const uint32_t stored = static_cast<uint32_t>(t[0]) | (static_cast<uint32_t>(t[1]) << 8) |
                                    (static_cast<uint32_t>(t[2]) << 16) | (static_cast<uint32_t>(t[3]) << 24);
            ok[i] = stored == crc ? ICRC_VERIFY_OK : ICRC_VERIFY_MISMATCH;
            if (trailer) std::memset(t, 0, 4);
        }
    }
    return ICRC_OK;
}

// Everything an engine holds on the device, in dependency order (no registry work: the callers,
// icrc_engine_destroy and icrc_shutdown, have already taken the engine out of the registries).  The
// HIP calls here run before the runtime's teardown: from the caller, or from icrc_shutdown.
int engine_teardown(icrc_engine *e) {
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != e->device) (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->side) (void)hipStreamSynchronize(e->side);
    const int rc = ring_free(e);
    for (Stage &s : e->st) stage_free(s);
    combiner_free(e);
    // a ring kernel that did not stop still reads the W = 64 table image: it is left with the ring
    if (rc == ICRC_OK && e->d_table) (void)hipFree(e->d_table);
    if (e->d_table_oct) (void)hipFree(e->d_table_oct);
    if (e->d_rx_flag) (void)hipFree(e->d_rx_flag);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->side) (void)hipStreamDestroy(e->side);
    if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
    if (e->join_ev) (void)hipEventDestroy(e->join_ev);
    if (prev >= 0 && prev != e->device) (void)hipSetDevice(prev);
    return rc;
}

}  // namespace

extern "C" {

const char *icrc_version(void) {
#ifdef ICRC_AB_BUILD
#define ICRC_BUILD_KIND " [A/B build: diagnostics]"
#else
#define ICRC_BUILD_KIND ""
#endif
    return "icrc_amd 0.4 gfx950: end-aligned column Horner (one packet per wave for long packets, eight per "
           "wave in 10-row frames for short ones), LDS byte tables replicated 32x from a 36 KiB compact image + "
           "per-lane nibble tables, prefetch rings, register-buffered results, verify by CRC-32 residue"
           ICRC_BUILD_KIND;
#undef ICRC_BUILD_KIND
}

uint32_t icrc_abi_version(void) { return ICRC_ABI_VERSION; }

int icrc_abi_check(uint32_t abi_version, size_t write_msg_bytes, size_t rx_desc_bytes, size_t ack_ctx_bytes,
                   size_t synth_desc_bytes) {
    return abi_version == ICRC_ABI_VERSION && write_msg_bytes == sizeof(icrc_write_msg) &&
                   rx_desc_bytes == sizeof(icrc_rx_desc) && ack_ctx_bytes == sizeof(icrc_ack_ctx) &&
                   synth_desc_bytes == sizeof(icrc_synth_desc)
               ? ICRC_OK
               : ICRC_EINVAL;
}

int icrc_engine_set_host_path(icrc_engine *e, int path) {
    if (!e || (path != ICRC_HOST_RING && path != ICRC_HOST_LAUNCH)) return ICRC_EINVAL;
    e->host_path.store(path, std::memory_order_relaxed);
    return ICRC_OK;
}

int icrc_engine_host_stats(icrc_engine *e, uint64_t out[4]) {
    if (!e || !out) return ICRC_EINVAL;
    out[0] = out[1] = out[2] = out[3] = 0;
    std::lock_guard<std::mutex> lk(e->ring_mu);
    if (e->ring && e->ring->ring) {
        const icrc::RingStats s = e->ring->ring->stats();
        out[0] = s.jobs;
        out[1] = s.launches;
        out[2] = s.relaunches;
        out[3] = s.timeouts;
    }
    return ICRC_OK;
}

int icrc_device_count(void) {
    if (shut_down()) return 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int icrc_engine_create(int device, icrc_engine **out) {
    if (!out) return ICRC_EINVAL;
    *out = nullptr;
    if (shut_down()) return ICRC_EDEVICE;
    int ndev = icrc_device_count();
    if (ndev <= 0) return ICRC_ENODEV;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= ndev) return ICRC_ENODEV;
    DeviceGuard g(device);
    if (!g.ok) return ICRC_ENODEV;
    auto *e = new (std::nothrow) icrc_engine();
    if (!e) return ICRC_ENOMEM;
    e->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete e;
        return ICRC_EDEVICE;
    }
    e->num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 1;
    // each device table buffer: the full LDS image, then its compact form (icrc_internal.h)
    constexpr size_t kBufBytes = icrc::kTableBufWords * 4u;
    std::vector<uint32_t> img(icrc::kTableBufWords), img_oct(icrc::kTableBufWords);
    icrc::build_table_image(img.data());
    icrc::append_compact_image(img.data());
    icrc::build_table_image_oct(img_oct.data());
    icrc::append_compact_image(img_oct.data());
    if (hipMalloc(&e->d_table, kBufBytes) != hipSuccess ||
        hipMemcpy(e->d_table, img.data(), kBufBytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&e->d_table_oct, kBufBytes) != hipSuccess ||
        hipMemcpy(e->d_table_oct, img_oct.data(), kBufBytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->join_ev, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&e->d_rx_flag, 256) != hipSuccess || hipMemset(e->d_rx_flag, 0, 256) != hipSuccess) {
        (void)engine_teardown(e);
        delete e;
        return ICRC_EDEVICE;
    }
    {
        std::lock_guard<std::recursive_mutex> lk(g_registry_mu);
        if (g_shutdown.load(std::memory_order_acquire)) {  // icrc_shutdown ran meanwhile
            (void)engine_teardown(e);
            delete e;
            return ICRC_EDEVICE;
        }
        g_engines.insert(e);
    }
    *out = e;
    return ICRC_OK;
}

int icrc_engine_destroy(icrc_engine *e) {
    if (!e) return ICRC_EINVAL;
    {
        std::lock_guard<std::recursive_mutex> lk(g_registry_mu);
        if (g_engines.erase(e) == 0) return ICRC_EINVAL;  // not live: destroyed, or gone with icrc_shutdown
        for (auto it = g_default.begin(); it != g_default.end(); ++it)
            if (it->second == e) {
                g_default.erase(it);
                break;
            }
    }
    const int rc = engine_teardown(e);
    delete e;
    return rc;
}

int icrc_shutdown(void) {
    std::vector<icrc_engine *> live;
    {
        std::lock_guard<std::recursive_mutex> lk(g_registry_mu);
        if (g_shutdown.exchange(true, std::memory_order_acq_rel)) return ICRC_OK;  // idempotent
        live.assign(g_engines.begin(), g_engines.end());
        g_engines.clear();
        g_default.clear();
    }
    int rc = ICRC_OK;
    for (icrc_engine *e : live) {
        const int r = engine_teardown(e);
        if (rc == ICRC_OK) rc = r;
        delete e;
        g_engines_torn_down.fetch_add(1, std::memory_order_relaxed);
    }
    std::vector<void *> slots;
    {
        std::lock_guard<std::mutex> lk(g_slot_mu);
        slots.assign(g_slots.begin(), g_slots.end());
        g_slots.clear();
    }
    for (void *h : slots) (void)hipHostFree(h);
    g_slots_freed_at_shutdown.fetch_add(slots.size(), std::memory_order_relaxed);
    return rc;
}

int icrc_engine_default(int device, icrc_engine **out) {
    if (!out) return ICRC_EINVAL;
    if (shut_down()) return ICRC_EDEVICE;
    if (device < 0) {
        if (icrc_device_count() <= 0) return ICRC_ENODEV;
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    std::lock_guard<std::recursive_mutex> lk(g_registry_mu);
    auto it = g_default.find(device);
    if (it != g_default.end()) {
        *out = it->second;
        return ICRC_OK;
    }
    icrc_engine *e = nullptr;
    int rc = icrc_engine_create(device, &e);
    if (rc) return rc;
    g_default[device] = e;
    *out = e;
    return ICRC_OK;
}

int icrc_engine_device_ordinal(const icrc_engine *e) { return e ? e->device : ICRC_EINVAL; }

int icrc_engine_set_kernel_variant(icrc_engine *e, int variant) {
    const bool hybrid = icrc::is_short_variant(variant - icrc::kHybridVariantBase) ||
                        icrc::is_short_variant(variant - icrc::kHybridCompactBase);
    const bool rx = variant == icrc::kRxVariantBase + 1 || variant == icrc::kRxVariantBase + 2;
    if (!e || (variant != -1 && !icrc::is_batch_variant(variant) && !hybrid && !rx)) return ICRC_EINVAL;
    e->variant = variant < 0 ? -1 : variant;
    return ICRC_OK;
}

void *icrc_engine_stream(const icrc_engine *e) { return e ? static_cast<void *>(e->stream) : nullptr; }

uint32_t icrc_compute(const uint8_t *pkt, size_t len, int *err) {
    int dummy;
    int *rc = err ? err : &dummy;
    *rc = ICRC_OK;
    if (!pkt || len < ICRC_MIN_PACKET || len > 0xFFFFu) {
        *rc = ICRC_EINVAL;
        return 0;
    }
    uint32_t out = 0;
    *rc = scalar_call(pkt, len, &out);
    return *rc == ICRC_OK ? out : 0;
}

int icrc_verify(uint8_t *pkt, size_t len, int zero_trailer, int *ok) {
    if (!pkt || !ok || len < ICRC_MIN_PACKET || len > 0xFFFFu) return ICRC_EINVAL;
    // The device computes the ICRC (the same launch as concurrent icrc_compute callers: the
    // submitter combines them) and the comparison with the trailer, which this thread holds
    // anyway, runs here (is_icrc_valid, packet_processor.rs:344-352).  A verify launch would
    // return one ok byte per packet through mapped host memory: sub-dword PCIe writes, measured
    // twice as slow from three threads.
    uint32_t crc = 0;
    const int rc = scalar_call(pkt, len, &crc);
    if (rc != ICRC_OK) return rc;
    const uint8_t *t = pkt + len - 4;
    const uint32_t stored = static_cast<uint32_t>(t[0]) | (static_cast<uint32_t>(t[1]) << 8) |
                            (static_cast<uint32_t>(t[2]) << 16) | (static_cast<uint32_t>(t[3]) << 24);
    *ok = (stored == crc);
    if (zero_trailer) std::memset(pkt + len - 4, 0, 4);  // is_icrc_valid, packet_processor.rs:350
    return ICRC_OK;
}

int icrc_compute_batch_ex(icrc_engine *e, uint8_t *base, const uint64_t *off, const uint32_t *len,
                          uint32_t n, uint32_t *out_icrc, int write_trailer) {
    return host_batch(e, icrc::kCompute, base, off, len, n, out_icrc, nullptr, write_trailer);
}

int icrc_verify_batch_ex(icrc_engine *e, uint8_t *base, const uint64_t *off, const uint32_t *len,
                         uint32_t n, uint8_t *ok, int zero_trailer) {
    return host_batch(e, icrc::kVerify, base, off, len, n, nullptr, ok, zero_trailer);
}

int icrc_compute_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                       uint32_t *out_icrc, int write_trailer) {
    int rc = validate_host(base, off, len, n);
    if (rc) return rc;
    icrc_engine *e = nullptr;
    rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    return icrc_compute_batch_ex(e, base, off, len, n, out_icrc, write_trailer);
}

int icrc_verify_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n, uint8_t *ok,
                      int zero_trailer) {
    int rc = validate_host(base, off, len, n);
    if (rc) return rc;
    icrc_engine *e = nullptr;
    rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    return icrc_verify_batch_ex(e, base, off, len, n, ok, zero_trailer);
}

int icrc_compute_batch_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                              uint32_t n, uint32_t *d_out, int write_trailer, uint32_t *d_nerr,
                              void *stream) {
    if (!d_off || !d_len) return ICRC_EINVAL;
    return device_batch(e, icrc::kCompute, d_base, d_off, d_len, 0, 0, n, d_out, nullptr, write_trailer,
                        d_nerr, stream);
}

int icrc_verify_batch_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                             uint32_t n, uint8_t *d_ok, int zero_trailer, uint32_t *d_nerr, void *stream) {
    if (!d_off || !d_len) return ICRC_EINVAL;
    return device_batch(e, icrc::kVerify, d_base, d_off, d_len, 0, 0, n, nullptr, d_ok, zero_trailer, d_nerr,
                        stream);
}

int icrc_compute_strided_device(icrc_engine *e, uint8_t *d_base, uint64_t stride, uint32_t len, uint32_t n,
                                uint32_t *d_out, int write_trailer, void *stream) {
    return device_batch(e, icrc::kCompute, d_base, nullptr, nullptr, stride, len, n, d_out, nullptr,
                        write_trailer, nullptr, stream);
}

int icrc_verify_strided_device(icrc_engine *e, uint8_t *d_base, uint64_t stride, uint32_t len, uint32_t n,
                               uint8_t *d_ok, int zero_trailer, void *stream) {
    return device_batch(e, icrc::kVerify, d_base, nullptr, nullptr, stride, len, n, nullptr, d_ok, zero_trailer,
                        nullptr, stream);
}

int icrc_synth_device(icrc_engine *e, uint8_t *d_base, const icrc_synth_desc *d_desc, const uint8_t *d_hdr,
                      uint32_t n, void *stream) {
    if (!e || !d_base || !d_desc || !d_hdr) return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    return icrc::launch_synth(d_base, d_desc, d_hdr, n, stream);
}

// ICRC_AB_RX_OCT (A/B library): 0 the two passes, 1 the one pass, 2..5 its cuts (launch_oct_rx).
static int rx_oct_knob() {
#ifdef ICRC_AB_BUILD
    const char *v = std::getenv("ICRC_AB_RX_OCT");
    return v ? std::atoi(v) : 1;
#else
    return 1;
#endif
}

int icrc_rx_parse_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                         uint64_t stride, uint32_t len, uint32_t n, icrc_rx_desc *d_desc, uint8_t *d_ok,
                         int zero_trailer, uint32_t *d_nerr, void *stream) {
    if (!e || !d_base || !d_desc) return ICRC_EINVAL;
    if (n == 0) return ICRC_OK;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    BatchParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.ulen = len;
    p.n = n;
    p.ok = d_ok;
    p.nerr = d_nerr;
    p.table = e->d_table;
    p.trailer = zero_trailer ? 1 : 0;
    p.rx = d_desc;
    const int rxv = e->variant >= icrc::kRxVariantBase ? e->variant - icrc::kRxVariantBase : 0;
    if (rxv != 0) {  // A/B: the fused single-pass kernel on any batch (301: a store per packet, 302: per block)
        p.variant = rxv;
        return icrc::launch_rx(p, grid_for(e, n), stream);
    }
    // Small batches (at most one packet per wave, e.g. a 16 MiB message): ONE pass, verify +
    // descriptors (icrc_rx_kernel, descriptors collected per 64-packet block and stored with the
    // results): 4096 x 4156 B in 12.1 us instead of 15.3, 256 x 316 B in 8.9 instead of 12.4
    // (scripts/probe_rx_small.py).  On large batches the same fused pass measured slower than the
    // two passes (786 K x 4156 B: 0.70 vs 0.59 ms, profiles/r02_rx_fused_ab.jsonl).
    if (e->variant < 0 && n <= static_cast<uint32_t>(e->num_cu) * icrc::kWavesPerGroup) {
        p.variant = 2;
        // (A/B, ICRC_AB_RX_SMALL_PPW: packets per wave of this grid, as the compute dispatch's small
        // batches; 2 measured 1 % slower here, 4 +46 %: profiles/r06/rx/rx_small_grid_ppw.jsonl)
        int ppw = 1;
#ifdef ICRC_AB_BUILD
        if (const char *v = std::getenv("ICRC_AB_RX_SMALL_PPW")) ppw = std::max(1, std::min(16, std::atoi(v)));
#endif
        const uint32_t per_wg = icrc::kWavesPerGroup * static_cast<uint32_t>(ppw);
        const int grid = ppw > 1 ? static_cast<int>(std::max<uint32_t>(1u, (n + per_wg - 1) / per_wg)) : grid_for(e, n);
        return icrc::launch_rx(p, grid, stream);
    }
    // Strided batches of short packets: ONE pass (icrc_oct_rx_kernel): the oct verify keeps each
    // packet's header words as loaded and stores the descriptors itself, so the header lines are not
    // read twice.  (A/B: ICRC_AB_RX_OCT=0 keeps the two passes.)
    if (e->variant < 0 && !d_off && !d_len && len >= ICRC_MIN_PACKET && len <= icrc::oct_max_len() && len % 4u == 0 &&
        stride % 4u == 0 && stride <= (1ull << 24) && reinterpret_cast<uintptr_t>(d_base) % 4u == 0 && rx_oct_knob() != 0) {
        p.table_oct = e->d_table_oct;
        return icrc::launch_oct_rx(p, grid_for(e, n), stream, rx_oct_knob());
    }
    // Ragged batches with whole 64-packet blocks per wave: the same one-pass receive on the packets
    // the oct kernel takes and the long-packet verify + descriptors on the rest in one launch, then
    // (only when the ring's tail loop took any) descriptors for those from their header words
    // (icrc_rx_sweep_kernel).  p.ok carries the tail loop's results to that last step: a
    // stream-ordered scratch array when the caller passes none.  (A/B: ICRC_AB_RX_OCT=0 keeps the
    // two passes.)
    {
        const int grid = grid_for(e, n);
        if (e->variant < 0 && (d_off || d_len) && rx_oct_knob() != 0 &&
            static_cast<uint64_t>(n) > 32ull * icrc::kWavesPerGroup * static_cast<uint64_t>(grid)) {
            p.table_oct = e->d_table_oct;
            p.split_len = icrc::split_len_for(icrc::kDefaultRaggedVariant);
            p.ab_long_walk = static_cast<uint32_t>(dispatch_knobs().long_walk);
            uint32_t gen = e->rx_gen.fetch_add(1u, std::memory_order_relaxed) + 1u;
            p.rx_flag = e->d_rx_flag;
            p.rx_gen = gen ? gen : 1u;  // (after a wrap the flag stays high: every call sweeps, still exact)
            uint8_t *scratch = nullptr;
            hipStream_t s = static_cast<hipStream_t>(stream);
            if (!d_ok) HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&scratch), n, s));
            p.ok = d_ok ? d_ok : scratch;
            int rc = icrc::launch_hybrid_rx(p, grid, e->num_cu, stream);
            if (scratch && hipFreeAsync(scratch, s) != hipSuccess && rc == ICRC_OK) rc = ICRC_EDEVICE;
            return rc;
        }
    }
    // Otherwise two passes (icrc_kernels.hip, icrc_rx_desc_kernel): the verify dispatch writes the
    // ok bytes (into d_ok, or a stream-ordered scratch array when the caller passes none), then the
    // descriptors are built from the header words and those bytes.
    p.table_oct = e->d_table_oct;
    uint8_t *scratch = nullptr;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!d_ok) HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&scratch), n, s));
    p.ok = d_ok ? d_ok : scratch;
    int rc = dispatch(e, icrc::kVerify, p, stream);
    p.split_len = 0;
    if (rc == ICRC_OK) rc = icrc::launch_rx_desc(p, e->num_cu, stream);
    if (scratch && hipFreeAsync(scratch, s) != hipSuccess && rc == ICRC_OK) rc = ICRC_EDEVICE;
    return rc;
}

int icrc_ack_from_rx_device(icrc_engine *e, const icrc_rx_desc *d_desc, const icrc_ack_ctx *d_ctx, uint32_t n,
                            uint8_t *d_out, uint32_t out_stride, uint32_t *d_out_len, uint32_t flags, void *stream) {
    if (n == 0) return ICRC_OK;
    const uint32_t need = (flags & ICRC_ACK_UDP_PAYLOAD_ONLY) ? 20u : 48u;
    if (!e || !d_desc || !d_ctx || !d_out || out_stride < need || out_stride % 4 != 0 ||
        reinterpret_cast<uintptr_t>(d_out) % 4 != 0 || (flags & ~ICRC_ACK_UDP_PAYLOAD_ONLY) != 0)
        return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    return icrc::launch_ack(d_desc, d_ctx, n, d_out, out_stride, d_out_len, flags, e->num_cu, stream);
}

int icrc_ipv4_checksum_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, uint64_t stride, uint32_t n,
                              uint16_t *d_csum, int fill, void *stream) {
    if (!e || !d_base) return ICRC_EINVAL;
    if (n == 0) return ICRC_OK;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    return icrc::launch_ipv4_checksum(d_base, d_off, stride, n, d_csum, fill ? 1 : 0, stream);
}

uint32_t icrc_write_segment_count(uint64_t local_va, uint32_t total_len, uint32_t pmtu) {
    if (pmtu == 0) return 0;
    const uint32_t first = icrc::write_first_segment(local_va, total_len, pmtu);
    const uint32_t rest = total_len - first;
    return 1u + rest / pmtu + (rest % pmtu ? 1u : 0u);
}

uint32_t icrc_write_packet_len(uint64_t local_va, uint32_t total_len, uint32_t pmtu, uint32_t s) {
    const uint32_t n = icrc_write_segment_count(local_va, total_len, pmtu);
    if (s >= n) return 0;
    const uint32_t first = icrc::write_first_segment(local_va, total_len, pmtu);
    uint32_t len = first;
    if (s > 0) {
        const uint32_t start = first + (s - 1) * pmtu;
        len = std::min(pmtu, total_len - start);
    }
    return 56u + len + ((4u - (len & 3u)) & 3u) + 4u;
}

int icrc_write_packetize_device(icrc_engine *e, const uint8_t *d_src, uint64_t src_bytes,
                                const icrc_write_msg *d_msgs, uint32_t nmsgs, uint32_t npackets,
                                uint8_t *d_wire, uint64_t wire_bytes, uint32_t *d_pkt_len, uint32_t *d_icrc,
                                void *stream) {
    if (npackets == 0) return ICRC_OK;
    if (!e || !d_msgs || nmsgs == 0 || !d_wire || (!d_src && src_bytes != 0)) return ICRC_EINVAL;
    if (reinterpret_cast<uintptr_t>(d_msgs) % alignof(icrc_write_msg) != 0) return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    icrc::PacketizeParams p;
    p.src = d_src;
    p.src_bytes = d_src ? src_bytes : 0;
    p.msgs = d_msgs;
    p.nmsgs = nmsgs;
    p.npackets = npackets;
    p.wire = d_wire;
    p.wire_bytes = wire_bytes;
    p.pkt_len = d_pkt_len;
    p.icrc = d_icrc;
    p.table = e->d_table;
    return icrc::launch_packetize(p, grid_for(e, npackets), stream);
}

// Host-only helper for tests: the LDS table image (no GPU needed).
int icrc_table_image(uint32_t *out_words, uint32_t nwords) {
    if (!out_words || nwords < icrc::kLdsWords) return ICRC_EINVAL;
    icrc::build_table_image(out_words);
    if (nwords >= icrc::kTableBufWords) icrc::append_compact_image(out_words);  // the device buffer
    return ICRC_OK;
}

int icrc_table_image_oct(uint32_t *out_words, uint32_t nwords) {
    if (!out_words || nwords < icrc::kLdsWords) return ICRC_EINVAL;
    icrc::build_table_image_oct(out_words);
    if (nwords >= icrc::kTableBufWords) icrc::append_compact_image(out_words);  // the device buffer
    return ICRC_OK;
}

// Removed in ABI 5 (the quad kernels were retired in round 5); kept exported for one release so that
// an existing dynamic link still resolves.  Always ICRC_EINVAL.
int icrc_table_image_quad(uint32_t *out_words, uint32_t nwords) {
    (void)out_words;
    (void)nwords;
    return ICRC_EINVAL;
}

}  // extern "C"

// Test hook (not in include/icrc.h): the teardown's record.  out[0] 1 once icrc_shutdown has run,
// [1] engines it destroyed, [2] staging slots it freed, [3] entry points refused afterwards (each of
// them returned before any HIP call).
extern "C" int icrc_teardown_stats(uint64_t out[4]) {
    if (!out) return ICRC_EINVAL;
    out[0] = g_shutdown.load(std::memory_order_acquire) ? 1u : 0u;
    out[1] = g_engines_torn_down.load(std::memory_order_relaxed);
    out[2] = g_slots_freed_at_shutdown.load(std::memory_order_relaxed);
    out[3] = g_refused_after_shutdown.load(std::memory_order_relaxed);
    return ICRC_OK;
}

// Test hook (not in include/icrc.h): `threads` callers each run `jobs` copy-pool jobs of 1..300
// tasks at once; every task of every job must run exactly once and each job must return only
// after all of its tasks (the per-job counters of CopyPool).  0 = as specified.
extern "C" int icrc_copy_pool_selftest(int threads, int jobs) {
    if (threads < 1 || jobs < 1) return -1;
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int k = 0; k < threads; ++k)
        th.emplace_back([&, k] {
            uint32_t x = 0x9E3779B9u * static_cast<uint32_t>(k + 1);
            for (int j = 0; j < jobs; ++j) {
                x ^= x << 13;
                x ^= x >> 17;
                x ^= x << 5;
                const uint32_t n = 1u + x % 300u;
                std::vector<std::atomic<uint32_t>> hits(n);
                for (auto &h : hits) h.store(0);
                CopyPool::get().run(n, [&](uint32_t t) {
                    for (volatile int spin = 0; spin < static_cast<int>(t % 7u) * 50; spin = spin + 1) {
                    }
                    hits[t].fetch_add(1);
                });
                for (auto &h : hits)
                    if (h.load() != 1u) bad.fetch_add(1);
            }
        });
    for (auto &t : th) t.join();
    return bad.load() == 0 ? 0 : 1;
}
