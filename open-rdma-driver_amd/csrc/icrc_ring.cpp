// icrc_ring.cpp — host side of the host-message submission ring (icrc_ring.h), and its CPU self-test.
//
// One call = one job in one slot: the caller copies the (offset, length) arrays of a ragged message
// into the slot's arrays, writes the slot line's fields, then its cmd word (release), and waits until
// every workgroup serving the slot has stored that cmd in its done word.  No device call sits on that
// path unless the service kernel has to be (re)started: the host reads the exited word of the launch's
// first workgroup (all end together, through the kernel's exit flag) to know whether it must launch.
#include "icrc_ring.h"

#include <immintrin.h>

#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

namespace icrc {

uint64_t ring_now_us() {
    return static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count());
}

HostRing::HostRing(RingDevice *dev, const RingMemory &mem, uint32_t nslots, uint32_t wg_per_slot, uint64_t watchdog_us)
    : dev_(dev),
      mem_(mem),
      nslots_(nslots),
      wg_per_slot_(wg_per_slot),
      wps_(wg_per_slot),
      watchdog_us_(watchdog_us),
      free_mask_(nslots >= 32u ? ~0u : (1u << nslots) - 1u) {}

RingStats HostRing::stats() const {
    std::lock_guard<std::mutex> lk(stats_mu_);
    return stats_;
}

int HostRing::acquire_slot(uint32_t *slot) {
    std::unique_lock<std::mutex> lk(slot_mu_);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(watchdog_us_);
    while (free_mask_ == 0u) {
        if (retired()) return ICRC_EDEVICE;
        if (slot_cv_.wait_until(lk, deadline) == std::cv_status::timeout && free_mask_ == 0u) return ICRC_ETIMEDOUT;
    }
    const uint32_t s = static_cast<uint32_t>(__builtin_ctz(free_mask_));
    free_mask_ &= ~(1u << s);
    *slot = s;
    return ICRC_OK;
}

void HostRing::release_slot(uint32_t slot) {
    {
        std::lock_guard<std::mutex> lk(slot_mu_);
        free_mask_ |= 1u << slot;
    }
    slot_cv_.notify_one();
}

bool HostRing::launch_ended() const {
    // workgroup 0 of slot 0 ends only when every workgroup of the launch ends (stop bit, exit flag)
    return __atomic_load_n(&mem_.exited[0], __ATOMIC_ACQUIRE) == epoch_;
}

int HostRing::ensure_running(bool ask_device) {
    std::lock_guard<std::mutex> lk(launch_mu_);
    bool need = !launched_ || launch_ended();
    if (!need && ask_device) {  // a launch that never ran its first workgroup (or ended abnormally)
        const int e = dev_->ended();
        if (e < 0) return ICRC_EDEVICE;
        need = e == 1;
    }
    if (!need) return ICRC_OK;
    const uint32_t next = epoch_ + 1u == 0u ? 1u : epoch_ + 1u;
    const int rc = dev_->launch(next);
    if (rc != ICRC_OK) return rc;
    epoch_ = next;
    std::lock_guard<std::mutex> sk(stats_mu_);
    if (launched_) stats_.relaunches++;
    stats_.launches++;
    launched_ = true;
    return ICRC_OK;
}

bool HostRing::job_done(uint32_t slot, uint32_t cmd) const {
    const uint32_t *d = mem_.done + static_cast<size_t>(slot) * wps_;
    for (uint32_t w = 0; w < wps_; ++w)
        if (__atomic_load_n(d + w, __ATOMIC_ACQUIRE) != cmd) return false;
    return true;
}

int HostRing::submit(const RingJob &j) {
    if (j.n == 0 || j.n > kRingMaxPackets || !j.res || (j.ulen == 0 && (!j.off || !j.len))) return ICRC_EINVAL;
    if (retired()) return ICRC_EDEVICE;
    uint32_t s = 0;
    int rc = acquire_slot(&s);
    if (rc != ICRC_OK) return rc;
    RingSlot *S = mem_.slots + s;
    if (j.ulen == 0) {
        std::memcpy(mem_.off[s], j.off, j.n * sizeof(uint64_t));
        std::memcpy(mem_.len[s], j.len, j.n * sizeof(uint32_t));
    }
    uint32_t cmd = (seq_[s] + 1u) & ~kRingStop;
    if (cmd == 0u) cmd = 1u;
    seq_[s] = cmd;
    RingSlot line;  // the new line: fields, hash (over cmd too), then in memory: fields, hash, cmd
    std::memset(&line, 0, sizeof line);
    line.cmd = cmd;
    line.n = j.n;
    line.ulen = j.ulen;
    line.base = j.dbase;
    line.stride = j.stride;
    line.off = mem_.d_off[s];
    line.len = mem_.d_len[s];
    line.out = mem_.d_res[s];
    line.reserved = 0u;
    line.hash = ring_line_hash(reinterpret_cast<const uint32_t *>(&line));
    uint32_t *w = reinterpret_cast<uint32_t *>(S);
    const uint32_t *nw = reinterpret_cast<const uint32_t *>(&line);
    for (int k = 2; k < 16; ++k) __atomic_store_n(w + k, nw[k], __ATOMIC_RELAXED);
    const uint32_t act = activity_.fetch_add(1u, std::memory_order_relaxed) + 1u;
    for (uint32_t k = 0; k < nslots_; ++k) __atomic_store_n(&mem_.slots[k].activity, act, __ATOMIC_RELAXED);
    __atomic_store_n(&S->cmd, cmd, __ATOMIC_RELEASE);  // publishes the fields above (x86: ordered stores)
    if ((rc = ensure_running(false)) != ICRC_OK) {
        retired_.store(true, std::memory_order_release);
        release_slot(s);  // nothing was launched for this job
        return rc;
    }
    const uint64_t t0 = ring_now_us();
    uint64_t next_check = t0 + 10u, next_query = t0 + 500u;
    for (uint32_t spin = 1;; ++spin) {
        if (job_done(s, cmd)) break;
        _mm_pause();
        if ((spin & 31u) != 0u) continue;
        const uint64_t now = ring_now_us();
        if (now - t0 > watchdog_us_ || retired()) {  // the host watchdog: fail the call, retire the ring
            retired_.store(true, std::memory_order_release);
            std::lock_guard<std::mutex> sk(stats_mu_);
            stats_.timeouts++;
            return now - t0 > watchdog_us_ ? ICRC_ETIMEDOUT : ICRC_EDEVICE;  // the slot stays taken
        }
        if (now >= next_check) {  // the launch ended under this job (an idle or lifetime exit racing it)
            next_check = now + 10u;
            const bool query = now >= next_query;  // and, rarely, ask the device (a launch that never ran)
            if (query) next_query = now + 500u;
            if ((rc = ensure_running(query)) != ICRC_OK) {
                retired_.store(true, std::memory_order_release);
                return rc;
            }
        }
    }
    std::memcpy(j.res, mem_.res[s], j.n * sizeof(uint32_t));
    release_slot(s);
    std::lock_guard<std::mutex> sk(stats_mu_);
    stats_.jobs++;
    return ICRC_OK;
}

int HostRing::stop(uint64_t wait_us) {
    stopped_.store(true, std::memory_order_release);
    retired_.store(true, std::memory_order_release);
    slot_cv_.notify_all();
    std::lock_guard<std::mutex> lk(launch_mu_);
    for (uint32_t k = 0; k < nslots_; ++k) __atomic_or_fetch(&mem_.slots[k].cmd, kRingStop, __ATOMIC_RELEASE);
    if (!launched_) return ICRC_OK;
    const uint64_t t0 = ring_now_us();
    const size_t nw = static_cast<size_t>(nslots_) * wps_;
    for (;;) {
        bool all = true;
        for (size_t w = 0; all && w < nw; ++w) all = __atomic_load_n(&mem_.exited[w], __ATOMIC_ACQUIRE) == epoch_;
        if (all) {
            launched_ = false;
            return ICRC_OK;
        }
        if (ring_now_us() - t0 > wait_us) return ICRC_ETIMEDOUT;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// ---- CPU self-test: the protocol against a simulated service kernel -------------------------------
namespace {

uint32_t sim_icrc(uint32_t i, uint32_t cmd, uint64_t dbase) {  // a stand-in result (not an ICRC)
    return static_cast<uint32_t>((i + 1u) * 2654435761u) ^ cmd ^ static_cast<uint32_t>(dbase >> 4);
}

// Emulates icrc_ring_kernel's workgroups on a host thread: per workgroup, last = its done word at
// launch; a new cmd -> its contiguous share of the packets -> results -> done word; the stop bit ends
// the launch.  Misbehaviours by scenario:
//   1 never completes a job (the watchdog must fail the call);
//   2 the launch ends (every workgroup stores exited) in the middle of every 5th job, after half of
//     the workgroups finished their share: the host must relaunch and the new launch finish the job;
//   3 launch() fails (the call must fail with that error and retire the ring);
//   4 every launch ends after one job (an idle exit before each next call).
struct SimDevice final : RingDevice {
    RingMemory mem;
    uint32_t nslots, wps, scenario;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t pending_epoch = 0;  // a launch to start
    bool running = false, quit = false;
    uint32_t jobs_seen = 0;
    std::thread th;

    SimDevice(const RingMemory &m, uint32_t ns, uint32_t w, uint32_t sc) : mem(m), nslots(ns), wps(w), scenario(sc) {
        th = std::thread([this] { loop(); });
    }
    ~SimDevice() override {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv.notify_all();
        th.join();
    }
    int launch(uint32_t epoch) override {
        if (scenario == 3) return ICRC_EDEVICE;
        std::lock_guard<std::mutex> lk(mu);
        pending_epoch = epoch;
        running = true;
        cv.notify_all();
        return ICRC_OK;
    }
    int ended() override {
        std::lock_guard<std::mutex> lk(mu);
        return running ? 0 : 1;
    }
    void end_launch(uint32_t epoch) {
        for (size_t w = 0; w < static_cast<size_t>(nslots) * wps; ++w) __atomic_store_n(&mem.exited[w], epoch, __ATOMIC_RELEASE);
        std::lock_guard<std::mutex> lk(mu);
        if (pending_epoch == 0) running = false;  // a launch requested meanwhile is still to run
    }
    void loop() {
        for (;;) {
            uint32_t epoch;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return quit || pending_epoch != 0; });
                if (quit) return;
                epoch = pending_epoch;
                pending_epoch = 0;
            }
            std::vector<uint32_t> last(static_cast<size_t>(nslots) * wps);
            for (size_t w = 0; w < last.size(); ++w) last[w] = __atomic_load_n(&mem.done[w], __ATOMIC_ACQUIRE);
            bool end = false;
            while (!end) {
                {
                    std::lock_guard<std::mutex> lk(mu);
                    if (quit) return;
                }
                bool any = false;
                for (uint32_t s = 0; s < nslots && !end; ++s) {
                    const uint32_t cmd = __atomic_load_n(&mem.slots[s].cmd, __ATOMIC_ACQUIRE);
                    if (cmd & kRingStop) {
                        end = true;
                        break;
                    }
                    if (cmd == last[static_cast<size_t>(s) * wps] && cmd == last[static_cast<size_t>(s) * wps + wps - 1]) continue;
                    any = true;
                    const RingSlot &S = mem.slots[s];
                    uint32_t line[16];  // what the kernel checks before it takes the fields
                    for (int k = 0; k < 16; ++k) line[k] = __atomic_load_n(reinterpret_cast<const uint32_t *>(&S) + k, __ATOMIC_ACQUIRE);
                    if (line[0] != cmd || ring_line_hash(line) != line[15]) continue;  // torn: read again
                    if (scenario == 1) continue;  // never completes
                    const uint32_t job = ++jobs_seen;
                    const uint32_t chunk = (S.n + wps - 1u) / wps;
                    for (uint32_t w = 0; w < wps; ++w) {
                        if (last[static_cast<size_t>(s) * wps + w] == cmd) continue;
                        if (scenario == 2 && job % 5u == 0u && w == wps / 2u) {  // the launch ends mid-job
                            end = true;
                            break;
                        }
                        const uint32_t lo = w * chunk < S.n ? w * chunk : S.n;
                        const uint32_t hi = lo + chunk < S.n ? lo + chunk : S.n;
                        for (uint32_t i = lo; i < hi; ++i) mem.res[s][i] = sim_icrc(i, cmd, S.base);
                        __atomic_store_n(&mem.done[static_cast<size_t>(s) * wps + w], cmd, __ATOMIC_RELEASE);
                        last[static_cast<size_t>(s) * wps + w] = cmd;
                    }
                    if (scenario == 4) end = true;
                }
                if (!any) std::this_thread::yield();
            }
            end_launch(epoch);
        }
    }
};

}  // namespace

}  // namespace icrc

// Test hook (not part of include/icrc.h): runs the ring protocol against the simulated device.
// Returns 0 when the scenario behaves as specified, else a positive failure code.
extern "C" int icrc_ring_selftest(int scenario, int threads, int jobs_per_thread) {
    using namespace icrc;
    constexpr uint32_t ns = 4, wgs = 8, wps = wgs;
    std::vector<RingSlot> slots(ns);
    std::vector<uint32_t> done(ns * wps, 0u), exited(ns * wps, 0u);
    std::vector<std::vector<uint64_t>> off(ns, std::vector<uint64_t>(kRingMaxPackets));
    std::vector<std::vector<uint32_t>> len(ns, std::vector<uint32_t>(kRingMaxPackets)), res(ns, std::vector<uint32_t>(kRingMaxPackets));
    std::memset(slots.data(), 0, sizeof(RingSlot) * ns);
    RingMemory mem;
    mem.slots = slots.data();
    mem.done = done.data();
    mem.exited = exited.data();
    for (uint32_t s = 0; s < ns; ++s) {
        mem.off[s] = off[s].data();
        mem.len[s] = len[s].data();
        mem.res[s] = res[s].data();
    }
    SimDevice dev(mem, ns, wps, static_cast<uint32_t>(scenario));
    HostRing ring(&dev, mem, ns, wgs, scenario == 1 ? 200000u : 5000000u);
    std::atomic<int> bad{0}, timeouts{0}, devfail{0};
    auto worker = [&](int t) {
        std::vector<uint32_t> out(kRingMaxPackets);
        std::vector<uint64_t> o(kRingMaxPackets);
        std::vector<uint32_t> l(kRingMaxPackets, 316u);
        for (int k = 0; k < jobs_per_thread; ++k) {
            RingJob j;
            j.n = 1u + static_cast<uint32_t>((t * 131 + k * 17) % 200);
            j.dbase = 0x100000ull * static_cast<uint64_t>(t + 1) + 0x1000ull * static_cast<uint64_t>(k);
            if (k & 1) {
                j.ulen = 316;
                j.stride = 316;
            } else {
                for (uint32_t i = 0; i < j.n; ++i) o[i] = 320ull * i;
                j.off = o.data();
                j.len = l.data();
            }
            j.res = out.data();
            const int rc = ring.submit(j);
            if (rc == ICRC_ETIMEDOUT) {
                timeouts++;
                return;
            }
            if (rc != ICRC_OK) {
                devfail++;
                return;
            }
            // the job's cmd is unknown here: recompute from the slot's published results' pattern
            for (uint32_t i = 0; i < j.n; ++i) {
                const uint32_t x = out[i] ^ static_cast<uint32_t>((i + 1u) * 2654435761u) ^ static_cast<uint32_t>(j.dbase >> 4);
                const uint32_t x0 = out[0] ^ 2654435761u ^ static_cast<uint32_t>(j.dbase >> 4);
                if (x != x0 || x == 0u) bad++;  // every result carries the same (nonzero) cmd
            }
        }
    };
    std::vector<std::thread> ths;
    for (int t = 0; t < threads; ++t) ths.emplace_back(worker, t);
    for (auto &th : ths) th.join();
    const RingStats st = ring.stats();
    const int stop_rc = ring.stop(1000000u);
    switch (scenario) {
    case 0:  // normal: every job right, one launch
        if (bad || timeouts || devfail) return 1;
        if (st.jobs != static_cast<uint64_t>(threads) * jobs_per_thread || st.launches != 1u) return 2;
        break;
    case 1:  // the watchdog fails the call with ICRC_ETIMEDOUT and retires the ring
        if (timeouts == 0 || !ring.retired()) return 3;
        break;
    case 2:  // launches ending mid-job: relaunched, every job right
        if (bad || timeouts || devfail) return 4;
        if (st.jobs != static_cast<uint64_t>(threads) * jobs_per_thread || st.relaunches == 0u) return 5;
        break;
    case 3:  // the launch fails: the calls fail with ICRC_EDEVICE, the ring is retired
        if (devfail == 0 || timeouts || !ring.retired()) return 6;
        break;
    case 4:  // an idle exit before every call: relaunched each time, every job right
        if (bad || timeouts || devfail) return 7;
        if (st.relaunches + 1u < st.jobs / 2u) return 8;
        break;
    default:
        return 99;
    }
    return scenario == 1 ? 0 : (stop_rc == ICRC_OK ? 0 : 9);
}
