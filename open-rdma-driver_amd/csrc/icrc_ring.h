// icrc_ring.h — host side of the host-message submission ring (layout and device kernel:
// icrc_internal.h RingSlot / RingParams, icrc_kernels.hip icrc_ring_kernel).
//
// The protocol is kept free of HIP calls: the device side is reached through RingDevice (launch an
// instance of the service kernel, ask whether the last one has ended), so the CPU suite drives the
// same code with a simulated device (icrc_ring_selftest, icrc_ring.cpp), watchdog and relaunch paths
// included.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>

#include "icrc_internal.h"

namespace icrc {

// Host addresses of the ring's memory (coherent, device-visible) and their device views.
struct RingMemory {
    RingSlot *slots = nullptr;      // [nslots] lines
    uint32_t *done = nullptr;       // [nslots][workgroups per slot]
    uint32_t *exited = nullptr;     // [nslots][workgroups per slot]
    uint64_t *off[kRingMaxSlots] = {};  // per slot: kRingMaxPackets offsets, lengths, results
    uint32_t *len[kRingMaxSlots] = {};
    uint32_t *res[kRingMaxSlots] = {};
    uint64_t d_slots = 0, d_off[kRingMaxSlots] = {}, d_len[kRingMaxSlots] = {}, d_res[kRingMaxSlots] = {};
};

// What the protocol needs from the device.
struct RingDevice {
    virtual int launch(uint32_t epoch) = 0;  // start an instance of the service kernel (ICRC_OK or an error)
    virtual int ended() = 0;                 // 1: the last instance has ended; 0: running or queued; < 0: error
    virtual ~RingDevice() = default;
};

// One message: n packets at dbase (device view), either uniform (ulen != 0: packet i at i * stride)
// or ragged (ulen == 0: off[i] / len[i], host arrays copied into the slot).  res: n ICRCs out.
struct RingJob {
    uint64_t dbase = 0;
    uint64_t stride = 0;
    uint32_t ulen = 0;
    const uint64_t *off = nullptr;
    const uint32_t *len = nullptr;
    uint32_t n = 0;
    uint32_t *res = nullptr;
};

struct RingStats {
    uint64_t jobs = 0, launches = 0, relaunches = 0, timeouts = 0;
};

class HostRing {
   public:
    // watchdog_us: a job not done after this long fails with ICRC_ETIMEDOUT and the ring is
    // retired (the caller runs the job, and later ones, as kernel launches).
    HostRing(RingDevice *dev, const RingMemory &mem, uint32_t nslots, uint32_t wg_per_slot, uint64_t watchdog_us);
    // Runs one job.  ICRC_OK; ICRC_EINVAL (n == 0 or > kRingMaxPackets); ICRC_ETIMEDOUT (watchdog);
    // ICRC_EDEVICE (launch failed, or the ring was retired).
    int submit(const RingJob &job);
    // Sets kRingStop in every slot and waits (host memory only: no device call) until every workgroup
    // of the current launch has stored its exited word, or wait_us.  Returns ICRC_OK or ICRC_ETIMEDOUT.
    int stop(uint64_t wait_us);
    bool retired() const { return retired_.load(std::memory_order_acquire); }
    // stop() has been called (engine destruction, process exit): unlike a ring retired by its
    // watchdog, callers must not fall back to kernel launches.
    bool stopped() const { return stopped_.load(std::memory_order_acquire); }
    RingStats stats() const;
    uint32_t epoch() const { return epoch_; }
    // A hint for device dispatch (no lock, no device call): an instance of the service kernel has
    // been launched and its workgroups have not all ended, so they hold their CUs.
    bool live() const { return launched_.load(std::memory_order_acquire) && !launch_ended(); }
    uint32_t workgroups() const { return nslots_ * wg_per_slot_; }
    uint32_t words_per_slot() const { return wps_; }

   private:
    int acquire_slot(uint32_t *slot);
    void release_slot(uint32_t slot);
    int ensure_running(bool force);
    bool job_done(uint32_t slot, uint32_t cmd) const;
    bool launch_ended() const;

    RingDevice *dev_;
    RingMemory mem_;
    uint32_t nslots_, wg_per_slot_, wps_;  // wps_: done / exited words per slot (one per workgroup)
    uint64_t watchdog_us_;
    std::mutex slot_mu_;
    std::condition_variable slot_cv_;
    uint32_t free_mask_;
    uint32_t seq_[kRingMaxSlots] = {};
    std::mutex launch_mu_;
    std::atomic<uint32_t> epoch_{0};
    std::atomic<bool> launched_{false};
    std::atomic<bool> retired_{false};
    std::atomic<bool> stopped_{false};
    std::atomic<uint32_t> activity_{0};
    mutable std::mutex stats_mu_;
    RingStats stats_;
};

uint64_t ring_now_us();

}  // namespace icrc
