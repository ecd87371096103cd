// icrc_ring_kernel.hip — the service kernel of the host-message submission ring (protocol and layout:
// icrc_internal.h RingSlot / RingParams; host side: icrc_ring.cpp, icrc_capi.cpp).  Its workgroups run
// the one-packet pipeline of icrc_long.h on each job — the same ICRC code as the batch kernel,
// bit-exact with compute_icrc (blue-rdma-device/src/third_party/net/packet_processor.rs:275-301).
#include <hip/hip_runtime.h>

#include "icrc_device.h"
#include "icrc_internal.h"
#include "icrc_long.h"

namespace icrc {
namespace {

// ---- host-message service kernel (the submission ring, icrc_internal.h / icrc_ring.cpp) -----------
// Workgroup b serves slot b / wg_per_slot.  While idle only wave 0 of each workgroup runs (the others
// wait at a barrier): it polls the slot's 64-byte line in coherent host memory, the whole line in one
// load (dword k in lane k).  On a new cmd whose line hash matches (ring_line_hash: a read torn by
// the host's writes is simply read again) it copies the line into the workgroup's decision line in
// device memory and invalidates this CU's and this XCD's cached lines of host memory (a system-scope
// acquire: the caller may have rewritten its packets since an earlier job read them, trailers or a new
// message in the same buffer, and the slot's offset / length arrays are rewritten every job; loads
// with sc0 sc1 alone were measured to return such a stale line, and so did skipping the acquire for
// coherent host memory — hipHostMallocCoherent lines are cached too).  Every wave reads the decision
// line after a barrier, so all of them take the same branch (the host line may change meanwhile: a
// stop bit).  The workgroup's waves take contiguous chunks of its share on the one-packet pipeline,
// results straight into the slot's coherent result array by system-scope stores; once every wave's
// stores have completed (s_waitcnt, then a barrier) wave 0 stores the cmd in the workgroup's done word.
// The end: kRingStop in the slot, or the exit flag, which the slot's leader (wave 0 of its first
// workgroup) sets when the host has made no call (RingSlot::activity) for idle_ticks or the launch
// has run for life_ticks (a persistent launch must not hold its CUs from other kernels for long:
// the host relaunches it on the next call).  The poll loop advances s_memrealtime on every path and
// its count is capped as well.
__device__ __forceinline__ uint32_t sys_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ void dev_store(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The 16 dwords of a 64-byte line, dword k in lane k (lanes 16..63: dword k & 15), one load.
__device__ __forceinline__ uint32_t line_load_sys(const RingSlot *line, uint32_t lane) {
    return sys_load(reinterpret_cast<const uint32_t *>(line) + (lane & 15u));
}
__device__ __forceinline__ uint32_t line_load_dev(const RingSlot *line, uint32_t lane) {
    return __hip_atomic_load(reinterpret_cast<const uint32_t *>(line) + (lane & 15u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t line_u64(uint32_t v, int dword) {
    return static_cast<uint64_t>(readlane_u32(v, dword)) | (static_cast<uint64_t>(readlane_u32(v, dword + 1)) << 32);
}

// The W = 64 table image into LDS from its compact form (table_fill's work, icrc_device.h, for a
// workgroup of NT threads: each thread takes the shares of threads t, t + NT, ...).
template <int NT>
__device__ __forceinline__ void ring_table_fill(uint4 *lds4, const uint32_t *table) {
    const uint32_t *cf = table + kLdsWords;
    for (uint32_t v = threadIdx.x; v < 1024u; v += NT) {
        const uint32_t bulk = cf[v];
        const uint32_t b = v >> 8, x = v & 255u;
        const uint32_t row = ((b >> 1) * 65536u + x * 256u + (b & 1u) * 128u) / 16u;
        const uint4 q = make_uint4(bulk, bulk, bulk, bulk);
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) lds4[row + ((k + x) & 7u)] = q;
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k)
            lds4[kFinalBase / 16u + v + k * 1024u] = reinterpret_cast<const uint4 *>(cf + 1024u)[v + k * 1024u];
    }
    __syncthreads();
}

template <int NT>
__global__ __launch_bounds__(NT) void icrc_ring_kernel(RingParams rp) {
    constexpr uint32_t kWaves = NT / 64;
    __shared__ uint4 lds4[kLdsBytes / 16];
    ring_table_fill<NT>(lds4, rp.table);  // ends in a barrier
    const char *lds = reinterpret_cast<const char *>(lds4);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    LaneConsts c;
    c.pc = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    c.fin = kFinalBase + lane * 4u;
    const uint32_t slot = blockIdx.x / rp.wg_per_slot, sub = blockIdx.x - slot * rp.wg_per_slot;
    const RingSlot *S = rp.slots + slot;
    const uint32_t widx = slot * rp.wg_per_slot + sub;
    RingSlot *D = rp.decision + widx;
    const bool leader = sub == 0u && wave == 0u;
    // jobs this workgroup finished in an earlier launch (the host may be waiting for the others)
    uint32_t last = __builtin_amdgcn_readfirstlane(sys_load(rp.done + widx));
    uint32_t act = 0u;
    uint64_t t_act = 0, t_launch = 0;
    if (leader) {
        act = readlane_u32(line_load_sys(S, lane), 1);
        t_act = t_launch = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t max_polls = 8ull * rp.idle_ticks + 4096u;  // a poll takes well over 1 tick
    uint64_t *tr = (rp.trace && sub == 0u && wave == 0u) ? rp.trace + slot * kRingTraceJobs * 4u : nullptr;
    uint64_t t_seen = 0;
    for (;;) {
        if (wave == 0u) {
            uint32_t dec = kRingStop;
            // Is this poll's (exit flag, line) the end of the wait?  dec is set when it is a job.
            auto look = [&](uint32_t efv, uint32_t v) __attribute__((always_inline)) -> bool {
                if (__builtin_amdgcn_readfirstlane(efv) == rp.epoch) return true;
                const uint32_t cmd = readlane_u32(v, 0);
                if (cmd & kRingStop) return true;
                if (cmd != last) {
                    uint32_t h = ring_line_hash(0x9E3779B9u, cmd);
                    for (int k = 2; k < 15; ++k) h = ring_line_hash(h, readlane_u32(v, k));
                    if (h != readlane_u32(v, 15)) return false;  // a torn line: read it again
                    if (lane >= 1u && lane < 16u)  // dword 0 (cmd) last, below
                        __hip_atomic_store(reinterpret_cast<uint32_t *>(D) + lane, v, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    if (!(rp.ab & 1u)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // stale host-memory lines out
                    dec = cmd;
                    if (tr) t_seen = __builtin_amdgcn_s_memrealtime();
                    return true;
                }
                if (leader) {
                    const uint32_t a = readlane_u32(v, 1);
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (a != act) {
                        act = a;
                        t_act = now;
                    }
                    // idle, or the launch's time is up (also while calls keep coming)
                    if (now - t_act > rp.idle_ticks || now - t_launch > rp.life_ticks) return true;
                }
                if (!(rp.ab & 4u)) __builtin_amdgcn_s_sleep(2);
                return false;
            };
            // one poll at a time: two in flight (the next loads issued before this pair is looked at)
            // compiled to a full wait at the loop head anyway
            for (uint64_t polls = 0; polls < max_polls; ++polls) {
                const uint32_t efv = __hip_atomic_load(rp.exit_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (look(efv, line_load_sys(S, lane))) break;  // the whole line: dword k in lane k
            }
            // no job (stop bit, exit flag, idle, lifetime or the poll cap): the whole launch ends
            if (dec == kRingStop) dev_store(rp.exit_flag, rp.epoch);
            dev_store(&D->cmd, dec);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();  // every wave reads wave 0's decision
        const uint32_t dl = line_load_dev(D, lane);  // RingSlot dwords: 0 cmd, 2 n, 3 ulen, 4-5 base, 6-7 stride,
        const uint32_t cmd = readlane_u32(dl, 0);     // 8-9 off, 10-11 len, 12-13 out
        if (cmd & kRingStop) break;
        const uint64_t t_dec = tr ? __builtin_amdgcn_s_memrealtime() : 0u;
        const uint32_t n = readlane_u32(dl, 2);
        BatchParams p{};
        p.n = n;
        p.ulen = readlane_u32(dl, 3);
        p.base = reinterpret_cast<uint8_t *>(line_u64(dl, 4));
        p.stride = line_u64(dl, 6);
        if (p.ulen == 0u) {
            p.off = reinterpret_cast<const uint64_t *>(line_u64(dl, 8));
            p.len = reinterpret_cast<const uint32_t *>(line_u64(dl, 10));
        }
        p.out = reinterpret_cast<uint32_t *>(line_u64(dl, 12));
        p.table = rp.table;
        p.skew = 0u;
        if (n <= kRingMaxPackets && !(rp.ab & 8u)) {  // the host never posts more; a corrupt line does nothing
            const uint32_t nwaves = rp.wg_per_slot * kWaves;
            const uint32_t chunk = (n + nwaves - 1u) / nwaves;
            const uint32_t w = sub * kWaves + wave;
            const uint32_t lo = w * chunk < n ? w * chunk : n;
            const uint32_t nq = (n - lo) < chunk ? (n - lo) : chunk;
            run_pipelined<kCompute, 2, 1, RingHostResults>(p, lds, c, lane, lo, nq);
        }
        // the results (system-scope stores: written through, complete once acknowledged — plain
        // stores without a release fence were measured to reach the host after the done word), then
        // (every wave past the barrier) the done word; an explicit wait the compiler cannot drop
        if (rp.ab & 2u) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // A/B: the fence as well
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // also: every wave has read the decision before wave 0 rewrites it
        const uint64_t t_res = tr ? __builtin_amdgcn_s_memrealtime() : 0u;
        if (wave == 0u && lane == 0u) sys_store(rp.done + widx, cmd);
        if (tr) {  // A/B trace (ICRC_RING_TRACE), record (job number % kRingTraceJobs): the done store's completion too
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t t_done = __builtin_amdgcn_s_memrealtime();
            const uint32_t tj = cmd % kRingTraceJobs;
            if (lane < 4u) tr[tj * 4u + lane] = lane == 0u ? t_seen : lane == 1u ? t_dec : lane == 2u ? t_res : t_done;
        }
        last = cmd;
    }
    if (wave == 0u) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0u) sys_store(rp.exited + widx, rp.epoch);
    }
}

}  // namespace

int launch_ring(const RingParams &rp, uint32_t nslots, void *stream) {
    if (nslots == 0 || rp.wg_per_slot == 0) return ICRC_EINVAL;
    const dim3 g(nslots * rp.wg_per_slot);
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (rp.threads) {
    case 256: hipLaunchKernelGGL(icrc_ring_kernel<256>, g, dim3(256), 0, s, rp); break;
    case 512: hipLaunchKernelGGL(icrc_ring_kernel<512>, g, dim3(512), 0, s, rp); break;
    case 1024: hipLaunchKernelGGL(icrc_ring_kernel<1024>, g, dim3(1024), 0, s, rp); break;
    default: return ICRC_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc
