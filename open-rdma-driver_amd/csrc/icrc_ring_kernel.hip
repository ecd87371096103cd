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
// wait at a barrier): it polls the slot's line in coherent host memory.  On a new cmd it reads the
// whole line again (one load per lane: the fields the host wrote before cmd) and copies it into the
// workgroup's decision line in device memory; every wave reads that line after a barrier, so all of
// them take the same branch (the host line may change meanwhile: a stop bit).  The workgroup's waves
// take contiguous chunks of its share on the one-packet pipeline — its row loads system-coherent
// (sc0 sc1: the caller may have rewritten its packets since an earlier job read them, trailers or a
// new message in the same buffer, and no cached line of host memory may answer) — results straight
// into the slot's coherent result array; after a system-scope release and a second barrier wave 0
// stores the cmd in the workgroup's done word.
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
__device__ __forceinline__ uint32_t dev_load(const uint32_t *p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
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
// The ring's row loads: system-coherent, read-once (sc0 nt sc1).
constexpr int kRingRowAux = 0x13;

__global__ __launch_bounds__(kThreadsPerGroup) void icrc_ring_kernel(RingParams rp) {
    __shared__ uint4 lds4[kLdsBytes / 16];
    table_fill(lds4, rp.table);  // ends in a barrier
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
        act = __builtin_amdgcn_readfirstlane(sys_load(&S->activity));
        t_act = t_launch = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t max_polls = 8ull * rp.idle_ticks + 4096u;  // a poll takes well over 1 tick
    for (;;) {
        if (wave == 0u) {
            uint32_t dec = kRingStop;
            for (uint64_t polls = 0; polls < max_polls; ++polls) {
                if (dev_load(rp.exit_flag) == rp.epoch) break;
                const uint32_t cmd = __builtin_amdgcn_readfirstlane(sys_load(&S->cmd));
                if (cmd & kRingStop) break;
                if (cmd != last) {
                    // the host wrote the fields, then cmd: read the line again after cmd has arrived
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const uint32_t v = line_load_sys(S, lane);
                    if (lane >= 1u && lane < 16u)  // dword 0 (cmd) last, below
                        __hip_atomic_store(reinterpret_cast<uint32_t *>(D) + lane, v, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    dec = cmd;
                    break;
                }
                if (leader) {
                    const uint32_t a = __builtin_amdgcn_readfirstlane(sys_load(&S->activity));
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (a != act) {
                        act = a;
                        t_act = now;
                    } else if (now - t_act > rp.idle_ticks || now - t_launch > rp.life_ticks) {
                        dev_store(rp.exit_flag, rp.epoch);  // idle, or the launch's time is up
                        break;
                    }
                    if (now - t_launch > rp.life_ticks) {  // time up while calls keep coming
                        dev_store(rp.exit_flag, rp.epoch);
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(2);
                if (polls + 1u == max_polls) dev_store(rp.exit_flag, rp.epoch);
            }
            dev_store(&D->cmd, dec);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();  // every wave reads wave 0's decision
        const uint32_t dl = line_load_dev(D, lane);  // RingSlot dwords: 0 cmd, 2 n, 3 ulen, 4-5 base, 6-7 stride,
        const uint32_t cmd = readlane_u32(dl, 0);     // 8-9 off, 10-11 len, 12-13 out
        if (cmd & kRingStop) break;
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
        if (n <= kRingMaxPackets) {  // the host never posts more; a corrupt line does nothing
            const uint32_t nwaves = rp.wg_per_slot * kWavesPerGroup;
            const uint32_t chunk = (n + nwaves - 1u) / nwaves;
            const uint32_t w = sub * kWavesPerGroup + wave;
            const uint32_t lo = w * chunk < n ? w * chunk : n;
            const uint32_t nq = (n - lo) < chunk ? (n - lo) : chunk;
            run_pipelined<kCompute, 2, 1, Ring<kRingRowAux>>(p, lds, c, lane, lo, nq);
        }
        // the results, then (every wave past the barrier) the done word: the release recipe of the
        // guide (fence, an explicit wait the compiler cannot drop, then the flag)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // also: every wave has read the decision before wave 0 rewrites it
        if (wave == 0u && lane == 0u) sys_store(rp.done + widx, cmd);
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
    hipLaunchKernelGGL(icrc_ring_kernel, dim3(nslots * rp.wg_per_slot), dim3(kThreadsPerGroup), 0,
                       static_cast<hipStream_t>(stream), rp);
    return hipGetLastError() == hipSuccess ? ICRC_OK : ICRC_EDEVICE;
}

}  // namespace icrc
