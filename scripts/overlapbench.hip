// scripts/overlapbench.hip — where the C1 kernel loses to its loads-only build (bench.py reports
// the kernel at ~0.93 of it).  Every form walks 1 Mi x 4156-B packets (17 end-aligned 256-B dword
// rows per packet, nt loads, one packet per wavefront) and applies the product's row step
// acc <- M^64(acc) ^ row (four v_perm-addressed LDS byte-table lookups) — no header masks, no final
// products: the question is memory/compute overlap, not the ICRC.  Forms:
//   loads      S = 2 chains, next set prefetched, no step (the access shape)
//   product    S = 2, D = 1, 128 KiB tables (32 bank copies), 1 workgroup / CU (16 waves)
//   dynamic    as product, but sets are handed out by atomic tickets (one per set), per XCD or
//              per workgroup
//   s1x2       S = 1, D = 1, 64 KiB tables (16 copies), 2 workgroups / CU (32 waves, <= 64 VGPRs)
//              (measured slower than product, profiles/r02_overlapbench.jsonl; not run any more)
//   s2 64K     product with 64 KiB tables (16 copies)
// Per-wave start / end times (s_memrealtime, 100 MHz) give the tail: how long after the median
// wave the last one ends.  Each form's per-lane XOR of results must agree with product's.
// Build: hipcc --offload-arch=gfx950 -O3 -o overlapbench overlapbench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr uint32_t kN = 1u << 20, kL = 4156, kR = 17;
constexpr int kWaves = 16;

struct Args {
    const uint8_t *base;
    const uint32_t *tab;  // table image (128 KiB or 64 KiB layout)
    uint32_t *out;        // per wave: 64 lanes of result XOR
    uint64_t *ts;         // per wave: start, end
    uint32_t *tickets;    // dynamic: 8 per-XCD counters (never reset; base below)
    uint32_t ticket_base; // dynamic: counter value at this launch's start
    uint32_t waves;       // waves in the grid
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// 128 KiB layout: (b >> 1) * 65536 + x * 256 + (b & 1) * 128 + (lane & 31) * 4
// 64 KiB layout:  x * 256 + b * 64 + (lane & 15) * 4
template <bool T64>
__device__ __forceinline__ uint32_t step(const char *lds, uint32_t s, uint32_t u, uint32_t pc) {
    auto at = [&](uint32_t a) { return *reinterpret_cast<const uint32_t *>(lds + a); };
    if constexpr (!T64) {
        return xor3(xor3(u, at(__builtin_amdgcn_perm(s, pc, 0x0C0C0400u)), at(__builtin_amdgcn_perm(s, pc, 0x0C0C0501u))),
                    at(__builtin_amdgcn_perm(s, pc, 0x0C020600u)), at(__builtin_amdgcn_perm(s, pc, 0x0C020701u)));
    } else {
        return xor3(xor3(u, at(__builtin_amdgcn_perm(s, pc, 0x0C0C0400u)), at(__builtin_amdgcn_perm(s, pc, 0x0C0C0501u))),
                    at(__builtin_amdgcn_perm(s, pc, 0x0C0C0602u)), at(__builtin_amdgcn_perm(s, pc, 0x0C0C0703u)));
    }
}

__device__ __forceinline__ void load_rows(const Args &a, uint32_t pk, bool live, uint32_t lane, uint32_t (&u)[kR]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.base) + (size_t)pk * kL, 0,
                                                                        live ? (int)(kL - 4) : 0, 0x00020000);
    const uint32_t vb = 4u * (lane - 50u);  // k0 = -49: rows end-aligned, row 0 lanes < 50 out of range
#pragma unroll
    for (int j = 0; j < (int)kR; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 256u * j), 0, 2);
}

// MODE 0 loads only, 1 step.  S chains per set, one set prefetched.  DYN: 0 static contiguous
// ranges; 1 sets handed out by per-XCD tickets; 2 by per-workgroup tickets.  A ticket is a buffer
// atomic (lane 0 in range, the others out of range: no branch) issued BEFORE the loads of the set
// in flight and read one iteration later, so waiting for it never waits for those loads.
// OPT: 0 plain; 1 s_setprio(3) around each set's load burst; 2 the next set's row loads issued
// one row per row step of the current set (pinned by sched_barrier)
template <int MODE, int S, bool T64, int DYN, int OPT = 0>
__device__ __forceinline__ void body(const Args &a, const char *lds) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t pc = T64 ? ((lane & 15u) * 4u) | (((lane & 15u) * 4u + 64u) << 8) | (((lane & 15u) * 4u + 128u) << 16) |
                                  (((lane & 15u) * 4u + 192u) << 24)
                            : ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 16);
    const uint32_t nsets_all = kN / S;
    const uint32_t owner = DYN == 1 ? (blockIdx.x & 7u) : blockIdx.x;  // ticket counter / set range
    const uint32_t per_owner = DYN == 1 ? nsets_all / 8u : nsets_all / gridDim.x;
    uint32_t lo = 0, nsets = 0;
    if (DYN == 0) {
        const uint32_t chunk = (nsets_all + a.waves - 1) / a.waves;
        lo = gw * chunk;
        nsets = lo < nsets_all ? (nsets_all - lo < chunk ? nsets_all - lo : chunk) : 0u;
    } else {
        lo = owner * per_owner;
        nsets = per_owner;
    }
    const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(a.tickets, 0, 1 << 20, 0x00020000);
    auto req = [&]() -> uint32_t {
        return (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, trs, (int)(lane == 0 ? owner * 128u : 0x80000000u), 0, 0);
    };
    auto take = [&](uint32_t raw) -> uint32_t { return __builtin_amdgcn_readfirstlane(raw) - a.ticket_base; };
    uint32_t ua[S][kR], ub[S][kR], tot = 0;
    uint32_t cur = DYN ? take(req()) : 0u, nraw = DYN ? req() : 0u;
    auto set_pk = [&](uint32_t st, int s) -> uint32_t { return (lo + st) * S + s; };
    auto live = [&](uint32_t st) { return st < nsets; };
#pragma unroll
    for (int s = 0; s < S; ++s) load_rows(a, set_pk(cur, s), live(cur), lane, ua[s]);
    auto process = [&](uint32_t (&u)[S][kR], uint32_t st) {
        uint32_t acc[S];
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = u[s][0];
#pragma unroll
        for (int j = 1; j < (int)kR; ++j)
#pragma unroll
            for (int s = 0; s < S; ++s) acc[s] = MODE == 0 ? acc[s] ^ u[s][j] : step<T64>(lds, acc[s], u[s][j], pc);
#pragma unroll
        for (int s = 0; s < S; ++s) tot ^= acc[s] * (set_pk(st, s) | 1u);
    };
    // OPT 2: step row j of the current set, then load row j of the next one
    auto process_il = [&](uint32_t (&u)[S][kR], uint32_t st, uint32_t (&v)[S][kR], uint32_t nst) {
        __amdgpu_buffer_rsrc_t rs[S];
#pragma unroll
        for (int s = 0; s < S; ++s)
            rs[s] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.base) + (size_t)set_pk(nst, s) * kL, 0,
                                                      live(nst) ? (int)(kL - 4) : 0, 0x00020000);
        const uint32_t vb = 4u * (lane - 50u);
        uint32_t acc[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            acc[s] = u[s][0];
            v[s][0] = __builtin_amdgcn_raw_buffer_load_b32(rs[s], (int)vb, 0, 2);
        }
#pragma unroll
        for (int j = 1; j < (int)kR; ++j) {
#pragma unroll
            for (int s = 0; s < S; ++s) acc[s] = step<T64>(lds, acc[s], u[s][j], pc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < S; ++s) v[s][j] = __builtin_amdgcn_raw_buffer_load_b32(rs[s], (int)(vb + 256u * j), 0, 2);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) tot ^= acc[s] * (set_pk(st, s) | 1u);
    };
    if constexpr (OPT == 2) {
        for (uint32_t it = 0;; it += 2) {
            if (!live(cur)) break;
            process_il(ua, cur, ub, it + 1);
            cur = it + 1;
            if (!live(cur)) break;
            process_il(ub, cur, ua, it + 2);
            cur = it + 2;
        }
    } else {
    for (uint32_t it = 0;; it += 2) {
        uint32_t nb = DYN ? take(nraw) : it + 1;
        if (DYN) nraw = req();
        if (OPT == 1) __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int s = 0; s < S; ++s) load_rows(a, set_pk(nb, s), live(nb), lane, ub[s]);
        if (OPT == 1) __builtin_amdgcn_s_setprio(0);
        if (!live(cur)) break;
        process(ua, cur);
        cur = nb;
        nb = DYN ? take(nraw) : it + 2;
        if (DYN) nraw = req();
        if (OPT == 1) __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int s = 0; s < S; ++s) load_rows(a, set_pk(nb, s), live(nb), lane, ua[s]);
        if (OPT == 1) __builtin_amdgcn_s_setprio(0);
        if (!live(cur)) break;
        process(ub, cur);
        cur = nb;
    }
    }
    a.out[gw * 64u + lane] = tot;
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        a.ts[2 * gw] = t0;
        a.ts[2 * gw + 1] = t1;
    }
}

template <int MODE, int S, bool T64, int DYN, int OPT = 0>
__global__ __launch_bounds__(1024) void k1(Args a) {
    __shared__ uint4 lds4[(T64 ? 65536 : 131072) / 16];
    if (MODE != 0) {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.tab);
        for (uint32_t i = threadIdx.x; i < (T64 ? 65536u : 131072u) / 16u; i += 1024u) lds4[i] = src[i];
        __syncthreads();
    }
    body<MODE, S, T64, DYN, OPT>(a, reinterpret_cast<const char *>(lds4));
}

// two workgroups per CU: 8 waves per SIMD, at most 64 VGPRs
__global__ __attribute__((amdgpu_flat_work_group_size(1024, 1024), amdgpu_waves_per_eu(8, 8))) void k2(Args a) {
    __shared__ uint4 lds4[65536 / 16];
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tab);
    for (uint32_t i = threadIdx.x; i < 65536u / 16u; i += 1024u) lds4[i] = src[i];
    __syncthreads();
    body<1, 1, true, 0>(a, reinterpret_cast<const char *>(lds4));
}

static uint32_t shift_bits(uint32_t s, int bits) {
    for (int i = 0; i < bits; ++i) s = (s >> 1) ^ ((s & 1u) ? 0xEDB88320u : 0u);
    return s;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::vector<uint32_t> col(32);
    for (int i = 0; i < 32; ++i) col[i] = shift_bits(1u << i, 2048);
    auto byte_tab = [&](int b, uint32_t x) {
        uint32_t v = 0;
        for (int i = 0; i < 8; ++i)
            if (x >> i & 1u) v ^= col[8 * b + i];
        return v;
    };
    std::vector<uint32_t> t128(32768), t64(16384);
    for (int b = 0; b < 4; ++b)
        for (uint32_t x = 0; x < 256; ++x) {
            const uint32_t v = byte_tab(b, x);
            for (uint32_t l = 0; l < 32; ++l) t128[((b >> 1) * 65536 + x * 256 + (b & 1) * 128 + l * 4) / 4] = v;
            for (uint32_t l = 0; l < 16; ++l) t64[(x * 256 + b * 64 + l * 4) / 4] = v;
        }
    uint8_t *d;
    uint32_t *tab128, *tab64, *out, *tickets;
    uint64_t *ts;
    const size_t bytes = (size_t)kN * kL;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&tab128, 131072));
    CK(hipMalloc(&tab64, 65536));
    const uint32_t max_waves = 2 * cus * kWaves;
    CK(hipMalloc(&out, (size_t)max_waves * 64 * 4));
    CK(hipMalloc(&ts, (size_t)max_waves * 16));
    CK(hipMalloc(&tickets, 1 << 20));
    CK(hipMemset(tickets, 0, 1 << 20));
    CK(hipMemcpy(tab128, t128.data(), 131072, hipMemcpyHostToDevice));
    CK(hipMemcpy(tab64, t64.data(), 65536, hipMemcpyHostToDevice));
    {
        std::vector<uint32_t> h(bytes / 4);
        uint64_t s = 0x9E3779B97F4A7C15ull;
        for (auto &w : h) {
            s ^= s << 13;
            s ^= s >> 7;
            s ^= s << 17;
            w = static_cast<uint32_t>(s);
        }
        CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint32_t ticket_base = 0;  // every counter advances by its sets + 3 failing tickets per wave, per launch
    std::vector<uint32_t> ref;
    auto run = [&](const char *name, auto kern, int grid, const uint32_t *tab, int dyn, int S) {
        Args a{d, tab, out, ts, tickets, 0, (uint32_t)grid * kWaves};
        const uint32_t owners = dyn == 1 ? 8u : (uint32_t)grid;
        const uint32_t inc = kN / S / owners + 3u * ((uint32_t)grid * kWaves / owners);
        CK(hipMemset(tickets, 0, 1 << 20));
        ticket_base = 0;
        auto launch = [&]() {
            a.ticket_base = ticket_base;
            kern<<<grid, 1024>>>(a);
            if (dyn) ticket_base += inc;
        };
        CK(hipMemset(out, 0, (size_t)max_waves * 256));
        launch();
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> all((size_t)grid * kWaves * 64), h(64, 0u);
        CK(hipMemcpy(all.data(), out, all.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < all.size(); ++i) h[i & 63] ^= all[i];
        int agree = -1;
        if (std::string(name) != "loads") {
            if (ref.empty()) ref = h;
            agree = ref == h;
        }
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::vector<uint64_t> t((size_t)grid * kWaves * 2);
        CK(hipMemcpy(t.data(), ts, t.size() * 8, hipMemcpyDeviceToHost));
        uint64_t s0 = ~0ull;
        std::vector<double> ends;
        for (size_t w = 0; w < t.size() / 2; ++w) s0 = std::min(s0, t[2 * w]);
        for (size_t w = 0; w < t.size() / 2; ++w) ends.push_back((t[2 * w + 1] - s0) * 0.01);  // us
        std::vector<double> wg;  // per workgroup: its last wave's end
        for (size_t g = 0; g < ends.size() / kWaves; ++g)
            wg.push_back(*std::max_element(ends.begin() + g * kWaves, ends.begin() + (g + 1) * kWaves));
        std::sort(ends.begin(), ends.end());
        std::sort(wg.begin(), wg.end());
        printf("{\"form\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GB/s\": %.1f, \"agrees\": %d, \"wave_end_us\": "
               "{\"min\": %.1f, \"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, \"wg_end_us\": {\"min\": %.1f, \"p50\": %.1f, "
               "\"max\": %.1f}}\n",
               name, grid, ms, (double)kN * (kL - 4) / (ms * 1e-3) / 1e9, agree, ends.front(), ends[ends.size() / 2],
               ends[ends.size() * 99 / 100], ends.back(), wg.front(), wg[wg.size() / 2], wg.back());
        fflush(stdout);
    };
    for (int round = 0; round < 2; ++round) {
        run("product", k1<1, 2, false, 0>, cus, tab128, 0, 2);
        run("loads", k1<0, 2, false, 0>, cus, tab128, 0, 2);
        run("product + setprio(3) around the load bursts", k1<1, 2, false, 0, 1>, cus, tab128, 0, 2);
        run("product, next set's loads interleaved with the row steps", k1<1, 2, false, 0, 2>, cus, tab128, 0, 2);
        run("S = 1, next packet's loads interleaved", k1<1, 1, false, 0, 2>, cus, tab128, 0, 1);
    }
    return 0;
}
