// scripts/coresbench.hip — would an oct workgroup and a long-packet workgroup sharing a CU beat
// running them one after the other?  ("let the two halves share CUs".)
//
// Two stand-ins with the product's access shapes and an LDS table step of 16 bank copies (the
// smallest image that stays conflict-light, profiles/r05/c2/stepbench_bank_copies.jsonl):
//   S (short half): 8 packets of 316 B per wave, 32-byte dword rows per packet (10 rows, end-aligned),
//     per row acc <- T(acc) ^ word (4 LDS reads), plus WORK dependent VALU per 8-packet set (the oct
//     kernel's per-set control), the next set's rows in flight;
//   L (long half): one 4096-byte packet per wave, 16 rows of 64 dwords, the same step, the next
//     packet's rows in flight.
// Bytes follow configs[2]'s split: S reads 5 Mi x 316 B (1.66 GB), L 56 K x 4096 B (0.23 GB).
// Each kernel asks for LDS_KIB of dynamic LDS, which sets how many workgroups share a CU
// (160 KiB: one; 80 KiB: two).  Timed (HIP events, 10 reps): each half alone with 1024-thread
// workgroups one per CU and with 512-thread ones two per CU; both halves one after the other (the
// hybrid launch today, minus its backfill); both halves in ONE launch of 512-thread workgroups,
// 80 KiB each, role by block parity (co-resident); and the two on two streams at once.
// Results are XOR-folded and stored once per wave; they are not ICRCs.
// Build: hipcc --offload-arch=gfx950 -O3 -o coresbench coresbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr uint32_t kOOR = 0x80000000u;
constexpr uint32_t kShortL = 316, kShortRows = 10;  // 10 x 32 B >= 316, end-aligned
constexpr uint32_t kLongRows = 16;                  // 16 x 256 B = 4096 B
constexpr uint32_t kTableWords = 4u * 256u * 16u;   // 16 bank copies: 64 KiB

__device__ __forceinline__ uint32_t step16(uint32_t acc, const char *t, uint32_t lane) {
    const uint32_t l = (lane & 15u) * 4u;
    const uint32_t a0 = ((acc & 0xFFu) << 6) | l, a1 = (((acc >> 8) & 0xFFu) << 6) | l;
    const uint32_t a2 = (((acc >> 16) & 0xFFu) << 6) | l, a3 = ((acc >> 24) << 6) | l;
    return *reinterpret_cast<const uint32_t *>(t + a0) ^ *reinterpret_cast<const uint32_t *>(t + 16384 + a1) ^
           *reinterpret_cast<const uint32_t *>(t + 32768 + a2) ^ *reinterpret_cast<const uint32_t *>(t + 49152 + a3);
}

template <int WORK>
__device__ void short_half(const uint8_t *base, uint32_t n, const char *t, uint32_t gw, uint32_t tw, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63u, grp = lane >> 3, col = lane & 7u;
    const uint32_t chunk = ((n + tw - 1) / tw + 7u) & ~7u;
    const uint32_t lo = gw * chunk;
    if (lo >= n) return;
    const uint32_t nq = n - lo < chunk ? n - lo : chunk;
    const uint32_t nsets = nq / 8u;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)lo * kShortL), 0, (int)(nq * kShortL), 0x00020000);
    uint32_t ua[kShortRows], ub[kShortRows], acc = 0;
    auto load = [&](uint32_t set, uint32_t(&u)[kShortRows]) __attribute__((always_inline)) {
        const uint32_t q = set * 8u + grp;
        const int vb = (int)(q * kShortL + kShortL) - (int)(kShortRows * 32u) + (int)(col * 4u);
#pragma unroll
        for (int j = 0; j < (int)kShortRows; ++j) {
            const int o = vb + 32 * j;
            u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (set < nsets && o >= (int)(q * kShortL)) ? o : (int)kOOR, 0, 0);
        }
    };
    auto fold = [&](uint32_t(&u)[kShortRows]) __attribute__((always_inline)) {
        uint32_t a = acc;
#pragma unroll
        for (int j = 0; j < (int)kShortRows; ++j) a = step16(a, t, lane) ^ u[j];
#pragma unroll
        for (int w = 0; w < WORK; ++w) a = __builtin_amdgcn_perm(a, a + static_cast<uint32_t>(w), 0x05040302u + w);
        acc = a;
    };
    load(0, ua);
    for (uint32_t s = 0; s < nsets; s += 2) {
        load(s + 1, ub);
        fold(ua);
        load(s + 2, ua);
        fold(ub);
    }
    out[gw * 64u + lane] = acc;
}

__device__ void long_half(const uint32_t *base, uint32_t n, const char *t, uint32_t gw, uint32_t tw, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunk = (n + tw - 1) / tw;
    const uint32_t lo = gw * chunk;
    if (lo >= n) return;
    const uint32_t hi = lo + chunk < n ? lo + chunk : n;
    const uint32_t *p = base + static_cast<size_t>(lo) * (kLongRows * 64u) + lane;
    uint32_t cur[kLongRows], nxt[kLongRows], total = 0;
#pragma unroll
    for (int r = 0; r < (int)kLongRows; ++r) cur[r] = __builtin_nontemporal_load(p + r * 64);
    for (uint32_t q = lo; q < hi; ++q) {
        const uint32_t *pn = p + (q + 1 < hi ? (q + 1 - lo) : 0u) * static_cast<size_t>(kLongRows * 64u);
#pragma unroll
        for (int r = 0; r < (int)kLongRows; ++r) nxt[r] = __builtin_nontemporal_load(pn + r * 64);
        uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
        for (int r = 0; r < (int)kLongRows; ++r) acc = step16(acc, t, lane) ^ cur[r];
        total ^= acc * (q | 1u);
#pragma unroll
        for (int r = 0; r < (int)kLongRows; ++r) cur[r] = nxt[r];
    }
    out[gw * 64u + lane] = total;
}

__device__ __forceinline__ void fill(uint32_t *lds, const uint32_t *tables) {
    for (uint32_t i = threadIdx.x; i < kTableWords; i += blockDim.x) lds[i] = tables[i];
    __syncthreads();
}

// ROLE: 0 short, 1 long, 2 by block parity (even: short, odd: long; each role gets gridDim / 2)
template <int ROLE, int WORK>
__global__ __launch_bounds__(1024) void cores_kernel(const uint8_t *sbase, uint32_t ns, const uint32_t *lbase,
                                                     uint32_t nl, const uint32_t *tables, uint32_t *out_s,
                                                     uint32_t *out_l) {
    extern __shared__ uint32_t lds[];
    fill(lds, tables);
    const char *t = reinterpret_cast<const char *>(lds);
    const uint32_t wpb = blockDim.x >> 6, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (ROLE == 2) {
        const uint32_t half = gridDim.x / 2u, b = blockIdx.x >> 1;
        if (blockIdx.x & 1u) long_half(lbase, nl, t, b * wpb + wave, half * wpb, out_l);
        else short_half<WORK>(sbase, ns, t, b * wpb + wave, half * wpb, out_s);
    } else if constexpr (ROLE == 1) {
        long_half(lbase, nl, t, blockIdx.x * wpb + wave, gridDim.x * wpb, out_l);
    } else {
        short_half<WORK>(sbase, ns, t, blockIdx.x * wpb + wave, gridDim.x * wpb, out_s);
    }
}

template <class F>
float time_it(F f, int reps, hipStream_t s) {  // events on s: every case forks / joins back to it
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int WORK>
void run_all(int cus, const uint8_t *sb, uint32_t ns, const uint32_t *lb, uint32_t nl, const uint32_t *tab,
             uint32_t *os, uint32_t *ol, hipStream_t s1, hipStream_t s2) {
    const size_t big = 160u << 10, half = 80u << 10;
    for (auto k : {(const void *)cores_kernel<0, WORK>, (const void *)cores_kernel<1, WORK>,
                   (const void *)cores_kernel<2, WORK>})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)big));
    const double bs = (double)ns * kShortL, bl = (double)nl * 4096.0;
    auto line = [&](const char *what, float ms, double bytes) {
        printf("{\"work\": %d, \"case\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f}\n", WORK, what, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const int reps = 10;
    line("short alone, 1024 x 1 / CU", time_it([&] { cores_kernel<0, WORK><<<cus, 1024, big, s1>>>(sb, ns, lb, nl, tab, os, ol); }, reps, s1), bs);
    line("short alone, 512 x 2 / CU", time_it([&] { cores_kernel<0, WORK><<<2 * cus, 512, half, s1>>>(sb, ns, lb, nl, tab, os, ol); }, reps, s1), bs);
    line("long alone, 1024 x 1 / CU", time_it([&] { cores_kernel<1, WORK><<<cus, 1024, big, s1>>>(sb, ns, lb, nl, tab, os, ol); }, reps, s1), bl);
    line("long alone, 512 x 2 / CU", time_it([&] { cores_kernel<1, WORK><<<2 * cus, 512, half, s1>>>(sb, ns, lb, nl, tab, os, ol); }, reps, s1), bl);
    line("short then long, 1024 x 1 / CU each", time_it([&] {
             cores_kernel<0, WORK><<<cus, 1024, big, s1>>>(sb, ns, lb, nl, tab, os, ol);
             cores_kernel<1, WORK><<<cus, 1024, big, s1>>>(sb, ns, lb, nl, tab, os, ol);
         }, reps, s1), bs + bl);
    line("one launch, 512 x 2 / CU, role by block parity (co-resident)", time_it([&] {
             cores_kernel<2, WORK><<<2 * cus, 512, half, s1>>>(sb, ns, lb, nl, tab, os, ol);
         }, reps, s1), bs + bl);
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    line("two streams at once, 512-thread 80 KiB workgroups, #CUs each", time_it([&] {
             CK(hipEventRecord(fork, s1));
             CK(hipStreamWaitEvent(s2, fork, 0));
             cores_kernel<0, WORK><<<cus, 512, half, s1>>>(sb, ns, lb, nl, tab, os, ol);
             cores_kernel<1, WORK><<<cus, 512, half, s2>>>(sb, ns, lb, nl, tab, os, ol);
             CK(hipEventRecord(join, s2));
             CK(hipStreamWaitEvent(s1, join, 0));
         }, reps, s1), bs + bl);
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint32_t ns = 5u << 20, nl = 56u << 10;
    uint8_t *sb;
    uint32_t *lb, *tab, *os, *ol;
    CK(hipMalloc(&sb, (size_t)ns * kShortL));
    CK(hipMalloc(&lb, (size_t)nl * 4096));
    CK(hipMemset(sb, 0x5a, (size_t)ns * kShortL));
    CK(hipMemset(lb, 0x3c, (size_t)nl * 4096));
    std::vector<uint32_t> h(kTableWords);
    uint32_t x = 0x12345u;
    for (auto &w : h) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        w = x;
    }
    CK(hipMalloc(&tab, kTableWords * 4));
    CK(hipMemcpy(tab, h.data(), kTableWords * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&os, (size_t)2 * cus * 16 * 64 * 4));
    CK(hipMalloc(&ol, (size_t)2 * cus * 16 * 64 * 4));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int round = 0; round < 2; ++round) {
        run_all<0>(cus, sb, ns, lb, nl, tab, os, ol, s1, s2);
        run_all<60>(cus, sb, ns, lb, nl, tab, os, ol, s1, s2);
    }
    return 0;
}
