// scripts/hostreadbench.hip — how fast can a kernel pull ONE configs[0] message (64 x 4156 B =
// 266 KB) out of pinned host memory, by load shape?  The submission ring's 64-packet job spends
// 13-14 us reading it (~20 GB/s, profiles/r05/ring/r05g) while four concurrent jobs move ~35 GB/s
// together: is a single burst limited by the load shape, the number of waves / CUs, or the link?
// Each case: `reps` launches, each wave stamps s_memrealtime before its first load and after its
// last load's data arrived; the burst = last end - first start (100 MHz ticks -> us), median over
// the launches.  Shapes: dword rows (the product's one-packet pipeline: 256 B per wave instruction)
// or dwordx4 (1 KiB per instruction), W waves in total (64 packets split evenly), workgroups of 16
// or 4 waves.  The data are XOR-folded (not ICRCs).
// Build: hipcc --offload-arch=gfx950 -O3 -o hostreadbench hostreadbench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr uint32_t kL = 4156, kN = 64, kBytes = kL * kN;  // 265,984 bytes

// The message as flat bytes [0, kBytes): wave w of W reads its share of dword (X4 = 0: 256 B per
// instruction) or dwordx4 (X4 = 1: 1 KiB) rows, all loads issued before the first use.
template <int X4>
__global__ void burst_kernel(const uint8_t *msg, uint32_t W, uint64_t *stamps, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= W) return;
    constexpr uint32_t RB = X4 ? 1024u : 256u;  // bytes per wave instruction
    const uint32_t rows = (kBytes + RB - 1) / RB;
    const uint32_t per = (rows + W - 1) / W;
    const uint32_t r0 = w * per, r1 = std::min(rows, r0 + per);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)msg, 0, (int)kBytes, 0x00020000);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    constexpr int MAXR = X4 ? 20 : 72;  // rows per wave at most (W >= 16: 65 dword / 17 dwordx4 rows)
    uint32_t v[MAXR * (X4 ? 4 : 1)];
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
        const uint32_t r = r0 + i;
        const int o = r < r1 ? (int)(r * RB + lane * (X4 ? 16u : 4u)) : (int)0x80000000;
        if constexpr (X4) {
            auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
            v[4 * i] = q[0];
            v[4 * i + 1] = q[1];
            v[4 * i + 2] = q[2];
            v[4 * i + 3] = q[3];
        } else {
            v[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < MAXR * (X4 ? 4 : 1); ++i) acc ^= v[i];
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        stamps[2 * w] = t0;
        stamps[2 * w + 1] = t1;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    uint8_t *msg = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&msg), kBytes, hipHostMallocDefault));
    for (uint32_t i = 0; i < kBytes; ++i) msg[i] = static_cast<uint8_t>(i * 131u + 7u);
    uint64_t *st;
    uint32_t *sink;
    CK(hipMalloc(&st, 2 * 1024 * sizeof(uint64_t)));
    CK(hipMalloc(&sink, 64));
    std::vector<uint64_t> h(2 * 1024);
    auto run = [&](const char *shape, auto kern, uint32_t W, uint32_t wpg) {
        std::vector<double> us;
        const uint32_t groups = (W + wpg - 1) / wpg;
        for (int rep = 0; rep < 60; ++rep) {
            kern<<<groups, wpg * 64>>>(msg, W, st, sink);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), st, 2 * W * sizeof(uint64_t), hipMemcpyDeviceToHost));
            uint64_t a = ~0ull, b = 0;
            for (uint32_t w = 0; w < W; ++w) {
                a = std::min(a, h[2 * w]);
                b = std::max(b, h[2 * w + 1]);
            }
            if (rep >= 10) us.push_back((b - a) * 0.01);
        }
        std::sort(us.begin(), us.end());
        const double med = us[us.size() / 2];
        printf("{\"shape\": \"%s\", \"waves\": %u, \"waves_per_group\": %u, \"burst_us_p50\": %.2f, \"burst_us_min\": %.2f, "
               "\"GB/s\": %.1f}\n", shape, W, wpg, med, us.front(), kBytes / (med * 1e-6) / 1e9);
        fflush(stdout);
    };
    for (int round = 0; round < 2; ++round) {
        for (uint32_t W : {16u, 32u, 64u, 128u, 256u}) {
            run("dword rows (256 B / instr)", burst_kernel<0>, W, 16);
            run("dword rows (256 B / instr)", burst_kernel<0>, W, 4);
            run("dwordx4 rows (1 KiB / instr)", burst_kernel<1>, W, 16);
            run("dwordx4 rows (1 KiB / instr)", burst_kernel<1>, W, 4);
        }
    }
    CK(hipHostFree(msg));
    return 0;
}
