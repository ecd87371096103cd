// scripts/membench.hip — achievable HBM read bandwidth on MI355X for the ICRC access shapes
// ("measured achievable streaming-read bandwidth ... as a secondary denominator").
// Reads a 1 Mi x 4156-B packet batch (4.36 GB, stride 4156 = 4-byte aligned packets) in:
//   A  flat dwordx4 grid-stride sweep (the copy-style ceiling), 16 or 32 waves/CU
//   B  wave per packet, 256-B rows of buffer_load_dword (the v1 kernel's shape), P in flight
//   C  wave per packet, 1-KiB rows of buffer_load_dwordx4 (16 B/lane), P in flight
// Each kernel XOR-folds what it reads and stores one word per wave (no dead-code removal).
// Build: hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
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

constexpr uint32_t kL = 4156;
constexpr uint32_t kN = 1u << 20;

__global__ void flat_x4(const uint4 *p, size_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int P>
__global__ __launch_bounds__(1024) void rows_dword(const uint8_t *base, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    uint32_t acc = 0;
    const int N = 1 + (kL - 4) / 4, R = (N + 63) / 64, k0 = N - 64 * R;
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + wave; i < kN; i += P * tw) {
        uint32_t u[P][17];
#pragma unroll
        for (int s = 0; s < P; ++s) {
            uint32_t pi = i + s * tw;
            const uint8_t *pkt = base + (size_t)(pi < kN ? pi : 0) * kL;
            auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)pkt, 0, pi < kN ? (int)(kL - 4) : 0, 0x00020000);
            uint32_t vb = 4u * (uint32_t)(k0 - 1 + (int)lane);
#pragma unroll
            for (int j = 0; j < 17; ++j) u[s][j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 256u * j), 0, 0);
        }
#pragma unroll
        for (int s = 0; s < P; ++s)
#pragma unroll
            for (int j = 0; j < 17; ++j) acc ^= u[s][j];
    }
    out[blockIdx.x * (blockDim.x / 64) + wave] = acc;
}

template <int P>
__global__ __launch_bounds__(1024) void rows_x4(const uint8_t *base, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    uint32_t acc = 0;
    const int N = 1 + (kL - 4) / 4, R = (N + 255) / 256, k0 = N - 256 * R;
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + wave; i < kN; i += P * tw) {
        uint4 u[P][5];
#pragma unroll
        for (int s = 0; s < P; ++s) {
            uint32_t pi = i + s * tw;
            const uint8_t *pkt = base + (size_t)(pi < kN ? pi : 0) * kL;
            auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)pkt, 0, pi < kN ? (int)(kL - 4) : 0, 0x00020000);
            uint32_t vb = 4u * (uint32_t)(k0 - 1 + 4 * (int)lane);
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vb + 1024u * j), 0, 0);
                u[s][j] = *reinterpret_cast<uint4 *>(&v);
            }
        }
#pragma unroll
        for (int s = 0; s < P; ++s)
#pragma unroll
            for (int j = 0; j < 5; ++j) acc ^= u[s][j].x ^ u[s][j].y ^ u[s][j].z ^ u[s][j].w;
    }
    out[blockIdx.x * (blockDim.x / 64) + wave] = acc;
}

// D: wave owns a contiguous chunk of packets (the pipelined kernel's assignment), one packet
// prefetched ahead; STORE = 0 none, 1 per-packet 4-B store, 2 one coalesced store per 64.
template <int STORE>
__global__ __launch_bounds__(1024) void rows_chunk(const uint8_t *base, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave;
    const uint32_t chunk = ((kN + tw - 1) / tw + 63) & ~63u;
    const uint32_t lo = gw * chunk;
    if (lo >= kN) return;
    const uint32_t nq = kN - lo < chunk ? kN - lo : chunk;
    const int N = 1 + (kL - 4) / 4, R = (N + 63) / 64, k0 = N - 64 * R;
    const uint32_t vb = 4u * (uint32_t)(k0 - 1 + (int)lane);
    uint32_t ua[17], ub[17], buf = 0;
    auto load = [&](uint32_t q, uint32_t(&u)[17]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)(lo + q) * kL), 0, (int)(kL - 4), 0x00020000);
#pragma unroll
        for (int j = 0; j < 17; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 256u * j), 0, 0);
    };
    auto fold = [&](uint32_t q, uint32_t(&u)[17]) {
        uint32_t a = 0;
#pragma unroll
        for (int j = 0; j < 17; ++j) a ^= u[j];
        a ^= __shfl_xor(a, 1);
        if (STORE == 1 && lane == 0) out[lo + q] = a;
        if (STORE == 2) {
            buf = (lane == (q & 63)) ? a : buf;
            if ((q & 63) == 63 || q + 1 == nq) out[lo + (q & ~63u) + lane] = buf;
        }
        if (STORE == 0 && a == 0x12345678u) out[0] = a;
    };
    load(0, ua);
    for (uint32_t q = 0; q < nq; q += 2) {
        if (q + 1 < nq) load(q + 1, ub);
        fold(q, ua);
        if (q + 1 >= nq) break;
        if (q + 2 < nq) load(q + 2, ua);
        fold(q + 1, ub);
    }
}

// E: four packets per wave (16 lanes each, the quad kernel's shape): a group's row is 64 B
// (one dword per lane), 65 rows per 4156-B packet; chunks of 13 rows double-buffered.
// X4 = 1: a group's row is 256 B (dwordx4 per lane), 17 rows.
template <int X4>
__global__ __launch_bounds__(1024) void quad_rows(const uint8_t *base, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave;
    const uint32_t chunk = ((kN + tw - 1) / tw + 3) & ~3u;
    const uint32_t lo = gw * chunk;
    if (lo >= kN) return;
    const uint32_t nq = kN - lo < chunk ? kN - lo : chunk;
    auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)lo * kL), 0, (int)(nq * kL), 0x00020000);
    uint32_t acc = 0;
    if (X4 == 0) {
        const int N = 1 + (kL - 4) / 4, R = (N + 15) / 16, k0 = N - 16 * R;  // R = 65
        constexpr int C = 13;
        uint32_t ua[C], ub[C];
        auto load = [&](uint32_t set, int c, uint32_t (&u)[C]) {
            const uint32_t vb = (set * 4 + grp) * kL + 4u * (uint32_t)(k0 - 1 + (int)col) + 64u * C * c;
#pragma unroll
            for (int j = 0; j < C; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 64u * j), 0, 2);
        };
        const uint32_t nsets = nq / 4, nch = nsets * 5;
        load(0, 0, ua);
        for (uint32_t t = 0; t < nch; t += 2) {
            if (t + 1 < nch) load((t + 1) / 5, (t + 1) % 5, ub);
#pragma unroll
            for (int j = 0; j < C; ++j) acc ^= ua[j];
            if (t + 1 >= nch) break;
            if (t + 2 < nch) load((t + 2) / 5, (t + 2) % 5, ua);
#pragma unroll
            for (int j = 0; j < C; ++j) acc ^= ub[j];
        }
    } else {
        const int N = 1 + (kL - 4) / 4, R = (N + 63) / 64, k0 = N - 64 * R;  // R = 17
        uint4 ua[17], ub[17];
        auto load = [&](uint32_t set, uint4 (&u)[17]) {
            const uint32_t vb = (set * 4 + grp) * kL + 4u * (uint32_t)(k0 - 1 + 4 * (int)col);
#pragma unroll
            for (int j = 0; j < 17; ++j) {
                auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vb + 256u * j), 0, 2);
                u[j] = *reinterpret_cast<uint4 *>(&v);
            }
        };
        const uint32_t nsets = nq / 4;
        load(0, ua);
        for (uint32_t t = 0; t < nsets; t += 2) {
            if (t + 1 < nsets) load(t + 1, ub);
#pragma unroll
            for (int j = 0; j < 17; ++j) acc ^= ua[j].x ^ ua[j].y ^ ua[j].z ^ ua[j].w;
            if (t + 1 >= nsets) break;
            if (t + 2 < nsets) load(t + 2, ua);
#pragma unroll
            for (int j = 0; j < 17; ++j) acc ^= ub[j].x ^ ub[j].y ^ ub[j].z ^ ub[j].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// G: P packets per wave (64/P lanes each, dword rows of 256/P bytes per packet), the packets
// of a set adjacent in memory; chunks of 16 rows double-buffered.  P = 2, 4, 8.
template <int P, int AUX = 2>
__global__ __launch_bounds__(1024) void multi_rows(const uint8_t *base, uint32_t *out) {
    constexpr int W = 64 / P;  // lanes (words) per packet row
    const uint32_t lane = threadIdx.x & 63, grp = lane / W, col = lane % W;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave;
    const uint32_t chunk = ((kN + tw - 1) / tw + P - 1) / P * P;
    const uint32_t lo = gw * chunk;
    if (lo >= kN) return;
    const uint32_t nq = kN - lo < chunk ? kN - lo : chunk;
    auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)lo * kL), 0, (int)(nq * kL), 0x00020000);
    const int N = 1 + (kL - 4) / 4, R = (N + W - 1) / W, k0 = N - W * R;
    constexpr int C = 16;
    const int nch = (R + C - 1) / C;
    uint32_t acc = 0, ua[C], ub[C];
    auto load = [&](uint32_t set, int ch, uint32_t (&u)[C]) {
        const uint32_t vb = (set * P + grp) * kL + 4u * (uint32_t)(k0 - 1 + (int)col) + 4u * W * C * ch;
#pragma unroll
        for (int j = 0; j < C; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 4u * W * j), 0, AUX);
    };
    const uint32_t nsets = nq / P, total = nsets * nch;
    load(0, 0, ua);
    for (uint32_t t = 0; t < total; t += 2) {
        if (t + 1 < total) load((t + 1) / nch, (t + 1) % nch, ub);
#pragma unroll
        for (int j = 0; j < C; ++j) acc ^= ua[j];
        if (t + 1 >= total) break;
        if (t + 2 < total) load((t + 2) / nch, (t + 2) % nch, ua);
#pragma unroll
        for (int j = 0; j < C; ++j) acc ^= ub[j];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// F: the packetizer's copy shape: packet t's payload (4096 B at src + 4096 t) is read in 256-B
// dword rows and written as a 4156-B wire packet (dst + 4156 t, 4-B aligned) in 256-B dword rows,
// rows end-aligned like the kernel (row 0 starts 200 B before the packet).  NT = load policy.
constexpr uint32_t kPay = 4096, kWire = 4156, kCopyN = 786432;
template <int NT, int STORE_NT>
__global__ __launch_bounds__(1024) void copy_rows(const uint8_t *src, uint8_t *dst) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave;
    const uint32_t chunk = ((kCopyN + tw - 1) / tw + 63) & ~63u;
    const uint32_t lo = gw * chunk;
    if (lo >= kCopyN) return;
    const uint32_t nq = kCopyN - lo < chunk ? kCopyN - lo : chunk;
    constexpr int R = 17;
    uint32_t ua[R], ub[R];
    auto load = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + (size_t)(lo + q) * kPay), 0, (int)kPay, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j)
            u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * (lane + 64u * j) - 256u), 0, NT ? 2 : 0);
    };
    auto store = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + (size_t)(lo + q) * kWire), 0, (int)(kWire - 4), 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j)
            __builtin_amdgcn_raw_buffer_store_b32(u[j], rs, (int)(4u * (lane + 64u * j) - 200u), 0, STORE_NT ? 2 : 0);
    };
    load(0, ua);
    for (uint32_t q = 0; q < nq; q += 2) {
        if (q + 1 < nq) load(q + 1, ub);
        store(q, ua);
        if (q + 1 >= nq) break;
        if (q + 2 < nq) load(q + 2, ua);
        store(q + 1, ub);
    }
}

template <class F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    int cus = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    const size_t bytes = (size_t)kN * kL;
    uint8_t *d;
    uint32_t *out;
    CK(hipMalloc(&d, bytes + 4096));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(d, 0x5a, bytes));
    const int reps = 10;
    auto report = [&](const char *name, float ms) {
        printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int wpc : {16, 32}) {
        int grid = cus * (wpc / 4);  // 256-thread blocks
        float ms = time_it([&] { flat_x4<<<grid, 256>>>((const uint4 *)d, bytes / 16, out); }, reps);
        char nm[64];
        snprintf(nm, sizeof nm, "A flat dwordx4 %d waves/CU", wpc);
        report(nm, ms);
    }
#define RUN_ROWS(K, P, NAME)                                                                     \
    {                                                                                            \
        float ms = time_it([&] { K<P><<<cus, 1024>>>(d, out); }, reps);                          \
        report(NAME, ms);                                                                        \
    }
    RUN_ROWS(rows_dword, 1, "B dword rows, 1 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_dword, 2, "B dword rows, 2 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_dword, 3, "B dword rows, 3 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_x4, 1, "C dwordx4 rows, 1 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_x4, 2, "C dwordx4 rows, 2 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_x4, 4, "C dwordx4 rows, 4 pkt/wave in flight, 16 waves/CU")
    RUN_ROWS(rows_chunk, 0, "D chunked dword rows, prefetch 1, no stores")
    RUN_ROWS(rows_chunk, 1, "D chunked dword rows, prefetch 1, per-packet 4-B store")
    RUN_ROWS(rows_chunk, 2, "D chunked dword rows, prefetch 1, coalesced store per 64")
    RUN_ROWS(rows_dword, 1, "B dword rows, 1 pkt/wave in flight, 16 waves/CU (again)")
    RUN_ROWS(quad_rows, 0, "E quad: 4 pkts/wave, 64-B dword group rows, 13-row chunks x2, nt")
    RUN_ROWS(quad_rows, 1, "E quad: 4 pkts/wave, 256-B dwordx4 group rows, 17-row sets x2, nt")
    RUN_ROWS(multi_rows, 2, "G 2 pkts/wave, 128-B dword rows per packet, 16-row chunks x2, nt")
    RUN_ROWS(multi_rows, 4, "G 4 pkts/wave, 64-B dword rows per packet, 16-row chunks x2, nt")
    RUN_ROWS(multi_rows, 8, "G 8 pkts/wave, 32-B dword rows per packet, 16-row chunks x2, nt")
    {
        float ms = time_it([&] { multi_rows<2, 0><<<cus, 1024>>>(d, out); }, reps);
        report("G 2 pkts/wave, default policy", ms);
        ms = time_it([&] { multi_rows<4, 0><<<cus, 1024>>>(d, out); }, reps);
        report("G 4 pkts/wave, default policy", ms);
        ms = time_it([&] { multi_rows<4, 1><<<cus, 1024>>>(d, out); }, reps);
        report("G 4 pkts/wave, glc (sc0)", ms);
        ms = time_it([&] { multi_rows<1, 2><<<cus, 1024>>>(d, out); }, reps);
        report("G 1 pkt/wave (same code), nt", ms);
        ms = time_it([&] { multi_rows<1, 0><<<cus, 1024>>>(d, out); }, reps);
        report("G 1 pkt/wave (same code), default", ms);
    }
    {
        uint8_t *wire;
        CK(hipMalloc(&wire, (size_t)kCopyN * kWire + 4096));
        auto copy_report = [&](const char *name, float ms) {
            const double b = (double)kCopyN * (kPay + kWire);
            printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GB/s (read+write)\": %.1f}\n", name, ms, b / (ms * 1e-3) / 1e9);
            fflush(stdout);
        };
        copy_report("F copy 4096-B payload -> 4156-B wire packets, 256-B dword rows, default",
                    time_it([&] { copy_rows<0, 0><<<cus, 1024>>>(d, wire); }, reps));
        copy_report("F copy ..., nt loads", time_it([&] { copy_rows<1, 0><<<cus, 1024>>>(d, wire); }, reps));
        copy_report("F copy ..., nt loads + nt stores", time_it([&] { copy_rows<1, 1><<<cus, 1024>>>(d, wire); }, reps));
        CK(hipFree(wire));
    }
    CK(hipFree(d));
    CK(hipFree(out));
    return 0;
}
