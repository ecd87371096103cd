// scripts/shortbench.hip — achievable HBM read bandwidth for SHORT packets (316 and 1084 bytes,
// the 256- and 1024-byte-MTU classes of C2) by access shape: P packets per wavefront, each lane
// loading 4 (dword) or 16 (dwordx4) bytes of a packet row, rows end-aligned to the packet like the
// kernels, three sets of P packets in flight per wave, cache policy default or nt.  The question:
// is the short-packet kernel's 4.3-4.8 TB/s the shape's ceiling or its own overhead?
// Each kernel XOR-folds what it reads (no dead-code removal); the results are not ICRCs.
// Build: hipcc --offload-arch=gfx950 -O3 -o shortbench shortbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr uint32_t kOOR = 0x80000000u;

// P packets per wave (W = 64 / P lanes each), X4: 16 bytes per lane per row, R rows per packet
// (row bytes RB = W * (X4 ? 16 : 4), R * RB >= L), AUX load policy (0 default, 2 nt).
// DEPTH: sets in flight while one is folded (3: two ahead, the default; 2: one ahead).  ST: result
// stores (the oct kernel stores a block's 64 results once per 8 sets): 1 = one store every 8 sets
// (uniform branch); 2 = a store every set, out of range except every 8th (no branch); 3 = four
// stores every 32 sets (branch); 4 = as 1 with the nt policy; 5 = as 2 with the nt policy;
// 6 = results held in a 16-register shift buffer (one entry per 8 sets), stored as a burst of 16
// when full and at the end; 7 = the same with a 4-register buffer (4 stores every 32 sets);
// 8 = the 16-register buffer stored only after the loop (no store in the loop body; results
// beyond 16 blocks per wave are dropped); 9 = the wave's chunk walked in passes of 16 blocks,
// each pass's loop drained before its 16 results are stored.
template <int P, int X4, int R, int AUX, int WORK = 0, int DEPTH = 3, int ST = 0>
__global__ __launch_bounds__(1024) void short_rows(const uint8_t *base, uint32_t L, uint32_t n, uint32_t *out) {
    constexpr int W = 64 / P;
    constexpr int B = X4 ? 16 : 4;
    constexpr int RB = W * B;
    constexpr int V = X4 ? 4 : 1;
    const uint32_t lane = threadIdx.x & 63, grp = lane / W, col = lane % W;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tw = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave;
    const uint32_t chunk = ((n + tw - 1) / tw + 63) & ~63u;
    const uint32_t lo = gw * chunk;
    if (lo >= n) return;
    const uint32_t nq = n - lo < chunk ? n - lo : chunk;
    const uint32_t nsets = (nq + P - 1) / P;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)lo * L), 0, (int)(nq * L), 0x00020000);
    uint32_t ua[R * V], ub[R * V], uc[R * V], acc = 0;
    auto load = [&](uint32_t set, uint32_t(&u)[R * V]) __attribute__((always_inline)) {
        const uint32_t q = set * P + grp;
        const int vb = (int)(q * L + L) - R * RB + (int)(col * B);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int o = vb + RB * j;
            const int oo = (set < nsets && o >= (int)(q * L)) ? o : (int)kOOR;
            if constexpr (X4) {
                auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, oo, 0, AUX);
                u[4 * j] = v[0];
                u[4 * j + 1] = v[1];
                u[4 * j + 2] = v[2];
                u[4 * j + 3] = v[3];
            } else {
                u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, oo, 0, AUX);
            }
        }
    };
    auto fold = [&](uint32_t(&u)[R * V]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < R * V; ++j) acc ^= u[j];
        // WORK dependent VALU ops per set (a stand-in for the CRC's per-set instruction count)
#pragma unroll
        for (int w = 0; w < WORK; ++w) acc = __builtin_amdgcn_perm(acc, acc + static_cast<uint32_t>(w), 0x05040302u + w);
    };
    const __amdgpu_buffer_rsrc_t rsout = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(n * 4u), 0x00020000);
    constexpr int NR = ST == 7 ? 4 : 16;
    uint32_t rb[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) rb[i] = 0;
    uint32_t nrb = 0, rb0 = 0;  // entries held; the block index of the oldest
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int o = (int)(4u * ((lo & ~63u) + 64u * (rb0 + i)) + 4u * lane);
            if (i >= NR - (int)nrb) __builtin_amdgcn_raw_buffer_store_b32(rb[i], rsout, o - 256 * (NR - (int)nrb), 0, 0);
        }
        rb0 += nrb;
        nrb = 0;
    };
    auto result = [&](uint32_t t) __attribute__((always_inline)) {  // after set t
        const int o = (int)(4u * ((lo + t * P) & ~63u) + 4u * lane);
        if constexpr (ST >= 6) {
            if ((t & 7u) == 7u) {
#pragma unroll
                for (int i = 0; i + 1 < NR; ++i) rb[i] = rb[i + 1];
                rb[NR - 1] = acc;
                nrb += nrb < NR ? 1u : 0u;
                if (ST != 8 && ST != 9 && nrb == NR) flush();
            }
        }
        if constexpr (ST == 1 || ST == 4) {
            if ((t & 7u) == 7u) __builtin_amdgcn_raw_buffer_store_b32(acc, rsout, o, 0, ST == 4 ? 2 : 0);
        } else if constexpr (ST == 2 || ST == 5) {
            __builtin_amdgcn_raw_buffer_store_b32(acc, rsout, (t & 7u) == 7u ? o : (int)kOOR, 0, ST == 5 ? 2 : 0);
        } else if constexpr (ST == 3) {
            if ((t & 31u) == 31u) {
#pragma unroll
                for (int k = 0; k < 4; ++k) __builtin_amdgcn_raw_buffer_store_b32(acc + k, rsout, o - 256 * 8 * k, 0, 0);
            }
        }
    };
    if constexpr (ST == 9) {  // passes of 128 sets (16 blocks), drained, then stored
        for (uint32_t t0 = 0; t0 < nsets; t0 += 128) {
            const uint32_t t1 = nsets - t0 < 128 ? nsets : t0 + 128;
            load(t0, ua);
            load(t0 + 1, ub);
            for (uint32_t t = t0; t < t1; t += 3) {
                load(t + 2 < t1 ? t + 2 : nsets, uc);
                fold(ua);
                result(t);
                load(t + 3 < t1 ? t + 3 : nsets, ua);
                fold(ub);
                result(t + 1);
                load(t + 4 < t1 ? t + 4 : nsets, ub);
                fold(uc);
                result(t + 2);
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the pass's loads are in
            if (nrb) flush();
        }
    } else if constexpr (DEPTH == 3) {
        load(0, ua);
        load(1, ub);
        for (uint32_t t = 0; t < nsets; t += 3) {
            load(t + 2, uc);
            fold(ua);
            result(t);
            load(t + 3, ua);
            fold(ub);
            result(t + 1);
            load(t + 4, ub);
            fold(uc);
            result(t + 2);
        }
    } else {
        load(0, ua);
        for (uint32_t t = 0; t < nsets; t += 2) {
            load(t + 1, ub);
            fold(ua);
            result(t);
            load(t + 2, ua);
            fold(ub);
            result(t + 1);
        }
    }
    if constexpr (ST >= 6 && ST != 9) {
        if (nrb) flush();
    }
    if (acc == 0x12345678u) out[0] = acc;
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

int main(int argc, char **argv) {
    const bool only_store = argc > 1 && argv[1][0] == 's';
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint8_t *d;
    uint32_t *out;
    const size_t cap = (size_t)5400 << 20;
    CK(hipMalloc(&d, cap));
    CK(hipMalloc(&out, (size_t)4 << 24));
    CK(hipMemset(d, 0x5a, cap));
    const int reps = 20;
    auto run = [&](const char *name, uint32_t L, uint32_t n, auto kern) {
        float ms = time_it([&] { kern<<<cus, 1024>>>(d, L, n, out); }, reps);
        const double bytes = (double)L * n;
        printf("{\"L\": %u, \"shape\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f}\n", L, name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int round = 0; round < 2; ++round) {
        const uint32_t n316 = 4u << 20, n1084 = 1u << 20;
        if (only_store) {  // the result-store shapes only
            run("8 pkts/wave, 32-B dword rows, default", 316, n316, short_rows<8, 0, 10, 0>);
            run("8 pkts/wave, 32-B dword rows, default, store / 8 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 1>);
            run("8 pkts/wave, 32-B dword rows, default, store every set (OOR but 1 in 8)", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 2>);
            run("8 pkts/wave, 32-B dword rows, default, 4 stores / 32 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 3>);
            run("8 pkts/wave, 32-B dword rows, default, nt store / 8 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 4>);
            run("8 pkts/wave, 32-B dword rows, default, nt store every set (OOR but 1 in 8)", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 5>);
            run("8 pkts/wave, 32-B dword rows, default, 16-register result buffer", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 6>);
            run("8 pkts/wave, 32-B dword rows, default, 4-register result buffer", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 7>);
            run("8 pkts/wave, 32-B dword rows, default, 16-register buffer stored after the loop", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 8>);
            run("8 pkts/wave, 32-B dword rows, default, passes of 16 blocks, stored after each", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 9>);
            run("8 pkts/wave, 32-B dword rows, default, passes of 16 blocks, stored after each", 316, 4 * n316, short_rows<8, 0, 10, 0, 0, 3, 9>);
            run("8 pkts/wave, 32-B dword rows, default, store / 8 sets", 316, 4 * n316, short_rows<8, 0, 10, 0, 0, 3, 1>);
            run("8 pkts/wave, 32-B dword rows, default", 316, 4 * n316, short_rows<8, 0, 10, 0>);
            run("8 pkts/wave, 32-B dword rows, default", 1084, n1084, short_rows<8, 0, 34, 0>);
            run("8 pkts/wave, 32-B dword rows, default, store / 8 sets", 1084, n1084, short_rows<8, 0, 34, 0, 0, 3, 1>);
            run("8 pkts/wave, 32-B dword rows, default, 16-register result buffer", 1084, n1084, short_rows<8, 0, 34, 0, 0, 3, 6>);
            run("8 pkts/wave, 32-B dword rows, default, 16-register buffer stored after the loop", 1084, n1084, short_rows<8, 0, 34, 0, 0, 3, 8>);
            run("8 pkts/wave, 32-B dword rows, default, passes of 16 blocks, stored after each", 1084, n1084, short_rows<8, 0, 34, 0, 0, 3, 9>);
            continue;
        }
        run("1 pkt/wave, 256-B dword rows, default", 316, n316, short_rows<1, 0, 2, 0>);
        run("1 pkt/wave, 256-B dword rows, nt", 316, n316, short_rows<1, 0, 2, 2>);
        run("2 pkts/wave, 128-B dword rows, default", 316, n316, short_rows<2, 0, 3, 0>);
        run("4 pkts/wave, 64-B dword rows, default", 316, n316, short_rows<4, 0, 5, 0>);
        run("8 pkts/wave, 32-B dword rows, default", 316, n316, short_rows<8, 0, 10, 0>);
        run("8 pkts/wave, 32-B dword rows, nt", 316, n316, short_rows<8, 0, 10, 2>);
        run("4 pkts/wave, 256-B dwordx4 rows, default", 316, n316, short_rows<4, 1, 2, 0>);
        run("8 pkts/wave, 128-B dwordx4 rows, default", 316, n316, short_rows<8, 1, 3, 0>);
        run("8 pkts/wave, 128-B dwordx4 rows, nt", 316, n316, short_rows<8, 1, 3, 2>);
        run("16 pkts/wave, 64-B dwordx4 rows, default", 316, n316, short_rows<16, 1, 5, 0>);
        run("16 pkts/wave, 16-B dword rows, default", 316, n316, short_rows<16, 0, 20, 0>);
        run("16 pkts/wave, 16-B dword rows, nt", 316, n316, short_rows<16, 0, 20, 2>);
        run("8 pkts/wave, 32-B dword rows, default, +50 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 50>);
        run("8 pkts/wave, 32-B dword rows, default, +100 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 100>);
        run("8 pkts/wave, 32-B dword rows, default, +150 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 150>);
        run("8 pkts/wave, 32-B dword rows, default, +200 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 200>);
        run("8 pkts/wave, 32-B dword rows, default, store every set (OOR but 1 in 8)", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 2>);
        run("8 pkts/wave, 32-B dword rows, default, 4 stores / 32 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 3>);
        run("8 pkts/wave, 32-B dword rows, default, nt store / 8 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 4>);
        run("8 pkts/wave, 32-B dword rows, default, nt store every set (OOR but 1 in 8)", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 5>);
        run("8 pkts/wave, 32-B dword rows, default, depth 2", 316, n316, short_rows<8, 0, 10, 0, 0, 2>);
        run("8 pkts/wave, 32-B dword rows, default, store / 8 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 3, 1>);
        run("8 pkts/wave, 32-B dword rows, default, depth 2, store / 8 sets", 316, n316, short_rows<8, 0, 10, 0, 0, 2, 1>);
        run("8 pkts/wave, 32-B dword rows, default, depth 2, +100 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 100, 2>);
        run("8 pkts/wave, 32-B dword rows, default, depth 2, store / 8 sets, +100 VALU/set", 316, n316, short_rows<8, 0, 10, 0, 100, 2, 1>);
        run("16 pkts/wave, 16-B dword rows, default, +50 VALU/set", 316, n316, short_rows<16, 0, 20, 0, 50>);
        run("16 pkts/wave, 16-B dword rows, default, +100 VALU/set", 316, n316, short_rows<16, 0, 20, 0, 100>);
        run("1 pkt/wave, 256-B dword rows, default", 1084, n1084, short_rows<1, 0, 5, 0>);
        run("8 pkts/wave, 32-B dword rows, default", 1084, n1084, short_rows<8, 0, 34, 0>);
        run("16 pkts/wave, 16-B dword rows, default", 1084, n1084, short_rows<16, 0, 68, 0>);
        run("8 pkts/wave, 128-B dwordx4 rows, default", 1084, n1084, short_rows<8, 1, 9, 0>);
        run("4 pkts/wave, 256-B dwordx4 rows, default", 1084, n1084, short_rows<4, 1, 5, 0>);
    }
    CK(hipFree(d));
    CK(hipFree(out));
    return 0;
}
