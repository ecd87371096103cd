// scripts/trailerbench.hip — what a per-packet ICRC trailer store costs on the C1 access shape
// (1 Mi x 4156-B packets, stride 4156, wave-per-packet 256-B dword rows, one packet prefetched),
// by store shape.  PacketWriter::write stores the trailer (packet_processor.rs:263) and
// is_icrc_valid zeroes it (350); the question is whether a 4-byte write into a line of its own
// is what costs, and whether writing the aligned 32 / 64 / 128-byte piece around it is cheaper.
// Stored values are arbitrary (this measures traffic shape, not results).
// Build: hipcc --offload-arch=gfx950 -O3 -o trailerbench trailerbench.hip
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

constexpr uint32_t kL = 4156;
constexpr uint32_t kN = 1u << 20;
constexpr uint32_t kOOR = 0x80000000u;

// SHAPE: 0 none; 1 lane 0 plain 4-B store in a branch; 2 4-B buffer store, every lane issues,
// lanes != 0 out of range; 3 / 4 / 5 the aligned 32 / 64 / 128-B piece holding the trailer
// (8 / 16 / 32 lanes); 7 the trailers of a 64-packet block stored together at its end, one
// scattered store instruction (lane q -> packet q's trailer); AUX = cache policy bits of the
// buffer store (0 default, 2 nt); LAUX = row-load policy (2 nt, 0 default).
template <int SHAPE, int AUX, int LAUX = 2, int LLAST = -1>
__global__ __launch_bounds__(1024) void rows_trailer(uint8_t *base, uint32_t *out) {
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
    // one descriptor over the wave's whole chunk (stores reach into the next packet)
    const auto whole = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)lo * kL), 0, (int)(nq * kL), 0x00020000);
    auto load = [&](uint32_t q, uint32_t (&u)[17]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)(lo + q) * kL), 0, (int)(kL - 4), 0x00020000);
#pragma unroll
        for (int j = 0; j < 16; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 256u * j), 0, LAUX);
        u[16] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(vb + 256u * 16), 0, LLAST >= 0 ? LLAST : LAUX);
    };
    auto fold = [&](uint32_t q, uint32_t (&u)[17]) {
        uint32_t a = 0;
#pragma unroll
        for (int j = 0; j < 17; ++j) a ^= u[j];
        a ^= __shfl_xor(a, 1);
        const uint32_t t = q * kL + kL - 4;  // trailer offset in the chunk
        if constexpr (SHAPE == 1) {
            if (lane == 0) *reinterpret_cast<uint32_t *>(base + (size_t)lo * kL + t) = a;
        } else if constexpr (SHAPE == 2) {
            __builtin_amdgcn_raw_buffer_store_b32(a, whole, (int)(lane == 0 ? t : kOOR), 0, AUX);
        } else if constexpr (SHAPE >= 3) {
            constexpr uint32_t G = SHAPE == 3 ? 32u : SHAPE == 4 ? 64u : 128u;
            const uint32_t c = t & ~(G - 1u);
            __builtin_amdgcn_raw_buffer_store_b32(a, whole, (int)(lane < G / 4 ? c + 4u * lane : kOOR), 0, AUX);
        }
        buf = (lane == (q & 63)) ? a : buf;
        if ((q & 63) == 63 || q + 1 == nq) {
            out[lo + (q & ~63u) + lane] = buf;
            if constexpr (SHAPE == 7) {
                const uint32_t qq = (q & ~63u) + lane;
                __builtin_amdgcn_raw_buffer_store_b32(buf, whole, (int)(qq < nq ? qq * kL + kL - 4 : kOOR), 0, AUX);
            }
        }
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

// Random fill (HBM power depends on the bits toggled; the bench packets are random too).
__global__ void fill_random(uint32_t *p, size_t nw) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = static_cast<uint32_t>(z ^ (z >> 31));
    }
}

// Separate pass: one thread per packet, a 4-B store at its trailer.
__global__ void trailer_pass(uint8_t *base, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *reinterpret_cast<uint32_t *>(base + (size_t)i * kL + kL - 4) = i;
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
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const size_t bytes = (size_t)kN * kL;
    uint8_t *d;
    uint32_t *out;
    CK(hipMalloc(&d, bytes + 4096));
    CK(hipMalloc(&out, (size_t)kN * 4 + 4096));
    fill_random<<<4096, 256>>>(reinterpret_cast<uint32_t *>(d), bytes / 4);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    auto report = [&](const char *name, float ms) {
        printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int round = 0; round < 1; ++round) {
#define RUN(S, A, NAME) report(NAME, time_it([&] { rows_trailer<S, A><<<cus, 1024>>>(d, out); }, reps))
        RUN(0, 0, "T0 rows, no trailer store");
        report("T8 default-policy loads + 4-B buffer store",
               time_it([&] { rows_trailer<2, 0, 0><<<cus, 1024>>>(d, out); }, reps));
        report("T9 nt loads but the trailer's row default policy + 4-B buffer store",
               time_it([&] { rows_trailer<2, 0, 2, 0><<<cus, 1024>>>(d, out); }, reps));
        report("T10 rows (nt, no store) then the separate trailer pass, both timed (cold trailer lines)",
               time_it([&] {
                   rows_trailer<0, 0><<<cus, 1024>>>(d, out);
                   trailer_pass<<<(kN + 255) / 256, 256>>>(d, kN);
               }, reps));
        report("T0d rows, no trailer store, default-policy loads",
               time_it([&] { rows_trailer<0, 0, 0><<<cus, 1024>>>(d, out); }, reps));
        RUN(7, 0, "T7 trailers of 64 packets in one scattered store at the block end");
        RUN(7, 2, "T7nt the same, nt");
        RUN(2, 1, "T2sc0 + 4-B buffer store, sc0");
        RUN(2, 16, "T2sc1 + 4-B buffer store, sc1 (write-through)");
        RUN(2, 17, "T2sc01 + 4-B buffer store, sc0 sc1");
        RUN(2, 18, "T2ntsc1 + 4-B buffer store, nt sc1");
        RUN(5, 16, "T5sc1 + aligned 128-B line, sc1");
        RUN(5, 17, "T5sc01 + aligned 128-B line, sc0 sc1");
        RUN(1, 0, "T1 + lane-0 4-B store (branch)");
        RUN(2, 0, "T2 + 4-B buffer store, every lane issues (OOR lanes)");
        RUN(2, 2, "T2nt + 4-B buffer store, nt");
        RUN(3, 0, "T3 + aligned 32-B piece");
        RUN(4, 0, "T4 + aligned 64-B piece");
        RUN(5, 0, "T5 + aligned 128-B line");
        RUN(4, 2, "T4nt + aligned 64-B piece, nt");
        RUN(5, 2, "T5nt + aligned 128-B line, nt");
#undef RUN
        report("T6 separate pass: thread per packet 4-B store",
               time_it([&] { trailer_pass<<<kN / 256, 256>>>(d, kN); }, reps));
    }
    CK(hipFree(d));
    CK(hipFree(out));
    return 0;
}
