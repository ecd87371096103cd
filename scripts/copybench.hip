// copybench.hip — the ceiling of the send packetizer's copy shape (measurement tool, not product
// code).  786 432 payloads of 4096 B (contiguous) become 4156-B wire packets (payload at packet
// offset 56, packets 4156 B apart, so the payload lands 4-B aligned).  Forms:
//   rows_dword<W>   256-B dword rows (the packetizer's shape), W waves per CU
//   rows_x4<W>      1-KiB dwordx4 rows (16 B per lane), W waves per CU
//   flat_x4         contiguous float4 grid-stride copy of the same byte count
//   hipMemcpy       device-to-device copy of the same byte count
// GB/s counts read + write bytes.  Output: one JSON line per form.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

constexpr uint32_t kPay = 4096, kWire = 4156, kN = 786432, kHdr = 56;

// one wave per packet, contiguous chunks, the next packet's rows loaded while the current one is
// stored (a two-slot register ring)
// LSHIFT: the payload loads start LSHIFT bytes before each 256-B source row (the packetizer's end-
// aligned rows put its loads 4 (k0 - 1 - hw) = -252 mod 256 bytes off the payload's lines, so every
// 256-B row load touches 5 lines instead of 4); the bytes outside the payload read as 0 (range check)
// WIRE / HDR: the wire slot stride and the payload's offset in it (4156 / 56: the packetizer's
// packets; 4160 / 0 with LSHIFT 56: every row store line-aligned, every row load 56 B off its lines)
template <int POLICY_ST, bool IL = false, int LSHIFT = 0, uint32_t WIRE = kWire, uint32_t HDR = kHdr>
__global__ __launch_bounds__(1024) void rows_dword(const uint8_t *src, uint8_t *dst, uint32_t waves) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // IL: packet q of the wave is gw + q * waves (the grid sweeps memory together); else the
    // wave owns the contiguous range [gw * chunk, ...)
    const uint32_t chunk = (kN + waves - 1) / waves;
    const uint32_t lo = IL ? 0u : gw * chunk;
    if (gw * chunk >= kN) return;
    const uint32_t nq = IL ? (kN - gw + waves - 1) / waves : (kN - lo < chunk ? kN - lo : chunk);
    auto pkt = [&](uint32_t q) -> size_t { return IL ? (size_t)gw + (size_t)q * waves : (size_t)(lo + q); };
    constexpr int R = 16;
    uint32_t ua[R], ub[R];
    auto load = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + pkt(q) * kPay), 0, (int)kPay, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int o = (int)(4u * lane + 256u * j) - LSHIFT;
            u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, o >= 0 ? o : (int)0x80000000, 0, 0);
        }
    };
    auto store = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + pkt(q) * WIRE), 0, (int)WIRE, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j)
            __builtin_amdgcn_raw_buffer_store_b32(u[j], rs, (int)(HDR + 4u * lane + 256u * j) - (HDR == 0 ? 0 : LSHIFT), 0, POLICY_ST);
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

template <int POLICY_ST, bool IL = false>
__global__ __launch_bounds__(1024) void rows_x4(const uint8_t *src, uint8_t *dst, uint32_t waves) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // IL: packet q of the wave is gw + q * waves (the grid sweeps memory together); else the
    // wave owns the contiguous range [gw * chunk, ...)
    const uint32_t chunk = (kN + waves - 1) / waves;
    const uint32_t lo = IL ? 0u : gw * chunk;
    if (gw * chunk >= kN) return;
    const uint32_t nq = IL ? (kN - gw + waves - 1) / waves : (kN - lo < chunk ? kN - lo : chunk);
    auto pkt = [&](uint32_t q) -> size_t { return IL ? (size_t)gw + (size_t)q * waves : (size_t)(lo + q); };
    constexpr int R = 4;
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    v4 ua[R], ub[R];
    auto load = [&](uint32_t q, v4 (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + pkt(q) * kPay), 0, (int)kPay, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * lane + 1024u * j), 0, 0);
    };
    auto store = [&](uint32_t q, v4 (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + pkt(q) * kWire), 0, (int)kWire, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(u[j], rs, (int)(kHdr + 16u * lane + 1024u * j), 0, POLICY_ST);
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

// the C1 read shape alone: 1 Mi x 4156-B packets, 17 dword rows per packet, nt loads
template <bool IL>
__global__ __launch_bounds__(1024) void read_rows(const uint8_t *src, uint32_t *out, uint32_t waves, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t chunk = (n + waves - 1) / waves;
    if (gw * chunk >= n) return;
    const uint32_t nq = IL ? (n - gw + waves - 1) / waves : (n - gw * chunk < chunk ? n - gw * chunk : chunk);
    auto pkt = [&](uint32_t q) -> size_t { return IL ? (size_t)gw + (size_t)q * waves : (size_t)gw * chunk + q; };
    constexpr int R = 17;
    uint32_t ua[R], ub[R], acc = 0;
    auto load = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + pkt(q) * 4156u), 0, 4152, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * lane + 256u * j) - 200, 0, 2);
    };
    load(0, ua);
    for (uint32_t q = 0; q < nq; q += 2) {
        if (q + 1 < nq) load(q + 1, ub);
#pragma unroll
        for (int j = 0; j < R; ++j) acc ^= ua[j];
        if (q + 1 >= nq) break;
        if (q + 2 < nq) load(q + 2, ua);
#pragma unroll
        for (int j = 0; j < R; ++j) acc ^= ub[j];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// COPY_READ=1 forms (round 6): the C1 read set (1 Mi x 4156-B packets, 4152 B read each) with
// wider lanes: E = 8 / 16 bytes per lane (512-B / 1-KiB rows, 9 / 5 row loads per packet, the last
// partial), one wave per packet, two packets in flight; and a flat grid-stride 16-B read of the same
// bytes (XOR fold, stored only on a magic value)
// SHIFT: the loads start SHIFT bytes before the packet (end-aligned rows of a kernel: 968 B for x4
// rows of 4156-B packets, 456 for x2); lanes wholly before the packet read out of range (0)
template <int E, int SHIFT = 0>
__global__ __launch_bounds__(1024) void read_rows_w(const uint8_t *src, uint32_t *out, uint32_t waves, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t chunk = (n + waves - 1) / waves;
    if (gw * chunk >= n) return;
    const uint32_t nq = n - gw * chunk < chunk ? n - gw * chunk : chunk;
    constexpr int R = (4152 + SHIFT + 64 * E - 1) / (64 * E);
    typedef uint32_t vv __attribute__((ext_vector_type(E / 4)));
    vv ua[R], ub[R];
    uint32_t acc = 0;
    auto load = [&](uint32_t q, vv (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + ((size_t)gw * chunk + q) * 4156u), 0, 4152, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int o0 = (int)(E * lane + 64 * E * j) - SHIFT;
            const int o = o0 >= 0 ? o0 : (int)0x80000000;
            if constexpr (E == 16) u[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 2);
            else u[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 2);
        }
    };
    auto fold = [&](vv (&u)[R]) {
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
            for (int k = 0; k < E / 4; ++k) acc ^= u[j][k];
    };
    load(0, ua);
    for (uint32_t q = 0; q < nq; q += 2) {
        if (q + 1 < nq) load(q + 1, ub);
        fold(ua);
        if (q + 1 >= nq) break;
        if (q + 2 < nq) load(q + 2, ua);
        fold(ub);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void flat_read_x4(const uint4 *s, size_t n16, uint32_t *out) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 *p = reinterpret_cast<const v4 *>(s);
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const v4 v = __builtin_nontemporal_load(p + i);
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// COPY_RAND=1: the source filled with splitmix64 bytes instead of a constant
__global__ void fill_rand(uint64_t *p, size_t n8) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ void flat_x4(const uint4 *s, uint4 *d, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// COPY_ORDER=1 forms (round 6, what separates the packetizer's shape from flat_x4):
// flat_slots<E>: the flat grid-stride order, but each E-byte element lands in the packetizer's
// wire slots (payload element c of packet c / (kPay / E) at slot offset kHdr + ...): the flat
// copy's order with the packetizer's layout
template <int E, uint32_t WIRE = kWire, uint32_t HDR = kHdr>
__global__ void flat_slots(const uint8_t *src, uint8_t *dst) {
    constexpr uint32_t per = kPay / E;
    const size_t n = (size_t)kN * per;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t q = i / per, k = i % per;
        uint8_t *d = dst + q * WIRE + HDR + k * E;
        const uint8_t *s = src + i * E;
        if constexpr (E == 16) {
            typedef uint32_t v4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<v4 *>(d) = *reinterpret_cast<const v4 *>(s);
        } else {
            *reinterpret_cast<uint32_t *>(d) = *reinterpret_cast<const uint32_t *>(s);
        }
    }
}

// The packetizer's WHOLE write set (header 56 B + payload + 4-B trailer: contiguous 4156-B packets,
// every byte written) without the CRC:
// rows_full: one wave per packet (contiguous chunks, a two-packet register ring), 17 dword rows of
// 256 B from the packet's first byte; flat_out: the flat grid-stride order over the output stream
// (16-B aligned stores, every output line whole), each dword from the payload or a constant
// (IL: packet q of the wave is gw + q * waves, the grid's order; SAUX: the stores' cache policy)
template <bool IL = false, int SAUX = 0>
__global__ __launch_bounds__(1024) void rows_full(const uint8_t *src, uint8_t *dst, uint32_t waves) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t chunk = (kN + waves - 1) / waves;
    if (gw * chunk >= kN) return;
    const uint32_t lo = IL ? gw : gw * chunk;
    const uint32_t nq = IL ? (kN - gw + waves - 1) / waves : (kN - lo < chunk ? kN - lo : chunk);
    auto pkt = [&](uint32_t q) -> size_t { return IL ? (size_t)gw + (size_t)q * waves : (size_t)(lo + q); };
    constexpr int R = 17;
    uint32_t ua[R], ub[R];
    auto load = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + pkt(q) * kPay), 0, (int)kPay, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int o = (int)(4u * lane + 256u * j) - (int)kHdr;
            u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, o >= 0 ? o : (int)0x80000000, 0, 0);
        }
    };
    auto store = [&](uint32_t q, uint32_t (&u)[R]) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + pkt(q) * kWire), 0, (int)kWire, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t o = 4u * lane + 256u * j;
            const uint32_t v = o < kHdr ? 0x11223344u : o >= kHdr + kPay ? 0xA5A5A5A5u : u[j];
            __builtin_amdgcn_raw_buffer_store_b32(v, rs, (int)o, 0, SAUX);
        }
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

// rows_wg: the whole packet written, one WORKGROUP per packet (wave w takes row w of the 17, wave 0
// also row 16), workgroups walking packets in the grid's order (g, g + G, ...): all rows of a
// packet leave together, and the grid writes a window of G packets at a time.  The next packet's
// row is loaded before the current one is stored.
__global__ __launch_bounds__(1024) void rows_wg(const uint8_t *src, uint8_t *dst) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t o0 = 4u * lane + 256u * w, o1 = 4u * lane + 256u * 16u;  // row w; row 16 (wave 0)
    auto ld = [&](uint32_t q, uint32_t o) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + (size_t)q * kPay), 0, (int)kPay, 0x00020000);
        const int s = (int)o - (int)kHdr;
        return __builtin_amdgcn_raw_buffer_load_b32(rs, s >= 0 ? s : (int)0x80000000, 0, 0);
    };
    auto st = [&](uint32_t q, uint32_t o, uint32_t u) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + (size_t)q * kWire), 0, (int)kWire, 0x00020000);
        const uint32_t v = o < kHdr ? 0x11223344u : o >= kHdr + kPay ? 0xA5A5A5A5u : u;
        __builtin_amdgcn_raw_buffer_store_b32(v, rs, (int)o, 0, 0);
    };
    uint32_t q = blockIdx.x;
    if (q >= kN) return;
    uint32_t a0 = ld(q, o0), a1 = w == 0 ? ld(q, o1) : 0u;
    for (;;) {
        const uint32_t qn = q + gridDim.x;
        uint32_t b0 = 0, b1 = 0;
        if (qn < kN) {
            b0 = ld(qn, o0);
            if (w == 0) b1 = ld(qn, o1);
        }
        st(q, o0, a0);
        if (w == 0) st(q, o1, a1);
        if (qn >= kN) break;
        q = qn;
        a0 = b0;
        a1 = b1;
    }
}

__global__ void flat_out(const uint32_t *src, uint4 *dst) {
    const uint32_t n16 = kN * (kWire / 4) / 4;  // 16-B output chunks (kWire is a multiple of 4, kN of 4)
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += gridDim.x * blockDim.x) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = 16u * c + 4u * k;  // < 2^32: 786432 x 4156 B
            const uint32_t q = p / kWire, w = p - q * kWire;
            v[k] = w < kHdr ? 0x11223344u : w >= kHdr + kPay ? 0xA5A5A5A5u : src[(q * kPay + w - kHdr) / 4u];
        }
        dst[c] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// quarter_rows<QR>: one wave per QR 256-B dword rows of a packet (QR = 4: a 1 KiB quarter, four
// waves per packet), units walked in the grid's order (unit g + k * waves), each unit's loads then
// its stores, two units in flight per wave
template <int QR>
__global__ __launch_bounds__(1024) void quarter_rows(const uint8_t *src, uint8_t *dst, uint32_t waves) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint32_t per = 16 / QR;  // units per packet
    const uint32_t units = kN * per;
    const uint32_t nq = gw < units ? (units - gw + waves - 1) / waves : 0u;
    uint32_t ua[QR], ub[QR];
    auto load = [&](uint32_t q, uint32_t (&u)[QR]) {
        const uint32_t g = gw + q * waves;
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + (size_t)(g / per) * kPay), 0, (int)kPay, 0x00020000);
#pragma unroll
        for (int j = 0; j < QR; ++j) u[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * lane + 256u * (QR * (g % per) + j)), 0, 0);
    };
    auto store = [&](uint32_t q, uint32_t (&u)[QR]) {
        const uint32_t g = gw + q * waves;
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + (size_t)(g / per) * kWire), 0, (int)kWire, 0x00020000);
#pragma unroll
        for (int j = 0; j < QR; ++j)
            __builtin_amdgcn_raw_buffer_store_b32(u[j], rs, (int)(kHdr + 4u * lane + 256u * (QR * (g % per) + j)), 0, 0);
    };
    if (nq == 0) return;
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
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint8_t *src, *dst;
    const size_t src_bytes = (size_t)1048576 * 4156 + 4096;  // >= kN * kPay; the C1 read shape reads 1 Mi x 4156 B
    CK(hipMalloc(&src, src_bytes));
    CK(hipMalloc(&dst, (size_t)kN * 4160 + 4096));
    CK(hipMemset(src, 0x5a, src_bytes));
    const bool rnd = getenv("COPY_RAND") && atoi(getenv("COPY_RAND")) == 1;
    if (rnd) {
        fill_rand<<<cus * 4, 256>>>((uint64_t *)src, src_bytes / 8);
        CK(hipDeviceSynchronize());
    }
    fprintf(stderr, "source: %s\n", rnd ? "splitmix64 bytes" : "constant 0x5a");
    CK(hipMemset(dst, 0, (size_t)kN * kWire));
    const int reps = 10;
    const double wire_bytes = (double)kN * (kPay + kPay);  // payload read + payload written
    auto report = [&](const char *name, float ms) {
        printf("{\"form\": \"%s\", \"ms\": %.4f, \"GB/s (read+write)\": %.1f}\n", name, ms, wire_bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    if (getenv("COPY_READ")) {  // the C1 read set with wider lanes, and a flat read of the same bytes
        const uint32_t n = 1048576u;
        const double rb = (double)n * 4152;
        uint32_t *o = (uint32_t *)dst;
        auto rep_r = [&](const char *name, float ms) {
            printf("{\"form\": \"%s\", \"ms\": %.4f, \"GB/s (read)\": %.1f}\n", name, ms, rb / (ms * 1e-3) / 1e9);
            fflush(stdout);
        };
        for (int rep = 0; rep < 3; ++rep) {
            rep_r("read C1 shape: dword rows (256 B), a wave per packet", time_it([&] { read_rows<false><<<cus, 1024>>>(src, o, cus * 16, n); }, reps));
            rep_r("read C1 set: dwordx2 rows (512 B), a wave per packet", time_it([&] { read_rows_w<8><<<cus, 1024>>>(src, o, cus * 16, n); }, reps));
            rep_r("read C1 set: dwordx4 rows (1 KiB), a wave per packet", time_it([&] { read_rows_w<16><<<cus, 1024>>>(src, o, cus * 16, n); }, reps));
            rep_r("read C1 set: dwordx4 rows end-aligned (968 B shift, 8 B off 16)", time_it([&] { read_rows_w<16, 968><<<cus, 1024>>>(src, o, cus * 16, n); }, reps));
            rep_r("read C1 set: dwordx2 rows end-aligned (456 B shift)", time_it([&] { read_rows_w<8, 456><<<cus, 1024>>>(src, o, cus * 16, n); }, reps));
            rep_r("flat grid-stride 16-B nt reads of the same byte count (256-thread groups, 16 waves/CU)",
                  time_it([&] { flat_read_x4<<<cus * 4, 256>>>((const uint4 *)src, (size_t)rb / 16, o); }, reps));
            rep_r("flat grid-stride 16-B nt reads of the same byte count (32 waves/CU)",
                  time_it([&] { flat_read_x4<<<cus * 8, 256>>>((const uint4 *)src, (size_t)rb / 16, o); }, reps));
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (getenv("COPY_ORDER")) {  // which part of the access order separates the packetizer from flat_x4
        const size_t n16 = (size_t)kN * kPay / 16;
        for (int rep = 0; rep < 2; ++rep) {
            report("flat_x4 contiguous 16 waves/CU (256-thread groups)",
                   time_it([&] { flat_x4<<<cus * 4, 256>>>((const uint4 *)src, (uint4 *)dst, n16); }, reps));
            report("flat_x4 contiguous 16 waves/CU (1024-thread groups)",
                   time_it([&] { flat_x4<<<cus, 1024>>>((const uint4 *)src, (uint4 *)dst, n16); }, reps));
            report("flat_slots x4: flat order, wire slots (256-thread groups)",
                   time_it([&] { flat_slots<16><<<cus * 4, 256>>>(src, dst); }, reps));
            report("flat_slots x4: flat order, slots of 4160 B, payload at 0 (line-aligned, a line skipped per slot)",
                   time_it([&] { flat_slots<16, 4160, 0><<<cus * 4, 256>>>(src, dst); }, reps));
            report("flat_slots x4: flat order, slots of 4096 B (contiguous, the slot index math)",
                   time_it([&] { flat_slots<16, 4096, 0><<<cus * 4, 256>>>(src, dst); }, reps));
            report("flat_slots x4: flat order, slots of 4160 B, payload at 56 (stores 8 B off their lines)",
                   time_it([&] { flat_slots<16, 4160, 56><<<cus * 4, 256>>>(src, dst); }, reps));
            report("flat_slots x4: flat order, slots of 4156 B, payload at 0 (4 B steps, no header gap)",
                   time_it([&] { flat_slots<16, 4156, 0><<<cus * 4, 256>>>(src, dst); }, reps));
            report("rows_dword: a wave per packet, slots of 4096 B (contiguous)",
                   time_it([&] { rows_dword<0, false, 0, 4096, 0><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("rows_x4: a wave per packet (1 KiB rows), slots of 4156 B at 56, grid order",
                   time_it([&] { rows_x4<0, true><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("quarter_rows 4: a wave per 1 KiB quarter, grid order",
                   time_it([&] { quarter_rows<4><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("quarter_rows 8: a wave per 2 KiB half, grid order",
                   time_it([&] { quarter_rows<8><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("quarter_rows 16: a wave per packet, grid order",
                   time_it([&] { quarter_rows<16><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("rows_dword 16 waves/CU (the packetizer's copy shape)",
                   time_it([&] { rows_dword<0><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("rows_full: a wave per packet, the whole 4156-B packet written (header, payload, trailer)",
                   time_it([&] { rows_full<<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("rows_full, packets in the grid's order",
                   time_it([&] { rows_full<true><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("rows_full, 32 waves per CU",
                   time_it([&] { rows_full<<<cus * 2, 1024>>>(src, dst, cus * 32); }, reps));
            report("rows_full, packets in the grid's order, 32 waves per CU",
                   time_it([&] { rows_full<true><<<cus * 2, 1024>>>(src, dst, cus * 32); }, reps));
            report("rows_full, nt stores",
                   time_it([&] { rows_full<false, 2><<<cus, 1024>>>(src, dst, cus * 16); }, reps));
            report("flat_out: flat order over the output stream, whole packets, 16-B aligned stores",
                   time_it([&] { flat_out<<<cus * 4, 256>>>((const uint32_t *)src, (uint4 *)dst); }, reps));
            report("rows_wg: a workgroup per packet (a wave per row), whole packets, grid order",
                   time_it([&] { rows_wg<<<cus, 1024>>>(src, dst); }, reps));
            report("rows_wg: a workgroup per packet, 2 workgroups per CU",
                   time_it([&] { rows_wg<<<cus * 2, 1024>>>(src, dst); }, reps));
            report("hipMemcpyDtoD contiguous",
                   time_it([&] { CK(hipMemcpyAsync(dst, src, (size_t)kN * kPay, hipMemcpyDeviceToDevice, 0)); }, reps));
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        {
            // read shape (C1): 1 Mi x 4156 B of src
            const uint32_t n = 1048576u;
            const double rb = (double)n * 4152;
            uint32_t *o = (uint32_t *)dst;  // written only if the XOR hits a magic value
            float ms = time_it([&] { read_rows<false><<<cus, 1024>>>(src, o, cus * 16, n); }, reps);
            printf("{\"form\": \"read C1 shape, contiguous chunks\", \"ms\": %.4f, \"GB/s (read)\": %.1f}\n", ms, rb / (ms * 1e-3) / 1e9);
            ms = time_it([&] { read_rows<true><<<cus, 1024>>>(src, o, cus * 16, n); }, reps);
            printf("{\"form\": \"read C1 shape, interleaved packets\", \"ms\": %.4f, \"GB/s (read)\": %.1f}\n", ms, rb / (ms * 1e-3) / 1e9);
        }
        for (int w : {16, 32}) {
            const uint32_t waves = cus * w;
            const int grid = cus * (w / 16);
            char nm[96];
            snprintf(nm, sizeof nm, "rows_dword %d waves/CU, interleaved packets", w);
            report(nm, time_it([&] { rows_dword<0, true><<<grid, 1024>>>(src, dst, waves); }, reps));
            snprintf(nm, sizeof nm, "rows_x4 %d waves/CU, interleaved packets", w);
            report(nm, time_it([&] { rows_x4<0, true><<<grid, 1024>>>(src, dst, waves); }, reps));
            snprintf(nm, sizeof nm, "rows_x4 %d waves/CU, interleaved packets, nt stores", w);
            report(nm, time_it([&] { rows_x4<2, true><<<grid, 1024>>>(src, dst, waves); }, reps));
        }
        if (getenv("COPY_SHIFT")) {  // the packetizer's load misalignment against the aligned rows
            const uint32_t waves = cus * 16;
            report("rows_dword 16 waves/CU (aligned loads)", time_it([&] { rows_dword<0><<<cus, 1024>>>(src, dst, waves); }, reps));
            report("rows_dword 16 waves/CU, loads 252 B before each row (packetizer shape)",
                   time_it([&] { rows_dword<0, false, 252><<<cus, 1024>>>(src, dst, waves); }, reps));
            report("rows_dword 16 waves/CU, loads 64 B before each row (line aligned)",
                   time_it([&] { rows_dword<0, false, 64><<<cus, 1024>>>(src, dst, waves); }, reps));
            report("rows_dword 16 waves/CU, loads 4 B before each row",
                   time_it([&] { rows_dword<0, false, 4><<<cus, 1024>>>(src, dst, waves); }, reps));
            report("rows_dword 16 waves/CU, slots of 4160 B: stores line-aligned, loads 56 B off",
                   time_it([&] { rows_dword<0, false, 56, 4160, 0><<<cus, 1024>>>(src, dst, waves); }, reps));
            report("rows_dword 16 waves/CU, slots of 4160 B: stores and loads line-aligned",
                   time_it([&] { rows_dword<0, false, 0, 4160, 0><<<cus, 1024>>>(src, dst, waves); }, reps));
            const size_t n16 = (size_t)kN * kPay / 16;
            report("flat_x4 contiguous 16 waves/CU", time_it([&] { flat_x4<<<cus * 4, 256>>>((const uint4 *)src, (uint4 *)dst, n16); }, reps));
            continue;
        }
        for (int w : {16, 32}) {
            const uint32_t waves = cus * w;
            const int grid = cus * (w / 16);
            char nm[96];
            snprintf(nm, sizeof nm, "rows_dword %d waves/CU", w);
            report(nm, time_it([&] { rows_dword<0><<<grid, 1024>>>(src, dst, waves); }, reps));
            snprintf(nm, sizeof nm, "rows_dword %d waves/CU, nt stores", w);
            report(nm, time_it([&] { rows_dword<2><<<grid, 1024>>>(src, dst, waves); }, reps));
            snprintf(nm, sizeof nm, "rows_x4 %d waves/CU", w);
            report(nm, time_it([&] { rows_x4<0><<<grid, 1024>>>(src, dst, waves); }, reps));
            snprintf(nm, sizeof nm, "rows_x4 %d waves/CU, nt stores", w);
            report(nm, time_it([&] { rows_x4<2><<<grid, 1024>>>(src, dst, waves); }, reps));
        }
        const size_t n16 = (size_t)kN * kPay / 16;
        for (int w : {8, 16, 32}) {
            char nm[96];
            snprintf(nm, sizeof nm, "flat_x4 contiguous %d waves/CU", w);
            report(nm, time_it([&] { flat_x4<<<cus * w / 4, 256>>>((const uint4 *)src, (uint4 *)dst, n16); }, reps));
        }
        report("hipMemcpyDtoD contiguous",
               time_it([&] { CK(hipMemcpyAsync(dst, src, (size_t)kN * kPay, hipMemcpyDeviceToDevice, 0)); }, reps));
    }
    CK(hipFree(src));
    CK(hipFree(dst));
    return 0;
}
