// icrc_capi.cpp — the C-ABI of include/icrc.h: engines, scalar drop-ins, host- and
// device-resident batches.  Every CRC is computed by the HIP kernel (icrc_kernels.hip);
// this file only moves bytes and launches.  There is deliberately no CPU CRC here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "icrc_internal.h"

struct icrc_engine {
    int device = 0;
    int num_cu = 0;
    int variant = icrc::kDefaultVariant;
    uint32_t *d_table = nullptr;
    hipStream_t stream = nullptr;
    std::mutex mu;  // guards the staging buffers below
    // host-batch / scalar staging
    uint8_t *d_stage = nullptr;
    size_t d_stage_cap = 0;
    uint64_t *d_off = nullptr;
    uint32_t *d_len = nullptr;
    uint32_t *d_res = nullptr;  // ICRCs or ok bytes
    size_t d_meta_cap = 0;      // packets
    uint8_t *h_stage = nullptr; // pinned
    size_t h_stage_cap = 0;
};

namespace {

using icrc::BatchParams;

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(expr)                                  \
    do {                                               \
        if ((expr) != hipSuccess) return ICRC_EDEVICE; \
    } while (0)

int grid_for(const icrc_engine *e, uint32_t n) {
    const uint64_t want = (static_cast<uint64_t>(n) + icrc::kWavesPerGroup - 1) / icrc::kWavesPerGroup;
    return static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(want, static_cast<uint64_t>(e->num_cu))));
}

int ensure_device_stage(icrc_engine *e, size_t bytes, size_t pkts) {
    if (bytes > e->d_stage_cap) {
        if (e->d_stage) (void)hipFree(e->d_stage);
        e->d_stage = nullptr;
        e->d_stage_cap = 0;
        size_t cap = std::max<size_t>(bytes, 1 << 20);
        if (hipMalloc(&e->d_stage, cap + 64) != hipSuccess) return ICRC_ENOMEM;
        e->d_stage_cap = cap;
    }
    if (pkts > e->d_meta_cap) {
        if (e->d_off) (void)hipFree(e->d_off);
        if (e->d_len) (void)hipFree(e->d_len);
        if (e->d_res) (void)hipFree(e->d_res);
        e->d_off = nullptr;
        e->d_len = nullptr;
        e->d_res = nullptr;
        e->d_meta_cap = 0;
        size_t cap = std::max<size_t>(pkts, 4096);
        if (hipMalloc(&e->d_off, cap * sizeof(uint64_t)) != hipSuccess) return ICRC_ENOMEM;
        if (hipMalloc(&e->d_len, cap * sizeof(uint32_t)) != hipSuccess) return ICRC_ENOMEM;
        if (hipMalloc(&e->d_res, cap * sizeof(uint32_t)) != hipSuccess) return ICRC_ENOMEM;
        e->d_meta_cap = cap;
    }
    return ICRC_OK;
}

int ensure_host_stage(icrc_engine *e, size_t bytes) {
    if (bytes <= e->h_stage_cap) return ICRC_OK;
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    e->h_stage = nullptr;
    e->h_stage_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1 << 20);
    if (hipHostMalloc(&e->h_stage, cap, hipHostMallocDefault) != hipSuccess) return ICRC_ENOMEM;
    e->h_stage_cap = cap;
    return ICRC_OK;
}

std::mutex g_registry_mu;
std::map<int, icrc_engine *> g_default;

// Host-resident batch: stage packets [lo, hi) of one chunk into device memory, run the
// kernel, return ICRCs (mode compute) or ok bytes (mode verify) in e->d_res.
constexpr size_t kChunkBytes = size_t(256) << 20;

int validate_host(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n) {
    if (n == 0) return ICRC_OK;
    if (!base || !off || !len) return ICRC_EINVAL;
    for (uint32_t i = 0; i < n; i++)
        if (len[i] < ICRC_MIN_PACKET) return ICRC_EINVAL;  // the reference panics here
    return ICRC_OK;
}

int host_batch(icrc_engine *e, int mode, uint8_t *base, const uint64_t *off, const uint32_t *len,
               uint32_t n, uint32_t *out_icrc, uint8_t *ok, int trailer) {
    if (!e) return ICRC_EINVAL;
    if (n && mode == icrc::kCompute && !out_icrc && !trailer) return ICRC_EINVAL;
    if (n && mode == icrc::kVerify && !ok) return ICRC_EINVAL;
    int vrc = validate_host(base, off, len, n);
    if (vrc) return vrc;
    if (n == 0) return ICRC_OK;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<uint64_t> doff;
    std::vector<uint32_t> res;
    uint32_t i0 = 0;
    while (i0 < n) {
        // Grow the chunk while the packed size stays under kChunkBytes.
        uint32_t i1 = i0;
        size_t packed = 0;
        while (i1 < n && (i1 == i0 || packed + len[i1] <= kChunkBytes)) {
            packed += (static_cast<size_t>(len[i1]) + 3) & ~size_t(3);
            i1++;
        }
        const uint32_t cnt = i1 - i0;
        int rc = ensure_device_stage(e, packed, cnt);
        if (rc) return rc;
        rc = ensure_host_stage(e, packed);
        if (rc) return rc;
        // Gather into pinned staging (4-aligned slots so the kernel takes its fast path).
        doff.resize(cnt);
        size_t pos = 0;
        for (uint32_t i = 0; i < cnt; i++) {
            std::memcpy(e->h_stage + pos, base + off[i0 + i], len[i0 + i]);
            doff[i] = pos;
            pos += (static_cast<size_t>(len[i0 + i]) + 3) & ~size_t(3);
        }
        HIP_TRY(hipMemcpyAsync(e->d_stage, e->h_stage, pos, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->d_off, doff.data(), cnt * sizeof(uint64_t), hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->d_len, len + i0, cnt * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
        BatchParams p{};
        p.base = e->d_stage;
        p.off = e->d_off;
        p.len = e->d_len;
        p.n = cnt;
        p.table = e->d_table;
        p.trailer = 0;  // trailers are written on the host copy below
        p.variant = e->variant;
        if (mode == icrc::kCompute) p.out = e->d_res;
        else p.ok = reinterpret_cast<uint8_t *>(e->d_res);
        rc = icrc::launch_batch(mode, p, grid_for(e, cnt), e->stream);
        if (rc) return rc;
        if (mode == icrc::kCompute) {
            res.resize(cnt);
            HIP_TRY(hipMemcpyAsync(res.data(), e->d_res, cnt * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
            HIP_TRY(hipStreamSynchronize(e->stream));
            for (uint32_t i = 0; i < cnt; i++) {
                if (out_icrc) out_icrc[i0 + i] = res[i];
                if (trailer) {
                    uint8_t *t = base + off[i0 + i] + len[i0 + i] - 4;
                    const uint32_t c = res[i];
                    t[0] = uint8_t(c);
                    t[1] = uint8_t(c >> 8);
                    t[2] = uint8_t(c >> 16);
                    t[3] = uint8_t(c >> 24);
                }
            }
        } else {
            HIP_TRY(hipMemcpyAsync(ok + i0, e->d_res, cnt, hipMemcpyDeviceToHost, e->stream));
            HIP_TRY(hipStreamSynchronize(e->stream));
            if (trailer)
                for (uint32_t i = 0; i < cnt; i++) std::memset(base + off[i0 + i] + len[i0 + i] - 4, 0, 4);
        }
        i0 = i1;
    }
    return ICRC_OK;
}

int device_batch(icrc_engine *e, int mode, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                 uint64_t stride, uint32_t ulen, uint32_t n, uint32_t *d_out, uint8_t *d_ok, int trailer,
                 uint32_t *d_nerr, void *stream) {
    if (!e || !d_base) return ICRC_EINVAL;
    if (mode == icrc::kVerify && !d_ok) return ICRC_EINVAL;
    if (n == 0) return ICRC_OK;
    if (!d_len && ulen < ICRC_MIN_PACKET) return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    BatchParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.ulen = ulen;
    p.n = n;
    p.out = d_out;
    p.ok = d_ok;
    p.nerr = d_nerr;
    p.table = e->d_table;
    p.trailer = trailer ? 1 : 0;
    p.variant = e->variant;
    return icrc::launch_batch(mode, p, grid_for(e, n), stream);
}

}  // namespace

extern "C" {

const char *icrc_version(void) {
    return "icrc_amd 0.1 gfx950: wave-per-packet end-aligned column Horner, LDS M^64 byte tables "
           "(32x bank-replicated) + per-lane M^(64-l) nibble tables";
}

int icrc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int icrc_engine_create(int device, icrc_engine **out) {
    if (!out) return ICRC_EINVAL;
    *out = nullptr;
    int ndev = icrc_device_count();
    if (ndev <= 0) return ICRC_ENODEV;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= ndev) return ICRC_ENODEV;
    DeviceGuard g(device);
    if (!g.ok) return ICRC_ENODEV;
    auto *e = new (std::nothrow) icrc_engine();
    if (!e) return ICRC_ENOMEM;
    e->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete e;
        return ICRC_EDEVICE;
    }
    e->num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 1;
    std::vector<uint32_t> img(icrc::kLdsWords);
    icrc::build_table_image(img.data());
    if (hipMalloc(&e->d_table, icrc::kLdsBytes) != hipSuccess ||
        hipMemcpy(e->d_table, img.data(), icrc::kLdsBytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        icrc_engine_destroy(e);
        return ICRC_EDEVICE;
    }
    *out = e;
    return ICRC_OK;
}

int icrc_engine_destroy(icrc_engine *e) {
    if (!e) return ICRC_EINVAL;
    {
        DeviceGuard g(e->device);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
        if (e->d_table) (void)hipFree(e->d_table);
        if (e->d_stage) (void)hipFree(e->d_stage);
        if (e->d_off) (void)hipFree(e->d_off);
        if (e->d_len) (void)hipFree(e->d_len);
        if (e->d_res) (void)hipFree(e->d_res);
        if (e->h_stage) (void)hipHostFree(e->h_stage);
        if (e->stream) (void)hipStreamDestroy(e->stream);
    }
    {
        std::lock_guard<std::mutex> lk(g_registry_mu);
        for (auto it = g_default.begin(); it != g_default.end(); ++it)
            if (it->second == e) {
                g_default.erase(it);
                break;
            }
    }
    delete e;
    return ICRC_OK;
}

int icrc_engine_default(int device, icrc_engine **out) {
    if (!out) return ICRC_EINVAL;
    if (device < 0) {
        if (icrc_device_count() <= 0) return ICRC_ENODEV;
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    std::lock_guard<std::mutex> lk(g_registry_mu);
    auto it = g_default.find(device);
    if (it != g_default.end()) {
        *out = it->second;
        return ICRC_OK;
    }
    icrc_engine *e = nullptr;
    int rc = icrc_engine_create(device, &e);
    if (rc) return rc;
    g_default[device] = e;
    *out = e;
    return ICRC_OK;
}

int icrc_engine_device_ordinal(const icrc_engine *e) { return e ? e->device : ICRC_EINVAL; }

int icrc_engine_set_kernel_variant(icrc_engine *e, int variant) {
    if (!e || variant < -1 || variant > icrc::kMaxVariant) return ICRC_EINVAL;
    e->variant = variant < 0 ? icrc::kDefaultVariant : variant;
    return ICRC_OK;
}

void *icrc_engine_stream(const icrc_engine *e) { return e ? static_cast<void *>(e->stream) : nullptr; }

uint32_t icrc_compute(const uint8_t *pkt, size_t len, int *err) {
    int dummy;
    int *rc = err ? err : &dummy;
    *rc = ICRC_OK;
    if (!pkt || len < ICRC_MIN_PACKET || len > 0xFFFFFFFFull) {
        *rc = ICRC_EINVAL;
        return 0;
    }
    icrc_engine *e = nullptr;
    if ((*rc = icrc_engine_default(-1, &e)) != ICRC_OK) return 0;
    uint64_t off = 0;
    uint32_t l = static_cast<uint32_t>(len);
    uint32_t out = 0;
    *rc = host_batch(e, icrc::kCompute, const_cast<uint8_t *>(pkt), &off, &l, 1, &out, nullptr, 0);
    return *rc == ICRC_OK ? out : 0;
}

int icrc_verify(uint8_t *pkt, size_t len, int zero_trailer, int *ok) {
    if (!pkt || !ok || len < ICRC_MIN_PACKET || len > 0xFFFFFFFFull) return ICRC_EINVAL;
    icrc_engine *e = nullptr;
    int rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    uint64_t off = 0;
    uint32_t l = static_cast<uint32_t>(len);
    uint8_t r = 0;
    rc = host_batch(e, icrc::kVerify, pkt, &off, &l, 1, nullptr, &r, zero_trailer);
    if (rc == ICRC_OK) *ok = (r == ICRC_VERIFY_OK);
    return rc;
}

int icrc_compute_batch_ex(icrc_engine *e, uint8_t *base, const uint64_t *off, const uint32_t *len,
                          uint32_t n, uint32_t *out_icrc, int write_trailer) {
    return host_batch(e, icrc::kCompute, base, off, len, n, out_icrc, nullptr, write_trailer);
}

int icrc_verify_batch_ex(icrc_engine *e, uint8_t *base, const uint64_t *off, const uint32_t *len,
                         uint32_t n, uint8_t *ok, int zero_trailer) {
    return host_batch(e, icrc::kVerify, base, off, len, n, nullptr, ok, zero_trailer);
}

int icrc_compute_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                       uint32_t *out_icrc, int write_trailer) {
    int rc = validate_host(base, off, len, n);
    if (rc) return rc;
    icrc_engine *e = nullptr;
    rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    return icrc_compute_batch_ex(e, base, off, len, n, out_icrc, write_trailer);
}

int icrc_verify_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n, uint8_t *ok,
                      int zero_trailer) {
    int rc = validate_host(base, off, len, n);
    if (rc) return rc;
    icrc_engine *e = nullptr;
    rc = icrc_engine_default(-1, &e);
    if (rc) return rc;
    return icrc_verify_batch_ex(e, base, off, len, n, ok, zero_trailer);
}

int icrc_compute_batch_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                              uint32_t n, uint32_t *d_out, int write_trailer, uint32_t *d_nerr,
                              void *stream) {
    if (!d_off || !d_len) return ICRC_EINVAL;
    return device_batch(e, icrc::kCompute, d_base, d_off, d_len, 0, 0, n, d_out, nullptr, write_trailer,
                        d_nerr, stream);
}

int icrc_verify_batch_device(icrc_engine *e, uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                             uint32_t n, uint8_t *d_ok, int zero_trailer, uint32_t *d_nerr, void *stream) {
    if (!d_off || !d_len) return ICRC_EINVAL;
    return device_batch(e, icrc::kVerify, d_base, d_off, d_len, 0, 0, n, nullptr, d_ok, zero_trailer, d_nerr,
                        stream);
}

int icrc_compute_strided_device(icrc_engine *e, uint8_t *d_base, uint64_t stride, uint32_t len, uint32_t n,
                                uint32_t *d_out, int write_trailer, void *stream) {
    return device_batch(e, icrc::kCompute, d_base, nullptr, nullptr, stride, len, n, d_out, nullptr,
                        write_trailer, nullptr, stream);
}

int icrc_verify_strided_device(icrc_engine *e, uint8_t *d_base, uint64_t stride, uint32_t len, uint32_t n,
                               uint8_t *d_ok, int zero_trailer, void *stream) {
    return device_batch(e, icrc::kVerify, d_base, nullptr, nullptr, stride, len, n, nullptr, d_ok, zero_trailer,
                        nullptr, stream);
}

int icrc_synth_device(icrc_engine *e, uint8_t *d_base, const icrc_synth_desc *d_desc, const uint8_t *d_hdr,
                      uint32_t n, void *stream) {
    if (!e || !d_base || !d_desc || !d_hdr) return ICRC_EINVAL;
    DeviceGuard g(e->device);
    if (!g.ok) return ICRC_ENODEV;
    return icrc::launch_synth(d_base, d_desc, d_hdr, n, stream);
}

// Host-only helper for tests: the LDS table image (no GPU needed).
int icrc_table_image(uint32_t *out_words, uint32_t nwords) {
    if (!out_words || nwords < icrc::kLdsWords) return ICRC_EINVAL;
    icrc::build_table_image(out_words);
    return ICRC_OK;
}

}  // extern "C"
