// scripts/msg_probe.cpp — latency of ONE message through the host-resident batch drop-ins, the
// emulator's granularity for configs[0] (BASELINE.json: 1 QP, 64 x 4 KiB RDMA WRITE, ICRC compute
// + verify): icrc_compute_batch(write_trailer = 1) on the send side (PacketWriter::write,
// packet_processor.rs:260-263), icrc_verify_batch(zero_trailer = 1) on the receive side
// (is_icrc_valid, packet_processor.rs:341-353).  Cases: pinned / pageable message buffers; 64
// packets, and 1 packet (the per-call floor).  Run it under rocprofv3 --kernel-trace --stats to
// split each call into kernel time and the rest.  Prints one JSON line per case (p50 / p99 /
// mean microseconds per call); every verify must succeed.  MSG_PROBE_PATH=launch runs the host
// messages as one kernel launch each (ICRC_HOST_LAUNCH) instead of through the submission ring
// (the default); the last line is the ring's counters (icrc_engine_host_stats).
// Build: see scripts/Makefile (links libicrc_amd.so and the HIP runtime for pinned memory).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "icrc.h"

namespace {

using clk = std::chrono::steady_clock;

double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[static_cast<size_t>(q * (v.size() - 1))];
}

void run(const char *name, uint8_t *buf, uint32_t npk, uint32_t L, int calls) {
    std::vector<uint64_t> off(npk);
    std::vector<uint32_t> len(npk, L);
    for (uint32_t i = 0; i < npk; ++i) off[i] = static_cast<uint64_t>(i) * L;
    std::vector<uint32_t> crc(npk);
    std::vector<uint8_t> ok(npk);
    std::vector<double> tc, tv;
    long bad = 0;
    for (int c = 0; c < calls + 20; ++c) {
        const auto t0 = clk::now();
        const int r1 = icrc_compute_batch(buf, off.data(), len.data(), npk, crc.data(), 1);
        const auto t1 = clk::now();
        const int r2 = icrc_verify_batch(buf, off.data(), len.data(), npk, ok.data(), 1);
        const auto t2 = clk::now();
        if (r1 || r2) bad++;
        for (uint32_t i = 0; i < npk; ++i) bad += ok[i] != ICRC_VERIFY_OK;
        if (c >= 20) {
            tc.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            tv.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
        }
    }
    double mc = 0, mv = 0;
    for (double x : tc) mc += x;
    for (double x : tv) mv += x;
    printf("{\"case\": \"%s\", \"packets\": %u, \"packet_bytes\": %u, \"compute_p50_us\": %.1f, \"compute_p99_us\": %.1f, "
           "\"compute_mean_us\": %.1f, \"verify_p50_us\": %.1f, \"verify_p99_us\": %.1f, \"verify_mean_us\": %.1f, "
           "\"bad\": %ld}\n",
           name, npk, L, pct(tc, 0.5), pct(tc, 0.99), mc / tc.size(), pct(tv, 0.5), pct(tv, 0.99), mv / tv.size(), bad);
    fflush(stdout);
}

// T threads, each its own pinned (kind 1; kind 2: pinned and coherent; kind 3: 2 MiB transparent huge
// pages registered with hipHostRegister) or pageable (kind 0) copy of the message, each running `calls` messages
// (compute + verify): messages/s in total and p50 / p99 per message — the emulator's three callers.
void run_threads(const char *name, const std::vector<uint8_t> &src, int kind, uint32_t npk, uint32_t L,
                 int calls, int T) {
    const bool pinned_bufs = kind != 0;
    std::vector<uint8_t *> bufs(T);
    std::vector<std::vector<uint8_t>> pageable(T);
    for (int t = 0; t < T; ++t) {
        if (kind == 3) {
            const size_t hb = (src.size() + (2u << 20) - 1) & ~((size_t(2) << 20) - 1);
            void *m = nullptr;
            if (posix_memalign(&m, size_t(2) << 20, hb) != 0) exit(1);
            (void)madvise(m, hb, MADV_HUGEPAGE);
            std::memset(m, 0, hb);
            if (hipHostRegister(m, hb, hipHostRegisterMapped) != hipSuccess) {
                fprintf(stderr, "hipHostRegister failed\n");
                exit(1);
            }
            bufs[t] = static_cast<uint8_t *>(m);
        } else if (pinned_bufs) {
            const unsigned fl = kind == 2 ? hipHostMallocCoherent : hipHostMallocDefault;
            if (hipHostMalloc(reinterpret_cast<void **>(&bufs[t]), src.size(), fl) != hipSuccess) {
                fprintf(stderr, "hipHostMalloc failed\n");
                exit(1);
            }
        } else {
            pageable[t] = src;
            bufs[t] = pageable[t].data();
        }
        std::memcpy(bufs[t], src.data(), src.size());
    }
    std::vector<std::vector<double>> lat(T);
    std::atomic<long> bad{0};
    std::atomic<int> ready{0};
    auto worker = [&](int t) {
        std::vector<uint64_t> off(npk);
        std::vector<uint32_t> len(npk, L), crc(npk);
        std::vector<uint8_t> ok(npk);
        for (uint32_t i = 0; i < npk; ++i) off[i] = static_cast<uint64_t>(i) * L;
        for (int c = 0; c < 20; ++c) {  // warm-up (lane and staging allocations), outside the timed region
            icrc_compute_batch(bufs[t], off.data(), len.data(), npk, crc.data(), 1);
            icrc_verify_batch(bufs[t], off.data(), len.data(), npk, ok.data(), 1);
        }
        ready.fetch_add(1);
        while (ready.load() < T + 1) {
        }
        for (int c = 20; c < calls + 20; ++c) {
            const auto t0 = clk::now();
            const int r1 = icrc_compute_batch(bufs[t], off.data(), len.data(), npk, crc.data(), 1);
            const int r2 = icrc_verify_batch(bufs[t], off.data(), len.data(), npk, ok.data(), 1);
            const auto t1 = clk::now();
            long b = (r1 || r2) ? 1 : 0;
            for (uint32_t i = 0; i < npk; ++i) b += ok[i] != ICRC_VERIFY_OK;
            if (b) bad.fetch_add(b);
            if (c >= 20) lat[t].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
    while (ready.load() < T) {
    }
    const auto t0 = clk::now();
    ready.fetch_add(1);  // release the timed calls
    for (auto &x : th) x.join();
    const double secs = std::chrono::duration<double>(clk::now() - t0).count();
    std::vector<double> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    printf("{\"case\": \"%s\", \"threads\": %d, \"packets\": %u, \"packet_bytes\": %u, \"messages_per_s\": %.0f, "
           "\"message_p50_us\": %.1f, \"message_p99_us\": %.1f, \"bad\": %ld}\n",
           name, T, npk, L, T * calls / secs, pct(all, 0.5), pct(all, 0.99), bad.load());
    fflush(stdout);
    if (kind == 3) {
        for (auto *b : bufs) {
            (void)hipHostUnregister(b);
            free(b);
        }
    } else if (pinned_bufs) {
        for (auto *b : bufs) (void)hipHostFree(b);
    }
}

}  // namespace

void print_stats(const char *path) {
    icrc_engine *e = nullptr;
    uint64_t st[4] = {0, 0, 0, 0};
    if (icrc_engine_default(-1, &e) == ICRC_OK) (void)icrc_engine_host_stats(e, st);
    printf("{\"host_path\": \"%s\", \"ring_jobs\": %llu, \"ring_launches\": %llu, \"ring_relaunches\": %llu, "
           "\"ring_timeouts\": %llu}\n",
           path, static_cast<unsigned long long>(st[0]), static_cast<unsigned long long>(st[1]),
           static_cast<unsigned long long>(st[2]), static_cast<unsigned long long>(st[3]));
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 2000;
    const char *pv = getenv("MSG_PROBE_PATH");
    const bool launch = pv && strcmp(pv, "launch") == 0;
    {
        icrc_engine *e = nullptr;
        if (icrc_engine_default(-1, &e) != ICRC_OK ||
            icrc_engine_set_host_path(e, launch ? ICRC_HOST_LAUNCH : ICRC_HOST_RING) != ICRC_OK) {
            fprintf(stderr, "no engine\n");
            return 1;
        }
    }
    const char *path = launch ? "launch" : "ring";
    const uint32_t L = 4156, npk = 64;
    std::vector<uint8_t> pageable(static_cast<size_t>(npk) * L);
    uint32_t x = 12345;
    for (auto &b : pageable) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        b = static_cast<uint8_t>(x);
    }
    uint8_t *pinned = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&pinned), pageable.size(), hipHostMallocDefault) != hipSuccess) {
        fprintf(stderr, "hipHostMalloc failed\n");
        return 1;
    }
    std::memcpy(pinned, pageable.data(), pageable.size());
    if (argc > 2) {  // msg_probe CALLS THREADS...: the multi-threaded message rate only
        // MSG_PROBE_KINDS=pinned (bench.py's default-line leg): the pinned buffers alone
        const char *kinds = getenv("MSG_PROBE_KINDS");
        const bool all = !kinds || strcmp(kinds, "pinned") != 0;
        for (int a = 2; a < argc; ++a) {
            const int T = atoi(argv[a]);
            run_threads(launch ? "pinned, launch" : "pinned, ring", pageable, 1, npk, L, calls, T);
            if (!all) continue;
            run_threads(launch ? "pinned_coherent, launch" : "pinned_coherent, ring", pageable, 2, npk, L, calls, T);
            run_threads(launch ? "registered_huge, launch" : "registered_huge, ring", pageable, 3, npk, L, calls, T);
            run_threads(launch ? "pageable, launch" : "pageable, ring", pageable, 0, npk, L, calls, T);
        }
        print_stats(path);
        (void)hipHostFree(pinned);
        return icrc_shutdown() == ICRC_OK ? 0 : 1;  // the ring and engine go before the HIP runtime's teardown
    }
    run(launch ? "pinned, launch" : "pinned, ring", pinned, npk, L, calls);
    run(launch ? "pageable, launch" : "pageable, ring", pageable.data(), npk, L, calls);
    run(launch ? "pinned_1_packet, launch" : "pinned_1_packet, ring", pinned, 1, L, calls);
    run(launch ? "pageable_1_packet, launch" : "pageable_1_packet, ring", pageable.data(), 1, L, calls);
    print_stats(path);
    (void)hipHostFree(pinned);
    return icrc_shutdown() == ICRC_OK ? 0 : 1;
}
