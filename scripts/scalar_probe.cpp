// scripts/scalar_probe.cpp — latency of the scalar drop-ins icrc_compute / icrc_verify
// (compute_icrc, packet_processor.rs:275-301; is_icrc_valid, 341-353) under the reference's
// call pattern: one call per packet from the send thread (packet_processor.rs:260), the
// packet-handler thread and the rust_driver receive thread (udp_agent.rs:99) — 1 and 3
// concurrent threads, 4156-B WRITE packets and 48-B ACKs.  Prints one JSON line per case
// (p50 / p99 / mean in microseconds, calls per second) and checks every result: a verify of a
// packet whose trailer holds the computed ICRC must succeed, one with a flipped bit must fail.
// Build: g++ -O2 -std=c++17 -I../include scalar_probe.cpp -L../open-rdma-driver_amd/_build
//        -licrc_amd -Wl,-rpath,'$ORIGIN/../open-rdma-driver_amd/_build' -lpthread
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "icrc.h"

namespace {

using clk = std::chrono::steady_clock;

std::vector<uint8_t> make_packet(uint32_t L, uint32_t seed) {
    std::vector<uint8_t> p(L);
    uint32_t x = seed * 2654435761u + 1;
    for (auto &b : p) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        b = static_cast<uint8_t>(x);
    }
    p[0] = 0x45;
    return p;
}

struct Result {
    std::vector<double> us;
    long bad = 0;
};

// Each call: compute (send side) then verify with zeroing (receive side) on a copy, plus a
// negative every 16th call.
void worker(int tid, uint32_t L, int calls, bool verify, Result &r, std::atomic<int> &go) {
    std::vector<std::vector<uint8_t>> pk;
    for (int i = 0; i < 16; ++i) pk.push_back(make_packet(L, 1000u * tid + i));
    while (!go.load()) {
    }
    r.us.reserve(calls);
    for (int c = 0; c < calls; ++c) {
        auto &p = pk[c & 15];
        int err = 0;
        if (!verify) {
            const auto t0 = clk::now();
            const uint32_t v = icrc_compute(p.data(), p.size(), &err);
            const auto t1 = clk::now();
            r.us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            if (err) r.bad++;
            std::memcpy(p.data() + L - 4, &v, 4);
        } else {
            const uint32_t v = icrc_compute(p.data(), p.size(), &err);
            std::memcpy(p.data() + L - 4, &v, 4);
            const bool neg = (c & 15) == 7;
            if (neg) p[L / 2] ^= 1;
            int ok = -1;
            const auto t0 = clk::now();
            const int rc = icrc_verify(p.data(), p.size(), 1, &ok);
            const auto t1 = clk::now();
            r.us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            uint32_t tr;
            std::memcpy(&tr, p.data() + L - 4, 4);
            if (rc || err || ok != (neg ? 0 : 1) || tr != 0) r.bad++;
            if (neg) p[L / 2] ^= 1;
        }
    }
}

void run_case(const char *what, uint32_t L, int threads, int calls, bool verify) {
    std::vector<Result> res(threads);
    std::vector<std::thread> th;
    std::atomic<int> go{0};
    for (int t = 0; t < threads; ++t) th.emplace_back(worker, t, L, calls, verify, std::ref(res[t]), std::ref(go));
    const auto t0 = clk::now();
    go = 1;
    for (auto &t : th) t.join();
    const double secs = std::chrono::duration<double>(clk::now() - t0).count();
    std::vector<double> all;
    long bad = 0;
    for (auto &r : res) {
        // drop the first 32 calls of each thread (first-touch of staging, code paging)
        all.insert(all.end(), r.us.begin() + std::min<size_t>(32, r.us.size()), r.us.end());
        bad += r.bad;
    }
    std::sort(all.begin(), all.end());
    double mean = 0;
    for (double v : all) mean += v;
    mean /= all.empty() ? 1 : all.size();
    auto pct = [&](double q) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, size_t(q * all.size()))]; };
    printf("{\"call\": \"%s\", \"packet_bytes\": %u, \"threads\": %d, \"calls_per_thread\": %d, \"p50_us\": %.2f, "
           "\"p99_us\": %.2f, \"mean_us\": %.2f, \"max_us\": %.1f, \"calls_per_s\": %.0f, \"bad\": %ld}\n",
           what, L, threads, calls, pct(0.5), pct(0.99), mean, all.empty() ? 0.0 : all.back(),
           threads * calls / secs, bad);
    fflush(stdout);
}

}  // namespace

int main(int argc, char **argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 2000;
    if (icrc_device_count() <= 0) {
        fprintf(stderr, "no GPU\n");
        return 2;
    }
    int err = 0;
    auto warm = make_packet(4156, 7);
    (void)icrc_compute(warm.data(), warm.size(), &err);  // creates the default engine
    if (err) {
        fprintf(stderr, "icrc_compute failed: %d\n", err);
        return 1;
    }
    for (uint32_t L : {4156u, 48u})
        for (int threads : {1, 3}) {
            run_case("icrc_compute", L, threads, calls, false);
            run_case("icrc_verify", L, threads, calls, true);
        }
    return 0;
}
