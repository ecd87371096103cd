// scripts/hipq_probe.cpp — what the host-message path's pointer queries cost per call: the
// library asks HIP whether a caller buffer is pinned (hipPointerGetAttributes), for its device view
// (hipHostGetDevicePointer) and for its allocation's extent (hipMemGetAddressRange) on every
// message.  Mean ns per query from 1 and 3 threads, pinned and pageable pointers.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

int main() {
    void *pinned = nullptr;
    if (hipHostMalloc(&pinned, 1 << 20, hipHostMallocDefault) != hipSuccess) return 1;
    std::vector<char> pageable(1 << 20);
    const int reps = 100000;
    auto bench = [&](const char *what, int T, auto f) {
        std::atomic<int> go{0};
        std::vector<std::thread> th;
        std::vector<double> ns(T);
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                while (!go.load()) {
                }
                const auto a = clk::now();
                for (int i = 0; i < reps; ++i) f();
                ns[t] = std::chrono::duration<double, std::nano>(clk::now() - a).count() / reps;
            });
        go = 1;
        for (auto &x : th) x.join();
        double m = 0;
        for (double x : ns) m += x;
        printf("{\"query\": \"%s\", \"threads\": %d, \"ns_per_call\": %.0f}\n", what, T, m / T);
        fflush(stdout);
    };
    for (int T : {1, 3}) {
        bench("hipPointerGetAttributes(pinned)", T, [&] {
            hipPointerAttribute_t a;
            (void)hipPointerGetAttributes(&a, static_cast<char *>(pinned) + 4096);
        });
        bench("hipPointerGetAttributes(pageable)", T, [&] {
            hipPointerAttribute_t a;
            if (hipPointerGetAttributes(&a, pageable.data() + 4096) != hipSuccess) (void)hipGetLastError();
        });
        bench("hipHostGetDevicePointer(pinned)", T, [&] {
            void *d = nullptr;
            (void)hipHostGetDevicePointer(&d, static_cast<char *>(pinned) + 4096, 0);
        });
        bench("hipMemGetAddressRange(device view)", T, [&] {
            void *d = nullptr;
            (void)hipHostGetDevicePointer(&d, static_cast<char *>(pinned) + 4096, 0);
            hipDeviceptr_t b = nullptr;
            size_t s = 0;
            (void)hipMemGetAddressRange(&b, &s, d);
        });
    }
    (void)hipHostFree(pinned);
    return 0;
}
