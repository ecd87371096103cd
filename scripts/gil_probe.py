"""scripts/gil_probe.py — is the Python 3-thread message swing the GIL, not the library?

Stands in for bench.py's c0_message legs with no GPU and no icrc library: each "message" is two
ctypes calls into a C function that spins for SPIN_US microseconds with the GIL released (the
library's calls take ~20-25 us each through the ring), wrapped by the same numpy work as
icrc_amd.compute_icrc_batch / verify_icrc_batch (ascontiguousarray, zeros, count_nonzero).  Prints
messages/s for 1 and 3 threads, ROUNDS times, as JSON lines.  The spin function is built with gcc
into scripts/_build/libgilspin.so.

    python scripts/gil_probe.py [SPIN_US=22] [ROUNDS=5] [MESSAGES=1000] [SWITCH_INTERVAL_S]

SWITCH_INTERVAL_S: sys.setswitchinterval for the run (CPython's default is 0.005 s).
"""
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(ROOT, "_build", "libgilspin.so")
SRC = r"""
#include <stdint.h>
#include <time.h>
static uint64_t now_ns(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1000000000ull + t.tv_nsec; }
int gil_spin(uint64_t ns, uint32_t *out, uint32_t n) {
    const uint64_t end = now_ns() + ns;
    while (now_ns() < end) { __builtin_ia32_pause(); }
    for (uint32_t i = 0; i < n; ++i) out[i] = 1;
    return 0;
}
"""


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = SO[:-3] + ".c"
    with open(src, "w") as f:
        f.write(SRC)
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", SO, src], check=True)


def run(nth, spin_us, msgs, lib):
    off = np.arange(64, dtype=np.uint64) * 4156
    lens = np.full(64, 4156, np.uint32)
    ends = [0.0] * nth
    start = [0.0]
    lat = [[] for _ in range(nth)]
    gate = threading.Barrier(nth, action=lambda: start.__setitem__(0, time.perf_counter()))

    def call():
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros(o.size, dtype=np.uint32)
        lib.gil_spin(spin_us * 1000, out.ctypes.data, ln.size)
        return out

    def worker(k):
        for i in range(msgs + 20):
            if i == 20:
                gate.wait()
            t0 = time.perf_counter_ns()
            call()
            ok = call()
            t1 = time.perf_counter_ns()
            if i >= 20:
                lat[k].append((t1 - t0) / 1e3)
            int(np.count_nonzero(ok != 1))
        ends[k] = time.perf_counter()

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(nth)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    allv = np.concatenate([np.asarray(x) for x in lat])
    return {"threads": nth, "spin_us": spin_us, "messages_per_s": round(nth * msgs / (max(ends) - start[0]), 1),
            "p50_us": round(float(np.percentile(allv, 50)), 1), "mean_us": round(float(allv.mean()), 1)}


def main():
    spin = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    msgs = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    if len(sys.argv) > 4:
        sys.setswitchinterval(float(sys.argv[4]))
    if not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    lib.gil_spin.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
    for r in range(rounds):
        for nth in (1, 3):
            print(json.dumps(dict(round=r, switch_interval_s=sys.getswitchinterval(), **run(nth, spin, msgs, lib))),
                  flush=True)


if __name__ == "__main__":
    main()
