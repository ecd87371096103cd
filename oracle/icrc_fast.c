/*
 * oracle/icrc_fast.c — TEST INFRASTRUCTURE ONLY: the CPU baseline leg of bench.py.
 *
 * The reference hashes with crc32fast 1.4.2 (Cargo.lock:230-236).  On x86-64 with
 * SSE4.1 + PCLMULQDQ, crc32fast dispatches Hasher::update to its specialized PCLMULQDQ
 * folding path for buffers of >= 128 bytes (4 x 128-bit lanes folded 64 bytes at a time,
 * then 128->64->32-bit reduction and Barrett), and to its table "baseline" path
 * (slice-by-16) for shorter buffers and the tail.  This file restates that published
 * algorithm so the CPU baseline runs at the speed the reference's own hasher would,
 * and calls it exactly the way compute_icrc does (packet_processor.rs:276-300: three
 * update() calls of 8, 40 and len-44 bytes).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>
#include <wmmintrin.h>

#include "icrc_oracle.h"

static uint32_t T16[16][256];
static pthread_once_t t16_once = PTHREAD_ONCE_INIT;

static void t16_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        T16[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
        for (int t = 1; t < 16; t++) T16[t][i] = (T16[t - 1][i] >> 8) ^ T16[0][T16[t - 1][i] & 0xffu];
}

/* crc32fast baseline::update_fast_16 (slice-by-16), zlib chaining convention. */
uint32_t fast_crc32_slice16(uint32_t crc, const uint8_t *p, size_t n) {
    pthread_once(&t16_once, t16_init);
    uint32_t c = ~crc;
    while (n >= 16) {
        uint32_t w0, w1, w2, w3;
        memcpy(&w0, p, 4);
        memcpy(&w1, p + 4, 4);
        memcpy(&w2, p + 8, 4);
        memcpy(&w3, p + 12, 4);
        w0 ^= c;
        c = T16[15][w0 & 0xff] ^ T16[14][(w0 >> 8) & 0xff] ^ T16[13][(w0 >> 16) & 0xff] ^
            T16[12][w0 >> 24] ^ T16[11][w1 & 0xff] ^ T16[10][(w1 >> 8) & 0xff] ^
            T16[9][(w1 >> 16) & 0xff] ^ T16[8][w1 >> 24] ^ T16[7][w2 & 0xff] ^
            T16[6][(w2 >> 8) & 0xff] ^ T16[5][(w2 >> 16) & 0xff] ^ T16[4][w2 >> 24] ^
            T16[3][w3 & 0xff] ^ T16[2][(w3 >> 8) & 0xff] ^ T16[1][(w3 >> 16) & 0xff] ^
            T16[0][w3 >> 24];
        p += 16;
        n -= 16;
    }
    while (n--) c = T16[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return ~c;
}

/* Folding constants for the reflected polynomial 0xEDB88320 (x^(4*128+32) etc. mod P,
 * bit-reflected), Barrett mu and P' — the published crc32fast / Intel white-paper set. */
#define K1 0x154442bd4LL
#define K2 0x1c6e41596LL
#define K3 0x1751997d0LL
#define K4 0x0ccaa009eLL
#define K5 0x163cd6124LL
#define P_X 0x1DB710641LL
#define U_PRIME 0x1F7011641LL

__attribute__((target("sse4.1,pclmul"))) static inline __m128i reduce128(__m128i a, __m128i b,
                                                                          __m128i keys) {
    __m128i t1 = _mm_clmulepi64_si128(a, keys, 0x00);
    __m128i t2 = _mm_clmulepi64_si128(a, keys, 0x11);
    return _mm_xor_si128(_mm_xor_si128(b, t1), t2);
}

__attribute__((target("sse4.1,pclmul"))) static uint32_t crc32_pclmul(uint32_t crc,
                                                                       const uint8_t *p,
                                                                       size_t n) {
    __m128i x3 = _mm_loadu_si128((const __m128i *)p);
    __m128i x2 = _mm_loadu_si128((const __m128i *)(p + 16));
    __m128i x1 = _mm_loadu_si128((const __m128i *)(p + 32));
    __m128i x0 = _mm_loadu_si128((const __m128i *)(p + 48));
    p += 64;
    n -= 64;
    x3 = _mm_xor_si128(x3, _mm_cvtsi32_si128((int)~crc));
    const __m128i k1k2 = _mm_set_epi64x(K2, K1);
    while (n >= 64) {
        x3 = reduce128(x3, _mm_loadu_si128((const __m128i *)p), k1k2);
        x2 = reduce128(x2, _mm_loadu_si128((const __m128i *)(p + 16)), k1k2);
        x1 = reduce128(x1, _mm_loadu_si128((const __m128i *)(p + 32)), k1k2);
        x0 = reduce128(x0, _mm_loadu_si128((const __m128i *)(p + 48)), k1k2);
        p += 64;
        n -= 64;
    }
    const __m128i k3k4 = _mm_set_epi64x(K4, K3);
    __m128i x = reduce128(x3, x2, k3k4);
    x = reduce128(x, x1, k3k4);
    x = reduce128(x, x0, k3k4);
    while (n >= 16) {
        x = reduce128(x, _mm_loadu_si128((const __m128i *)p), k3k4);
        p += 16;
        n -= 16;
    }
    /* 128 -> 64 */
    x = _mm_xor_si128(_mm_clmulepi64_si128(x, k3k4, 0x10), _mm_srli_si128(x, 8));
    x = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x, _mm_set_epi32(0, 0, 0, ~0)),
                                           _mm_set_epi64x(0, K5), 0x00),
                      _mm_srli_si128(x, 4));
    /* Barrett 64 -> 32 */
    const __m128i pu = _mm_set_epi64x(U_PRIME, P_X);
    __m128i t1 = _mm_clmulepi64_si128(_mm_and_si128(x, _mm_set_epi32(0, 0, 0, ~0)), pu, 0x10);
    __m128i t2 = _mm_clmulepi64_si128(_mm_and_si128(t1, _mm_set_epi32(0, 0, 0, ~0)), pu, 0x00);
    uint32_t c = (uint32_t)_mm_extract_epi32(_mm_xor_si128(x, t2), 1);
    if (n) return fast_crc32_slice16(~c, p, n);
    return ~c;
}

static int have_pclmul(void) {
    static int cached = -1;
    if (cached < 0) {
        __builtin_cpu_init();
        cached = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    }
    return cached;
}

uint32_t fast_crc32(uint32_t crc, const uint8_t *p, size_t n) {
    if (n < 128 || !have_pclmul()) return fast_crc32_slice16(crc, p, n);
    return crc32_pclmul(crc, p, n);
}

/* compute_icrc with the crc32fast-equivalent hasher: same three update() calls. */
int fast_compute_icrc(const uint8_t *pkt, size_t len, uint32_t *out) {
    if (len < 44) return ORACLE_EINVAL;
    static const uint8_t prefix[8] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    uint8_t hdr[40];
    memcpy(hdr, pkt, 40);
    hdr[1] = hdr[8] = hdr[10] = hdr[11] = hdr[26] = hdr[27] = hdr[32] = 0xff;
    uint32_t c = fast_crc32(0, prefix, 8);
    c = fast_crc32(c, hdr, 40);
    c = fast_crc32(c, pkt + 40, len - 44);
    *out = c;
    return 0;
}

typedef struct {
    const uint8_t *base;
    uint64_t stride;
    uint32_t len;
    uint64_t lo, hi;
    uint32_t *out;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) fast_compute_icrc(j->base + i * j->stride, j->len, &j->out[i]);
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double fast_icrc_strided_timed(const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n,
                               uint32_t *out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    job_t jobs[256];
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t].base = base;
        jobs[t].stride = stride;
        jobs[t].len = len;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].out = out;
        if (threads == 1) worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return now_s() - t0;
}

/* generate_payload_from_msg cost model, util.rs:172-186 + common.rs:104-106. */
double fast_emulator_path_timed(const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n,
                                uint32_t *out) {
    double t0 = now_s();
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *pkt = base + i * stride;
        uint8_t *data = (uint8_t *)malloc(len);          /* vec![0u8; len] + DMA copy */
        memcpy(data, pkt, len);
        uint8_t *buf = (uint8_t *)calloc(8192, 1);        /* vec![0; 8192] */
        memcpy(buf, data, len);                           /* PacketWriter header+payload */
        fast_compute_icrc(buf, len, &out[i]);
        memcpy(buf + len - 4, &out[i], 4);
        uint8_t *udp = (uint8_t *)malloc(len - 28);       /* udp_datagram.payload().to_vec() */
        memcpy(udp, buf + 28, len - 28);
        __asm__ __volatile__("" ::"r"(udp) : "memory");
        free(udp);
        free(buf);
        free(data);
    }
    return now_s() - t0;
}

/* is_icrc_valid with the fast core (packet_processor.rs:341-353). */
static int fast_is_icrc_valid(uint8_t *pkt, size_t len, int zero) {
    uint32_t stored, c;
    memcpy(&stored, pkt + len - 4, 4);
    if (zero) memset(pkt + len - 4, 0, 4);
    fast_compute_icrc(pkt, len, &c);
    return stored == c;
}

typedef struct {
    uint8_t *base;
    uint64_t stride;
    uint32_t len;
    uint64_t lo, hi;
    uint8_t *ok;
    int zero;
} vjob_t;

static void *vworker(void *arg) {
    vjob_t *j = (vjob_t *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) j->ok[i] = (uint8_t)fast_is_icrc_valid(j->base + i * j->stride, j->len, j->zero);
    return NULL;
}

double fast_verify_strided_timed(uint8_t *base, uint64_t stride, uint32_t len, uint64_t n, uint8_t *ok,
                                 int threads, int zero) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if (len < 44) return -1.0;
    pthread_t tid[256];
    vjob_t jobs[256];
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t] = (vjob_t){base, stride, len, n * (uint64_t)t / (uint64_t)threads, n * (uint64_t)(t + 1) / (uint64_t)threads,
                           ok, zero};
        if (threads == 1) vworker(&jobs[t]);
        else pthread_create(&tid[t], NULL, vworker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return now_s() - t0;
}

typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    uint64_t n;
    int reps;
    uint64_t bad;
} c0job_t;

static void *c0worker(void *arg) {
    c0job_t *j = (c0job_t *)arg;
    for (int r = 0; r < j->reps; r++) {
        for (uint64_t i = 0; i < j->n; i++) {
            const uint8_t *pkt = j->base + j->off[i];
            const uint32_t L = j->len[i];
            if (L < 44) { j->bad++; continue; }
            /* send: generate_payload_from_msg (util.rs:172-186) around PacketWriter::write */
            uint8_t *data = (uint8_t *)malloc(L);
            memcpy(data, pkt, L);
            uint8_t *buf = (uint8_t *)calloc(8192, 1);
            memcpy(buf, data, L);
            uint32_t c;
            fast_compute_icrc(buf, L, &c);
            memcpy(buf + L - 4, &c, 4);
            uint8_t *udp = (uint8_t *)malloc(L - 28);
            memcpy(udp, buf + 28, L - 28);
            /* receive: the datagram as it arrives (IPv4 header + UDP payload), is_icrc_valid */
            uint8_t *rx = (uint8_t *)malloc(L);
            memcpy(rx, buf, 28);
            memcpy(rx + 28, udp, L - 28);
            if (!fast_is_icrc_valid(rx, L, 1)) j->bad++;
            __asm__ __volatile__("" ::"r"(rx) : "memory");
            free(rx);
            free(udp);
            free(buf);
            free(data);
        }
    }
    return NULL;
}

double fast_c0_roundtrip_timed(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                               int threads, int reps, uint64_t *bad) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    c0job_t jobs[256];
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t] = (c0job_t){base, off, len, n, reps, 0};
        if (threads == 1) c0worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, c0worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    const double secs = now_s() - t0;
    uint64_t b = 0;
    for (int t = 0; t < threads; t++) b += jobs[t].bad;
    if (bad) *bad = b;
    return secs;
}
