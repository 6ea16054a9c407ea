/*
 * csum_oracle.c — CPU restatement of wireglider's checksum hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see csum_oracle.h).  Never linked into, loaded
 * by, or called from the wireglider_amd product library.
 *
 * Reference citations are dinhngtu/wireglider @ 2024-11-01, relative to the
 * reference root.
 */
#define _GNU_SOURCE
#include "csum_oracle.h"
#include "orc_pin.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

/* ------------------------------------------------------------------------ */
/* Scalar arithmetic                                                        */
/* ------------------------------------------------------------------------ */

/* tests/checksum_tests.hpp:11-34: LE 16-bit words into a 64-bit sum, odd
 * trailing byte as the low byte (RFC 1071 erratum 3133, :20-26), fold with
 * a carry loop, complement. */
uint16_t orc_checksum_ref1(const uint8_t *data, size_t size) {
    uint64_t csum = 0;
    size_t i = size;
    while (i > 1) {
        uint16_t word;
        memcpy(&word, data + (size - i), sizeof(word));
        csum += word;
        i -= 2;
    }
    if (i == 1)
        csum += (uint16_t)data[size - 1];
    for (;;) {
        uint64_t carry = csum >> 16;
        if (!carry)
            break;
        csum = (csum & 0xffff) + carry;
    }
    return (uint16_t)(~csum & 0xffff);
}

/* One's-complement 64-bit add with end-around carry: the primitive of
 * checksum_impl::checksum_add / checksum_nofold<N> (include/netio/checksum.hpp:20-77). */
static inline uint64_t add_eac(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    return s + (s < b);
}

/* include/netio/checksum.hpp:79-100.  The reference dispatches to one of
 * fastcsum's nofold kernels; all of them satisfy the same contract, checked
 * by tests/test-checksum.cpp:11-51: the folded result equals checksum_ref1.
 * Here: LE 32-bit words summed into a 64-bit accumulator (no carry can be
 * lost below 2^32 words), then the 0..3 byte tail as a 16-bit word and a low
 * byte, then an end-around-carry add of `initial`.  The accumulator is
 * congruent to (initial + sum of LE 16-bit words) mod 0xFFFF and is zero only
 * when initial and every byte are zero, so it folds to the reference value. */
uint64_t orc_nofold_scalar(const uint8_t *b, size_t n, uint64_t initial) {
    uint64_t acc = 0;
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        uint32_t w;
        memcpy(&w, b + i, 4);
        acc += w;
    }
    if (n - i >= 2) {
        uint16_t w;
        memcpy(&w, b + i, 2);
        acc += w;
        i += 2;
    }
    if (n - i == 1)
        acc += b[i]; /* low byte on little-endian (checksum.hpp:69-77) */
    return add_eac(acc, initial);
}

/* The AVX2 arm of the same dispatch (include/netio/checksum.hpp:88-91:
 * fastcsum_nofold_vec256_align when AVX2 is available and the span is long).
 * fastcsum is un-vendored, so this is this repository's own
 * vector kernel with the same contract: per 32-B load, each 64-bit lane is
 * split into its two LE 32-bit words (mask / shift) and both are added into
 * 64-bit accumulator lanes (no lane can overflow below 2^31 iterations), so
 * the result is congruent mod 0xFFFF to the scalar sum and zero only when
 * every byte is.  It is the CPU BASELINE's nofold (bench.py cpu_baseline);
 * tests/test_oracle_golden.py pins it to the reference goldens and to
 * orc_nofold_scalar. */
#include <immintrin.h>

__attribute__((target("avx2"))) static uint64_t nofold_avx2(const uint8_t *b, size_t n, uint64_t initial) {
    const __m256i m32 = _mm256_set1_epi64x(0xffffffffll);
    __m256i a0 = _mm256_setzero_si256(), a1 = _mm256_setzero_si256();
    __m256i a2 = _mm256_setzero_si256(), a3 = _mm256_setzero_si256();
    __m256i b0 = _mm256_setzero_si256(), b1 = _mm256_setzero_si256();
    __m256i b2 = _mm256_setzero_si256(), b3 = _mm256_setzero_si256();
    while (n >= 128) {  /* two independent accumulator sets: 8 add chains in flight */
        const __m256i v0 = _mm256_loadu_si256((const __m256i *)b);
        const __m256i v1 = _mm256_loadu_si256((const __m256i *)(b + 32));
        const __m256i v2 = _mm256_loadu_si256((const __m256i *)(b + 64));
        const __m256i v3 = _mm256_loadu_si256((const __m256i *)(b + 96));
        a0 = _mm256_add_epi64(a0, _mm256_and_si256(v0, m32));
        a1 = _mm256_add_epi64(a1, _mm256_srli_epi64(v0, 32));
        a2 = _mm256_add_epi64(a2, _mm256_and_si256(v1, m32));
        a3 = _mm256_add_epi64(a3, _mm256_srli_epi64(v1, 32));
        b0 = _mm256_add_epi64(b0, _mm256_and_si256(v2, m32));
        b1 = _mm256_add_epi64(b1, _mm256_srli_epi64(v2, 32));
        b2 = _mm256_add_epi64(b2, _mm256_and_si256(v3, m32));
        b3 = _mm256_add_epi64(b3, _mm256_srli_epi64(v3, 32));
        b += 128;
        n -= 128;
    }
    a0 = _mm256_add_epi64(a0, b0);
    a1 = _mm256_add_epi64(a1, b1);
    a2 = _mm256_add_epi64(a2, b2);
    a3 = _mm256_add_epi64(a3, b3);
    while (n >= 64) {
        const __m256i v0 = _mm256_loadu_si256((const __m256i *)b);
        const __m256i v1 = _mm256_loadu_si256((const __m256i *)(b + 32));
        a0 = _mm256_add_epi64(a0, _mm256_and_si256(v0, m32));
        a1 = _mm256_add_epi64(a1, _mm256_srli_epi64(v0, 32));
        a2 = _mm256_add_epi64(a2, _mm256_and_si256(v1, m32));
        a3 = _mm256_add_epi64(a3, _mm256_srli_epi64(v1, 32));
        b += 64;
        n -= 64;
    }
    const __m256i t = _mm256_add_epi64(_mm256_add_epi64(a0, a1), _mm256_add_epi64(a2, a3));
    uint64_t lanes[4];
    _mm256_storeu_si256((__m256i *)lanes, t);
    uint64_t acc = add_eac(add_eac(lanes[0], lanes[1]), add_eac(lanes[2], lanes[3]));
    /* the < 64-byte tail: 64 is even, so its pairing is unchanged */
    return orc_nofold_scalar(b, n, add_eac(acc, initial));
}

static int g_have_avx2 = -1;

uint64_t orc_nofold(const uint8_t *b, size_t n, uint64_t initial) {
    if (n >= 256) {
        if (g_have_avx2 < 0)
            g_have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
        if (g_have_avx2)
            return nofold_avx2(b, n, initial);
    }
    return orc_nofold_scalar(b, n, initial);
}

int orc_have_avx2(void) {
    if (g_have_avx2 < 0)
        g_have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
    return g_have_avx2;
}

/* fastcsum_fold_complement: 64 -> 32 -> 16 with end-around carry, then ~. */
uint16_t orc_fold_complement(uint64_t sum) {
    uint64_t s = (sum & 0xffffffffu) + (sum >> 32);
    s = (s & 0xffffffffu) + (s >> 32);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    return (uint16_t)(~s & 0xffffu);
}

/* include/netio/checksum.hpp:146-149 */
uint16_t orc_checksum(const uint8_t *b, size_t n, uint64_t initial) {
    return orc_fold_complement(orc_nofold(b, n, initial));
}

/* include/netio/checksum.hpp:102-116: sum(src) + sum(dst) + the 4 bytes
 * {0x00, proto, l4Len>>8, l4Len&0xff} (store_big_u16 at :112-113). */
uint64_t orc_pseudo_header_nofold(uint8_t proto, const uint8_t *src, const uint8_t *dst,
                                  size_t addrlen, uint16_t l4len) {
    uint8_t tail[4] = {0, proto, (uint8_t)(l4len >> 8), (uint8_t)(l4len & 0xff)};
    uint64_t sum = orc_nofold(src, addrlen, 0);
    sum = orc_nofold(dst, addrlen, sum);
    return orc_nofold(tail, 4, sum);
}

/* include/netio/checksum.hpp:120-144 */
uint16_t orc_pseudo_header_checksum(uint8_t proto, const uint8_t *src, const uint8_t *dst,
                                    size_t addrlen, uint16_t l4len) {
    return orc_fold_complement(orc_pseudo_header_nofold(proto, src, dst, addrlen, l4len));
}

/* checksum.cpp:8-36.  v6 addresses at offsetof(ip6_hdr, ip6_src) = 8 and
 * +16 (:14-18); v4 at offsetof(struct ip, ip_src) = 12 and +4 (:24-28);
 * proto = istcp ? 6 : 17; l4Len = (uint16_t)(len - csum_start) (:23,33);
 * body = checksum(ippkt.subspan(csum_start), pseudo) (:35). */
uint16_t orc_calc_l4_checksum(const uint8_t *pkt, size_t len, int isv6, int istcp,
                              uint16_t csum_start) {
    const size_t ao = isv6 ? 8 : 12;
    const size_t al = isv6 ? 16 : 4;
    uint8_t src[16] = {0}, dst[16] = {0};
    for (size_t j = 0; j < al; j++) {
        if (ao + j < len)
            src[j] = pkt[ao + j];
        if (ao + al + j < len)
            dst[j] = pkt[ao + al + j];
    }
    uint64_t s = orc_pseudo_header_nofold(istcp ? 6 : 17, src, dst, al,
                                          (uint16_t)(len - csum_start));
    if (csum_start >= len)
        return orc_fold_complement(s);
    return orc_checksum(pkt + csum_start, len - csum_start, s);
}

/* Decap verify gates: evaluator.hpp:112-149 -> evaluator.cpp:14-58 ->
 * evaluator.hpp:59-65 (TCP) / :89-94 (UDP).  Only the checksum-related
 * decisions; GRO policy after them (TCP flag and doff rules, ECN, has_uso)
 * stays with the caller.  l4_out (optional) gets calc_l4_checksum when an L4
 * checksum was computed, else 0. */
uint8_t orc_verify(const uint8_t *pkt, size_t len, uint16_t *l4_out) {
    uint8_t v = 0;
    if (l4_out)
        *l4_out = 0;
    if (len < 1)
        return 0;
    const int isv6 = (pkt[0] >> 4) == 6;
    if (isv6)
        v |= ORC_V_V6;
    const size_t ihs = isv6 ? 40 : 20;
    if (len < ihs || len > 65535) /* evaluator.hpp:118-121 */
        return v;
    uint8_t proto;
    if (!isv6) {
        if ((pkt[0] & 0x0f) * 4u != 20) /* ip_hl, evaluator.cpp:19 */
            return v;
        if (len != (size_t)((pkt[2] << 8) | pkt[3])) /* ip_len, :21 */
            return v;
        if (((pkt[6] << 8) | pkt[7]) & ~0x4000) /* ip_off & ~IP_DF, :24 */
            return v;
        if (orc_checksum(pkt, 20, 0)) /* :27 */
            return v;
        proto = pkt[9];
    } else {
        if (len - 40 != (size_t)((pkt[4] << 8) | pkt[5])) /* ip6_plen, :47 */
            return v;
        proto = pkt[6];
    }
    v |= ORC_V_IP_OK;
    if (proto == 6) {
        v |= ORC_V_TCP;
        if (len - ihs <= 20) /* evaluator.hpp:61 */
            return v;
        uint16_t c = orc_calc_l4_checksum(pkt, len, isv6, 1, (uint16_t)ihs);
        if (l4_out)
            *l4_out = c;
        if (!c)
            v |= ORC_V_L4_OK;
    } else if (proto == 17) {
        v |= ORC_V_UDP;
        if (len - ihs <= 8) /* evaluator.hpp:91 */
            return v;
        uint16_t c = orc_calc_l4_checksum(pkt, len, isv6, 0, (uint16_t)ihs);
        if (l4_out)
            *l4_out = c;
        if (!c)
            v |= ORC_V_L4_OK;
    }
    return v;
}

/* ------------------------------------------------------------------------ */
/* Batched drivers                                                          */
/* ------------------------------------------------------------------------ */

typedef struct {
    int kind; /* 0 uniform l4, 1 desc l4, 2 desc checksum, 3 desc verify */
    const uint8_t *base;
    uint64_t total_len;
    uint32_t segment_size;
    uint16_t csum_start;
    uint32_t flags;
    const orc_pkt_desc *desc;
    uint16_t *out;
    uint8_t *verdict;
    uint8_t *wbase;
    orc_gro_desc *gdesc;
    const orc_gso_desc *sdesc;
    int8_t *status;
    uint64_t lo, hi;
    uint64_t acc; /* kind 7 (read probe): the words' sum, kept live */
} job_t;

static void run_job(job_t *j) {
    if (j->kind == 8) {
        /* NUMA re-touch: copy 4-KiB pages [lo, hi) back from the saved copy
         * (j->base) into the dropped range (j->wbase): the worker's first
         * write places each page on its own node */
        memcpy(j->wbase + j->lo * 4096u, j->base + j->lo * 4096u, (size_t)(j->hi - j->lo) * 4096u);
        return;
    }
    if (j->kind == 7) {
        /* read probe: 64-bit words of 4-KiB blocks [lo, hi) (vectorised by the
         * compiler: the memory path of these CPUs, no checksum work).  Summed
         * in registers and stored once: the jobs share cache lines, and a
         * store per block made the workers bounce them (round 6's first probe
         * read 173 GiB/s on 16 cores where the checksum itself ran 316) */
        uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        const uint64_t *w = (const uint64_t *)(j->base + j->lo * 4096u);
        const uint64_t *e = (const uint64_t *)(j->base + j->hi * 4096u);
        for (; w < e; w += 4) {
            a0 += w[0];
            a1 += w[1];
            a2 += w[2];
            a3 += w[3];
        }
        j->acc = a0 + a1 + a2 + a3;
        return;
    }
    for (uint64_t i = j->lo; i < j->hi; i++) {
        if (j->kind == 0) {
            uint64_t off = i * (uint64_t)j->segment_size;
            uint64_t len = j->total_len - off;
            if (len > j->segment_size)
                len = j->segment_size;
            j->out[i] = orc_calc_l4_checksum(j->base + off, (size_t)len, j->flags & 1,
                                             (j->flags >> 1) & 1, j->csum_start);
        } else if (j->kind == 1) {
            const orc_pkt_desc *d = &j->desc[i];
            j->out[i] = orc_calc_l4_checksum(j->base + d->offset, d->len, d->flags & 1,
                                             (d->flags >> 1) & 1, d->csum_start);
        } else if (j->kind == 2) {
            const orc_pkt_desc *d = &j->desc[i];
            j->out[i] = orc_checksum(j->base + d->offset, d->len, 0);
        } else if (j->kind == 3) {
            const orc_pkt_desc *d = &j->desc[i];
            j->verdict[i] = orc_verify(j->base + d->offset, d->len, j->out ? &j->out[i] : NULL);
        } else if (j->kind == 5) {
            const orc_gso_desc *d = &j->sdesc[i];
            orc_vnet_hdr v = d->vnet;
            orc_gso_result r;
            j->status[i] = (int8_t)orc_gso_split(j->wbase + d->in_offset, d->in_len, &v,
                                                 (uint8_t *)j->base + d->out_offset, d->out_cap, &r);
        } else {
            orc_gro_desc *d = &j->gdesc[i];
            d->status = (int8_t)orc_gro_finalize(j->wbase + d->hdr_offset, d->hdr_len, d->csum_start,
                                                 d->csum_offset, d->flags & 1, (d->flags >> 1) & 1,
                                                 d->payload_bytes);
        }
    }
}

#define ORC_MAX_THREADS 256

/* Persistent worker pool for the timed parallel runs (bench.py's CPU
 * baseline calls the same function back to back for seconds; a 64-B verify or
 * GRO call is ~1 ms of work, and creating + pinning + joining 16 threads per
 * call put the neighbours' scheduling noise into every repetition).  Workers
 * are created pinned (orc_spawn) and kept; a new thread count or a new
 * ORC_CPUS list (bench.py re-picks the quietest CPUs before each repetition)
 * rebuilds the pool.  Calls are serialised by pool_mu: the oracle is driven
 * from one thread. */
static struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    pthread_t tid[ORC_MAX_THREADS];
    job_t *jobs;
    int threads;
    unsigned long gen;   /* bumped per call (and to stop the workers: stop = 1) */
    int pending, stop;
    char cpus[4096];     /* the ORC_CPUS the workers were pinned under */
    pid_t pid;           /* the process that made them (a forked child has none) */
} pool = {.mu = PTHREAD_MUTEX_INITIALIZER, .go = PTHREAD_COND_INITIALIZER, .done = PTHREAD_COND_INITIALIZER};
static pthread_mutex_t pool_mu = PTHREAD_MUTEX_INITIALIZER;

typedef struct {
    int idx;
    unsigned long seen;  /* pool.gen when the worker was made: it runs the calls after that */
} worker_arg;
static worker_arg pool_args[ORC_MAX_THREADS];
/* Per-worker busy time and calls since the last orc_pool_stats_reset (the
 * CPU baseline's per-worker rates: a worker's share of the bytes over its own
 * busy time, so a slow CPU or a straggler shows against the others). */
static uint64_t pool_busy_ns[ORC_MAX_THREADS], pool_calls[ORC_MAX_THREADS];

static uint64_t mono_ns(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static void *pool_worker(void *arg) {
    const int idx = ((worker_arg *)arg)->idx;
    unsigned long seen = ((worker_arg *)arg)->seen;
    pthread_mutex_lock(&pool.mu);
    for (;;) {
        while (pool.gen == seen && !pool.stop)
            pthread_cond_wait(&pool.go, &pool.mu);
        if (pool.stop)
            break;
        seen = pool.gen;
        job_t *j = &pool.jobs[idx];
        pthread_mutex_unlock(&pool.mu);
        const uint64_t t0 = mono_ns();
        run_job(j);
        const uint64_t t1 = mono_ns();
        pthread_mutex_lock(&pool.mu);
        pool_busy_ns[idx] += t1 - t0;
        pool_calls[idx]++;
        if (--pool.pending == 0)
            pthread_cond_signal(&pool.done);
    }
    pthread_mutex_unlock(&pool.mu);
    return NULL;
}

static void pool_stop(void) {
    if (!pool.threads)
        return;
    pthread_mutex_lock(&pool.mu);
    pool.stop = 1;
    pthread_cond_broadcast(&pool.go);
    pthread_mutex_unlock(&pool.mu);
    for (int t = 0; t < pool.threads; t++)
        pthread_join(pool.tid[t], NULL);
    pool.threads = 0;
    pool.stop = 0;
}

static void run_parallel_acc(job_t proto, uint64_t n, int threads, uint64_t *acc) {
    if (threads < 1)
        threads = 1;
    if (threads > ORC_MAX_THREADS)
        threads = ORC_MAX_THREADS;
    if ((uint64_t)threads > n)
        threads = n ? (int)n : 1;
    if (threads == 1 && !orc_pin_single()) {
        proto.lo = 0;
        proto.hi = n;
        run_job(&proto);
        if (acc)
            *acc += proto.acc;
        return;
    }
    job_t jobs[ORC_MAX_THREADS];
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
    }
    pthread_mutex_lock(&pool_mu);
    if (pool.threads && pool.pid != getpid())
        pool.threads = 0;  /* forked: the parent's workers do not exist here */
    const char *cpus = getenv("ORC_CPUS");
    if (!cpus)
        cpus = "";
    if (pool.threads != threads || strncmp(pool.cpus, cpus, sizeof pool.cpus) != 0) {
        pool_stop();
        strncpy(pool.cpus, cpus, sizeof pool.cpus - 1);
        pool.cpus[sizeof pool.cpus - 1] = 0;
        int made = 0;
        for (int t = 0; t < threads; t++) {
            pool_args[t].idx = t;
            pool_args[t].seen = pool.gen;
            if (orc_spawn(&pool.tid[t], t, pool_worker, &pool_args[t]) != 0)
                break;
            made++;
        }
        pool.threads = made;
        pool.pid = getpid();
        if (made != threads) {  /* no pool: run here */
            pool_stop();
            pthread_mutex_unlock(&pool_mu);
            for (int t = 0; t < threads; t++) {
                run_job(&jobs[t]);
                if (acc)
                    *acc += jobs[t].acc;
            }
            return;
        }
    }
    pthread_mutex_lock(&pool.mu);
    pool.jobs = jobs;
    pool.pending = threads;
    pool.gen++;
    pthread_cond_broadcast(&pool.go);
    while (pool.pending)
        pthread_cond_wait(&pool.done, &pool.mu);
    pthread_mutex_unlock(&pool.mu);
    pthread_mutex_unlock(&pool_mu);
    if (acc)
        for (int t = 0; t < threads; t++)
            *acc += jobs[t].acc;
}

static void run_parallel(job_t proto, uint64_t n, int threads) { run_parallel_acc(proto, n, threads, NULL); }

void orc_l4_uniform(const uint8_t *base, uint64_t total_len, uint32_t segment_size,
                    uint16_t csum_start, uint32_t flags, uint16_t *out, int threads) {
    if (!segment_size)
        return;
    job_t j = {0};
    j.kind = 0;
    j.base = base;
    j.total_len = total_len;
    j.segment_size = segment_size;
    j.csum_start = csum_start;
    j.flags = flags;
    j.out = out;
    /* nr_segments(): include/worker/offload.hpp:26-28 */
    uint64_t n = (total_len + segment_size - 1) / segment_size;
    run_parallel(j, n, threads);
}

void orc_l4_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n, uint16_t *out,
                 int threads) {
    job_t j = {0};
    j.kind = 1;
    j.base = base;
    j.desc = desc;
    j.out = out;
    run_parallel(j, n, threads);
}

void orc_checksum_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n,
                       uint16_t *out, int threads) {
    job_t j = {0};
    j.kind = 2;
    j.base = base;
    j.desc = desc;
    j.out = out;
    run_parallel(j, n, threads);
}

void orc_verify_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n, uint8_t *verdict, uint16_t *l4,
                     int threads) {
    job_t j = {0};
    j.kind = 3;
    j.base = base;
    j.desc = desc;
    j.out = l4;
    j.verdict = verdict;
    run_parallel(j, n, threads);
}

void orc_gro_finalize_desc(uint8_t *base, orc_gro_desc *desc, uint64_t n, int threads) {
    job_t j = {0};
    j.kind = 4;
    j.wbase = base;
    j.gdesc = desc;
    run_parallel(j, n, threads);
}

void orc_gso_split_desc(uint8_t *in_base, const orc_gso_desc *desc, uint64_t n, uint8_t *out_base, int8_t *status,
                        int threads) {
    job_t j = {0};
    j.kind = 5;
    j.wbase = in_base;
    j.base = out_base;
    j.sdesc = desc;
    j.status = status;
    run_parallel(j, n, threads);
}

void orc_pool_stats_reset(void) {
    pthread_mutex_lock(&pool.mu);
    memset(pool_busy_ns, 0, sizeof pool_busy_ns);
    memset(pool_calls, 0, sizeof pool_calls);
    pthread_mutex_unlock(&pool.mu);
}

int orc_pool_stats(uint64_t *busy_ns, uint64_t *calls, int max) {
    pthread_mutex_lock(&pool.mu);
    const int n = pool.threads < max ? pool.threads : max;
    for (int t = 0; t < n; t++) {
        busy_ns[t] = pool_busy_ns[t];
        calls[t] = pool_calls[t];
    }
    pthread_mutex_unlock(&pool.mu);
    return n;
}

uint64_t orc_read_probe(const uint8_t *base, uint64_t nbytes, int threads) {
    job_t j = {0};
    j.kind = 7;
    j.base = base;
    const uint64_t n = nbytes / 4096u;
    uint64_t acc = 0;
    run_parallel_acc(j, n, threads, &acc);
    return acc;
}

int orc_numa_retouch(uint8_t *buf, uint64_t nbytes, int threads) {
    /* The buffer's whole pages moved to the nodes of the workers that will
     * read them (the CPU baseline's pinned pool, ORC_CPUS): saved, dropped
     * (MADV_DONTNEED: private anonymous pages refault on first touch), and
     * copied back by the workers, page range t to worker t as run_parallel
     * splits units.  Contents unchanged.  Returns 0, or -1 when the range
     * cannot be dropped (the buffer is then left as it was). */
    const uintptr_t ps = 4096u;
    const uintptr_t a0 = ((uintptr_t)buf + ps - 1) & ~(ps - 1);
    const uintptr_t a1 = ((uintptr_t)buf + nbytes) & ~(ps - 1);
    if (a1 <= a0)
        return 0;
    const uint64_t n = (uint64_t)(a1 - a0);
    uint8_t *save = (uint8_t *)malloc(n);
    if (!save)
        return -1;
    memcpy(save, (void *)a0, n);
    if (madvise((void *)a0, n, MADV_DONTNEED) != 0) {
        free(save);
        return -1;
    }
    job_t j = {0};
    j.kind = 8;
    j.base = save;
    j.wbase = (uint8_t *)a0;
    run_parallel(j, n / ps, threads);
    free(save);
    return 0;
}

double orc_time_l4_uniform(const uint8_t *base, uint64_t total_len, uint32_t segment_size,
                           uint16_t csum_start, uint32_t flags, uint16_t *out, int threads,
                           int reps) {
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int r = 0; r < reps; r++)
        orc_l4_uniform(base, total_len, segment_size, csum_start, flags, out, threads);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* ------------------------------------------------------------------------ */
/* GSO split: worker/offload.cpp:46-216                                     */
/* ------------------------------------------------------------------------ */

static inline uint16_t ld_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t ld_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline void st_be16(uint8_t *p, uint16_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
static inline void st_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

#define VNET_F_NEEDS_CSUM 1
#define VNET_GSO_NONE 0
#define VNET_GSO_TCPV4 1
#define VNET_GSO_TCPV6 4
#define VNET_GSO_UDP_L4 5 /* include/worker/offload.hpp:11-15 */
#define VNET_GSO_ECN 0x80

int orc_gso_split(uint8_t *in, size_t in_len, orc_vnet_hdr *v, uint8_t *out, size_t out_cap,
                  orc_gso_result *res) {
    memset(res, 0, sizeof(*res));
    const size_t cs = v->csum_start;
    const size_t l4off = (size_t)v->csum_start + v->csum_offset; /* :47 */
    /* Out of contract (-3) = inputs the reference reads out of bounds on, or
     * whose header geometry makes its fixups overlap the IP header: a packet
     * shorter than its fixed IP header, csum_start inside the fixed IP
     * header, or a checksum field outside the L4 header. */
    if (in_len < 1)
        return -3;
    const int isv6 = (in[0] >> 4) == 6; /* :48 */
    const size_t iph_min = isv6 ? 40u : 20u;
    if (in_len < iph_min)
        return -3;
    /* :49-53, IPTOS_ECN = & 0x03 */
    const uint8_t ecn = isv6 ? (uint8_t)((ld_be32(in) >> 20) & 3) : (uint8_t)(in[1] & 3);
    res->isv6 = (uint8_t)isv6;
    res->ecn = ecn;
    res->out_len = in_len;
    res->segment_size = in_len;
    res->passthrough = 1;
    res->hdr_len = v->hdr_len;

    switch (v->gso_type & ~VNET_GSO_ECN) { /* :55 */
    case VNET_GSO_NONE:
        if (v->flags & VNET_F_NEEDS_CSUM) { /* :56-78 */
            if (cs < iph_min || cs > in_len || l4off + 2 > in_len)
                return -3;
            if (!isv6) {
                in[10] = 0; /* ip_sum */
                in[11] = 0;
            }
            in[l4off] = 0;
            in[l4off + 1] = 0;
            int istcp = isv6 ? in[6] == 6 : in[9] == 6; /* ip6_nxt / ip_p */
            if (!isv6) {
                uint16_t c = orc_checksum(in, cs, 0);
                memcpy(in + 10, &c, 2); /* native order, :72-73 */
            }
            uint16_t l4 = orc_calc_l4_checksum(in, in_len, isv6, istcp, (uint16_t)cs);
            memcpy(in + l4off, &l4, 2);
        }
        return 0;
    case VNET_GSO_TCPV4:
    case VNET_GSO_TCPV6: {
        if (cs > in_len)
            return -3; /* :91 would wrap and read past the buffer */
        if (in_len - cs < 20) /* :91 */
            return 0;
        size_t thlen = 4u * (in[cs + 12] >> 4); /* tcphdr.doff, :100 */
        if (thlen < 20)                          /* :101 */
            return 0;
        v->hdr_len = (uint16_t)(cs + thlen); /* :110 */
        break;
    }
    case VNET_GSO_UDP_L4:
        v->hdr_len = (uint16_t)(cs + 8); /* :114 */
        break;
    default:
        return 0; /* :116-123 */
    }
    res->hdr_len = v->hdr_len;
    const size_t hdr_len = v->hdr_len;
    if (in_len < hdr_len) /* :126-134 */
        return 0;
    if (cs < iph_min || l4off < cs || l4off + 2 > hdr_len)
        return -3;

    const size_t rest_len = in_len - hdr_len;
    const size_t gso = v->gso_size;
    if (rest_len && !gso)
        return -1; /* the reference loops forever (:157-158) */
    const size_t nseg = gso ? (rest_len + gso - 1) / gso : 0;
    if (out_cap < in_len + nseg * hdr_len) /* reserve_size assert, :139-143 */
        return -2;

    if (!isv6) { /* :145-147 */
        in[10] = 0;
        in[11] = 0;
    }
    in[l4off] = 0; /* :149 */
    in[l4off + 1] = 0;

    const int istcp = v->gso_type == VNET_GSO_TCPV4 || v->gso_type == VNET_GSO_TCPV6; /* :151 */
    uint32_t seq0 = istcp ? ld_be32(in + cs + 4) : 0;                                   /* :152-154 */

    const uint8_t *rest = in + hdr_len;
    size_t remaining = rest_len, pb = 0;
    for (size_t i = 0; remaining; i++) { /* :157-208 */
        size_t datalen = remaining < gso ? remaining : gso;
        size_t pktlen = hdr_len + datalen;
        uint8_t *seg = out + pb;
        pb += pktlen;
        memcpy(seg, in, hdr_len);            /* :165 */
        memcpy(seg + hdr_len, rest, datalen); /* :166 */
        if (isv6) {
            st_be16(seg + 4, (uint16_t)(pktlen - cs)); /* ip6_plen, :168-172 */
        } else {
            if (i)
                st_be16(seg + 4, (uint16_t)(ld_be16(seg + 4) + i)); /* ip_id, :178-182 */
            st_be16(seg + 2, (uint16_t)pktlen);                     /* ip_len, :183 */
            uint16_t c = orc_checksum(seg, cs, 0);                  /* :184 */
            memcpy(seg + 10, &c, 2);
        }
        if (istcp) {
            st_be32(seg + cs + 4, (uint32_t)(seq0 + gso * i)); /* :190-192 */
            if (datalen < remaining)
                seg[cs + 13] &= (uint8_t)~0x09; /* fin, psh: :193-195 */
        } else {
            st_be16(seg + cs + 4, (uint16_t)(pktlen - cs)); /* udp->len, :197-199 */
        }
        uint16_t l4 = orc_calc_l4_checksum(seg, pktlen, isv6, istcp, (uint16_t)cs); /* :202 */
        memcpy(seg + l4off, &l4, 2);
        rest += datalen;
        remaining -= datalen;
    }
    res->passthrough = 0;
    res->out_len = pb;                      /* :210-215 */
    res->segment_size = hdr_len + gso;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* GRO finalize: include/worker/flowkey_ref.hpp:82-117                      */
/* ------------------------------------------------------------------------ */

int orc_gro_finalize(uint8_t *hdr, size_t hdr_len, uint16_t csum_start, uint16_t csum_offset, int isv6,
                     int istcp, uint64_t payload_bytes) {
    const size_t cs = csum_start, l4off = (size_t)csum_start + csum_offset;
    const size_t iph = isv6 ? 40 : 20;
    if (cs < iph || cs > hdr_len || l4off < cs || l4off + 2 > hdr_len || (!istcp && cs + 8 > hdr_len))
        return -3;
    const uint64_t l4len = hdr_len - cs + payload_bytes; /* :84 */
    if (!istcp)
        st_be16(hdr + cs + 4, (uint16_t)l4len); /* udp->len, :85-86 */
    size_t proto_off, src_off, dst_off, alen;
    if (isv6) {
        proto_off = 6; src_off = 8; dst_off = 24; alen = 16; /* :89-93 */
        st_be16(hdr + 4, (uint16_t)l4len);                  /* ip6_plen, :95 */
    } else {
        proto_off = 9; src_off = 12; dst_off = 16; alen = 4; /* :97-100 */
        st_be16(hdr + 2, (uint16_t)(hdr_len + payload_bytes)); /* ip_len, :103 */
        hdr[10] = 0;                                           /* :104 */
        hdr[11] = 0;
        uint16_t c = orc_checksum(hdr, cs, 0); /* :106, native order */
        memcpy(hdr + 10, &c, 2);
    }
    uint16_t seed = orc_pseudo_header_checksum(hdr[proto_off], hdr + src_off, hdr + dst_off, alen,
                                               (uint16_t)l4len); /* :108-112 (intended) */
    memcpy(hdr + l4off, &seed, 2); /* native order, :114 */
    return 0;
}
