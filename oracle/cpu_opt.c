/*
 * cpu_opt.c — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * The "optimised multi-threaded CPU codec" row of BASELINE.md / SURVEY §8(d):
 * the same byte work as the reference's codec (src/format.rs:23-77) written
 * the way a tuned CPU implementation would, on all the host cores it is
 * given -- no per-record allocation, spans instead of owned copies, and the
 * serial cursor walk of deserialize_from_bytes (src/format.rs:54-58) split
 * into byte ranges whose entries are guessed and then handed over in order
 * (a wrong guess is redone from the exact entry), as the GPU engine does.
 * Results are checked against hgo_decode / hgo_encode by the tests.
 */
#define _POSIX_C_SOURCE 200112L
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "horreum_oracle.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static inline uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8); /* little-endian host (x86-64 / aarch64) */
    return v;
}

/* Record at pos readable as the reference would read it (src/format.rs:63-69). */
static inline int rec_ok(const uint8_t* b, uint64_t len, uint64_t pos, uint64_t* next) {
    if (len - pos < 16) return 0;
    const uint64_t k = ld64(b + pos), v = ld64(b + pos + 8);
    if (k > UINT64_MAX - v || k + v > len - pos - 16) return 0;
    if ((k >> 32) | (v >> 32)) return 0;
    *next = pos + 16 + k + v;
    return 1;
}

/* Serial walk of the records starting in [x, stop): spans to out (<= cap),
 * count, exit.  Returns 0, or the error kind at *err_pos. */
static int walk_range(const uint8_t* b, uint64_t len, uint64_t x, uint64_t stop, hg_span* out,
                      uint64_t cap, uint64_t* cnt, uint64_t* exit, uint64_t* err_pos) {
    uint64_t n = 0, pos = x;
    int kind = HG_OK;
    while (pos < stop) {
        if (len - pos < 16) { kind = HG_ERR_TRUNCATED_HEADER; break; }
        const uint64_t k = ld64(b + pos), v = ld64(b + pos + 8);
        if (k > UINT64_MAX - v) { kind = HG_ERR_LEN_OVERFLOW; break; }
        if (k + v > len - pos - 16) { kind = HG_ERR_TRUNCATED_BODY; break; }
        if ((k >> 32) | (v >> 32)) { kind = HG_ERR_SPAN_RANGE; break; }
        if (n < cap) {
            out[n].off = pos;
            out[n].klen = (uint32_t)k;
            out[n].vlen = (uint32_t)v;
        }
        ++n;
        pos += 16 + k + v;
    }
    *cnt = n;
    *exit = pos;
    *err_pos = pos;
    return kind;
}

/* Guess of the first record start at or after b0: the first position whose
 * record and the next three chain as readable records (or reach len). */
static uint64_t guess_entry(const uint8_t* b, uint64_t len, uint64_t b0) {
    for (uint64_t p = b0; p + 16 <= len; ++p) {
        uint64_t q = p, nx;
        int ok = 1;
        for (int h = 0; h < 4 && q < len; ++h) {
            if (!rec_ok(b, len, q, &nx)) { ok = 0; break; }
            q = nx;
        }
        if (ok) return p;
    }
    return len;
}

/* Every multi-threaded entry below spawns its workers first and starts the
 * clock when all of them stand at a barrier (a service keeps a thread pool:
 * thread creation is not codec work), then runs its phases between barriers
 * with thread 0 (the caller) doing the short serial steps. */
typedef struct {
    const uint8_t* b;
    uint64_t len, lo, hi, guess, cnt, exit, err_pos, dst;
    hg_span* out;
    hg_span* spans;
    uint64_t cap, total_cap;
    int kind, place;
} range_job;

typedef struct {
    pthread_barrier_t bar;
    uint32_t nthreads;
    void* jobs;
    void (*phase[3])(void* job); /* run by every thread, a barrier after each */
    void (*serial[3])(void* pool); /* thread 0 between phase i and i + 1 (nullable) */
    size_t job_bytes;
    double t0;
} pool_run;

typedef struct {
    pool_run* p;
    uint32_t t;
} pool_arg;

static void pool_body(pool_run* p, uint32_t t) {
    pthread_barrier_wait(&p->bar);
    if (t == 0) p->t0 = now_s();
    pthread_barrier_wait(&p->bar);
    for (int i = 0; i < 3 && p->phase[i]; ++i) {
        p->phase[i]((char*)p->jobs + p->job_bytes * t);
        pthread_barrier_wait(&p->bar);
        if (t == 0 && p->serial[i]) p->serial[i](p);
        pthread_barrier_wait(&p->bar);
    }
}

static void* pool_thread(void* arg) {
    pool_arg* a = (pool_arg*)arg;
    pool_body(a->p, a->t);
    return NULL;
}

/* Runs p over p->nthreads threads; returns seconds from the release of the
 * start barrier to the end of the last phase. */
static double pool_go(pool_run* p) {
    pthread_t th[256];
    pool_arg args[256];
    pthread_barrier_init(&p->bar, NULL, p->nthreads);
    for (uint32_t t = 1; t < p->nthreads; ++t) {
        args[t].p = p;
        args[t].t = t;
        pthread_create(&th[t], NULL, pool_thread, &args[t]);
    }
    pool_body(p, 0);
    const double t1 = now_s();
    for (uint32_t t = 1; t < p->nthreads; ++t) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&p->bar);
    return t1 - p->t0;
}

static void range_walk(void* arg) {
    range_job* j = (range_job*)arg;
    j->guess = j->lo ? guess_entry(j->b, j->len, j->lo) : 0;
    j->kind = walk_range(j->b, j->len, j->guess, j->hi, j->out, j->cap, &j->cnt, &j->exit,
                         &j->err_pos);
}

/* thread 0: the entry handoff in order (a range entered off its guess is
 * walked again from the exact entry), then every range's output offset */
static uint64_t g_dec_total, g_dec_bad;
static void range_handoff(void* pool) {
    pool_run* p = (pool_run*)pool;
    range_job* jobs = (range_job*)p->jobs;
    uint64_t total = 0, bad = 0;
    for (uint32_t t = 0; t < p->nthreads; ++t) {
        range_job* j = &jobs[t];
        j->place = 0;
        if (bad) continue;
        if (t && j->guess != jobs[t - 1].exit) {
            j->guess = jobs[t - 1].exit;
            j->kind = walk_range(j->b, j->len, j->guess, j->hi, j->out, j->cap, &j->cnt, &j->exit,
                                 &j->err_pos);
        }
        j->dst = total;
        j->place = 1;
        total += j->cnt;
        if (j->kind != HG_OK) bad = 1;
    }
    g_dec_total = total;
    g_dec_bad = bad;
}

static void range_place(void* arg) {
    range_job* j = (range_job*)arg;
    if (!j->place || j->dst >= j->total_cap) return;
    const uint64_t m = j->dst + j->cnt <= j->total_cap ? j->cnt : j->total_cap - j->dst;
    if (m) memcpy(j->spans + j->dst, j->out, m * sizeof(hg_span));
}

uint64_t hgo_mt_decode(const uint8_t* bytes, uint64_t len, hg_span* spans, uint64_t cap,
                       hg_span* scratch, uint32_t nthreads, double* seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    static range_job jobs[256];
    for (uint32_t t = 0; t < nthreads; ++t) {
        range_job* j = &jobs[t];
        j->b = bytes;
        j->len = len;
        j->lo = len / nthreads * t;
        j->hi = t + 1 == nthreads ? len : len / nthreads * (t + 1);
        /* a range of W bytes holds <= W/16 + 1 starts; scratch holds
         * len/16 + 2*nthreads + 2 spans, regions never overlap */
        j->out = scratch + j->lo / 16 + 2 * (uint64_t)t;
        j->cap = (j->hi - j->lo) / 16 + 2;
        j->spans = spans;
        j->total_cap = cap;
    }
    pool_run p;
    memset(&p, 0, sizeof p);
    p.nthreads = nthreads;
    p.jobs = jobs;
    p.job_bytes = sizeof(range_job);
    p.phase[0] = range_walk;
    p.serial[0] = range_handoff;
    p.phase[1] = range_place;
    const double secs = pool_go(&p);
    if (seconds) *seconds = secs;
    return g_dec_bad ? UINT64_MAX : g_dec_total;
}

typedef struct {
    const uint8_t* arena;
    const hg_pair* pairs;
    uint64_t lo, hi, base, bytes;
    uint8_t* out;
} enc_job;

static void enc_size_worker(void* arg) {
    enc_job* j = (enc_job*)arg;
    uint64_t s = 0;
    for (uint64_t i = j->lo; i < j->hi; ++i) s += 16 + (uint64_t)j->pairs[i].klen + j->pairs[i].vlen;
    j->bytes = s;
}

static uint64_t g_enc_total;
static void enc_bases(void* pool) {
    pool_run* p = (pool_run*)pool;
    enc_job* jobs = (enc_job*)p->jobs;
    uint64_t base = 0;
    for (uint32_t t = 0; t < p->nthreads; ++t) {
        jobs[t].base = base;
        base += jobs[t].bytes;
    }
    g_enc_total = base;
}

static void enc_copy_worker(void* arg) {
    enc_job* j = (enc_job*)arg;
    uint8_t* o = j->out + j->base;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const hg_pair* p = &j->pairs[i];
        const uint64_t k = p->klen, v = p->vlen;
        memcpy(o, &k, 8);
        memcpy(o + 8, &v, 8);
        memcpy(o + 16, j->arena + p->key_off, k);
        if (v) memcpy(o + 16 + k, j->arena + p->val_off, v);
        o += 16 + k + v;
    }
}

uint64_t hgo_mt_encode(const uint8_t* arena, const hg_pair* pairs, uint64_t n, uint8_t* out,
                       uint32_t nthreads, double* seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    static enc_job jobs[256];
    for (uint32_t t = 0; t < nthreads; ++t) {
        jobs[t].arena = arena;
        jobs[t].pairs = pairs;
        jobs[t].out = out;
        jobs[t].lo = n / nthreads * t;
        jobs[t].hi = t + 1 == nthreads ? n : n / nthreads * (t + 1);
    }
    pool_run p;
    memset(&p, 0, sizeof p);
    p.nthreads = nthreads;
    p.jobs = jobs;
    p.job_bytes = sizeof(enc_job);
    p.phase[0] = enc_size_worker;
    p.serial[0] = enc_bases;
    p.phase[1] = enc_copy_worker;
    const double secs = pool_go(&p);
    if (seconds) *seconds = secs;
    return g_enc_total;
}

/* CPU roofline (BASELINE.md CPU-roof): n bytes copied by nthreads threads,
 * one contiguous slice each (memcpy, the libc's widest path). */
typedef struct {
    uint8_t* dst;
    const uint8_t* src;
    uint64_t n;
} cpy_job;

static void cpy_worker(void* arg) {
    cpy_job* j = (cpy_job*)arg;
    memcpy(j->dst, j->src, j->n);
}

void hgo_mt_memcpy(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t nthreads,
                   double* seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    static cpy_job jobs[256];
    const uint64_t per = (n / nthreads + 63) & ~63ull;
    for (uint32_t t = 0; t < nthreads; ++t) {
        const uint64_t lo = per * t < n ? per * t : n;
        const uint64_t hi = per * (t + 1) < n ? per * (t + 1) : n;
        jobs[t].dst = dst + lo;
        jobs[t].src = src + lo;
        jobs[t].n = hi - lo;
    }
    pool_run p;
    memset(&p, 0, sizeof p);
    p.nthreads = nthreads;
    p.jobs = jobs;
    p.job_bytes = sizeof(cpy_job);
    p.phase[0] = cpy_worker;
    const double secs = pool_go(&p);
    if (seconds) *seconds = secs;
}
