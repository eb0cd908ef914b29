/*
 * horreum_oracle.c — TEST INFRASTRUCTURE ONLY (see horreum_oracle.h).
 *
 * Plain-C restatement of the reference's record codec.  Parity is pinned by
 * the reference's own known-answer vectors (tests/golden/format_vectors.json,
 * transcribed from src/format.rs, src/sstable/{index,storage,table,manager}.rs
 * tests).  The reference's single third-party dependency on this path is
 * bincode 1.3.x (Cargo.toml:9): `bincode::serialize(&usize)` /
 * `deserialize::<usize>` with the default options = 8-byte little-endian
 * fixed-width integers, trailing bytes allowed (pinned by src/format.rs:94,
 * 103, 113-115).
 */
#define _POSIX_C_SOURCE 199309L
#include "horreum_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint64_t rd_le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

static void wr_le64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

/* src/format.rs:50-59 (cursor loop) and :63-77 (one record). */
int hgo_decode(const uint8_t* bytes, uint64_t len, hg_span* spans,
               uint64_t cap, uint64_t* n_out, hg_err* err) {
    uint64_t pos = 0, n = 0;
    int kind = HG_OK;
    /* :54 `while cursor.position() < bytes_length` */
    while (pos < len) {
        /* :64-65 read_exact(16) -> UnexpectedEof */
        if (len - pos < 16) { kind = HG_ERR_TRUNCATED_HEADER; break; }
        /* :66-67 bincode usize = u64 LE */
        uint64_t klen = rd_le64(bytes + pos);
        uint64_t vlen = rd_le64(bytes + pos + 8);
        /* :68 `key_length + value_length` */
        if (klen > UINT64_MAX - vlen) { kind = HG_ERR_LEN_OVERFLOW; break; }
        uint64_t body = klen + vlen;
        /* :69 read_exact(body) -> UnexpectedEof */
        if (body > len - pos - 16) { kind = HG_ERR_TRUNCATED_BODY; break; }
        /* engine limit: span fields are u32 (include/horreum_gpu.h) */
        if (klen > 0xFFFFFFFFull || vlen > 0xFFFFFFFFull) {
            kind = HG_ERR_SPAN_RANGE; break;
        }
        /* :70-75 key = [..k], value = Some iff vlen > 0 (vlen==0 <=> None) */
        if (n < cap) {
            spans[n].off = pos;
            spans[n].klen = (uint32_t)klen;
            spans[n].vlen = (uint32_t)vlen;
        }
        ++n;
        pos += 16 + body;
    }
    if (n_out) *n_out = n;
    if (err) { err->kind = kind; err->reserved = 0; err->offset = kind ? pos : 0; }
    if (kind != HG_OK) return kind;
    return n > cap ? HG_ERR_CAPACITY : HG_OK;
}

/* src/format.rs:23-37 per pair, :40-42 concatenation in the given order,
 * src/sstable/index.rs:55-67 blocks of `block_stride` pairs. */
int hgo_encode(const uint8_t* arena, const hg_pair* pairs, uint64_t n,
               uint8_t* out, uint64_t cap, uint64_t* rec_off,
               uint32_t block_stride, hg_block* blocks, uint64_t* out_len) {
    if (blocks && block_stride == 0) return HG_ERR_INVALID_ARG; /* chunks(0) panics */
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i)
        total += 16 + (uint64_t)pairs[i].klen + (uint64_t)pairs[i].vlen;
    if (out_len) *out_len = total;
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const hg_pair* p = &pairs[i];
        if (rec_off) rec_off[i] = off;
        if (total <= cap) {
            /* :24 key length; :25-28 value length or [0;8] for None */
            wr_le64(out + off, p->klen);
            wr_le64(out + off + 8, p->vlen);
            /* :31 key bytes; :32-34 value bytes iff Some */
            memcpy(out + off + 16, arena + p->key_off, p->klen);
            if (p->vlen) memcpy(out + off + 16 + p->klen, arena + p->val_off, p->vlen);
        }
        off += 16 + (uint64_t)p->klen + (uint64_t)p->vlen;
    }
    if (blocks) {
        /* index.rs:58-65: Block{key: chunk[0].key, position: bytes so far,
         * length: serialize_flatten(chunk).len()} */
        uint64_t nb = (n + block_stride - 1) / block_stride, pos = 0, r = 0;
        for (uint64_t b = 0; b < nb; ++b) {
            uint64_t first = b * block_stride, end = first + block_stride;
            if (end > n) end = n;
            uint64_t length = 0;
            for (r = first; r < end; ++r)
                length += 16 + (uint64_t)pairs[r].klen + (uint64_t)pairs[r].vlen;
            blocks[b].first_rec = first;
            blocks[b].position = pos;
            blocks[b].length = length;
            pos += length;
        }
    }
    return total <= cap ? HG_OK : HG_ERR_CAPACITY;
}

/* Vec<u8> Ord: lexicographic bytes, then shorter first. */
static int key_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
    uint64_t m = al < bl ? al : bl;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

/* src/sstable/index.rs:72-78: binary_search_by_key on block first keys;
 * Ok(pos) -> pos, Err(pos) -> pos-1 if pos > 0 else None.  (With unique
 * first keys every binary-search variant selects the same block.) */
int hgo_index_get(const hg_block* blocks, uint64_t nblocks,
                  const uint8_t* arena, const hg_pair* pairs,
                  const uint8_t* key, uint64_t klen,
                  uint64_t* pos, uint64_t* len) {
    uint64_t lo = 0, hi = nblocks; /* first index with first_key >= key */
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        const hg_pair* p = &pairs[blocks[mid].first_rec];
        if (key_cmp(arena + p->key_off, p->klen, key, klen) < 0) lo = mid + 1;
        else hi = mid;
    }
    uint64_t sel;
    if (lo < nblocks) {
        const hg_pair* p = &pairs[blocks[lo].first_rec];
        if (key_cmp(arena + p->key_off, p->klen, key, klen) == 0) { sel = lo; goto found; }
    }
    if (lo == 0) return 0;
    sel = lo - 1;
found:
    if (pos) *pos = blocks[sel].position;
    if (len) *len = blocks[sel].length;
    return 1;
}

/* Rust's slice::binary_search_by_key over records base + i * step, i in
 * [0, size), as the reference calls it (index.rs:74, table.rs:65).  Rust std
 * 1.52-1.81 (the reference pins no toolchain; this is the implementation
 * current from its tokio-1.0 era on): mid = left + size / 2 with size =
 * right - left, the first probe that compares Equal returns Ok(mid), else
 * Err(left).  The reference's own tests search unique keys only, so which
 * duplicate a search returns is this restatement's choice ("parity unpinned"
 * for duplicate keys).  Returns 1 (Ok) or 0 (Err) and the index in *pos. */
static int rust_search(const uint8_t* data, const hg_span* spans, uint64_t base, uint64_t step,
                       uint64_t size, const uint8_t* key, uint64_t klen, uint64_t* pos) {
    uint64_t left = 0, right = size;
    while (left < right) {
        const uint64_t mid = left + (right - left) / 2;
        const hg_span* s = &spans[base + mid * step];
        const int c = key_cmp(data + s->off + 16, s->klen, key, klen);
        if (c == 0) { *pos = mid; return 1; }
        if (c < 0) left = mid + 1;
        else right = mid;
    }
    *pos = left;
    return 0;
}

/* src/sstable/table.rs:54-70 (SSTable::get) on a decoded table: the block
 * index of Index::new (index.rs:55-67, blocks of `stride` records), its get
 * (index.rs:72-78: Ok(b) of the binary search over the blocks' first keys ->
 * block b, Err(b) -> block b - 1, none if b == 0), then binary_search_by_key
 * over the block's records.  Returns 1 and the record index if found. */
int hgo_table_get(const uint8_t* data, const hg_span* spans, uint64_t n, uint32_t stride,
                  const uint8_t* key, uint64_t klen, uint64_t* rec) {
    if (n == 0 || stride == 0) return 0;
    const uint64_t nb = (n + stride - 1) / stride;
    uint64_t b = 0, j = 0;
    if (!rust_search(data, spans, 0, stride, nb, key, klen, &b)) {
        if (b == 0) return 0;
        --b;
    }
    const uint64_t r0 = b * stride, cnt = n - r0 < stride ? n - r0 : stride;
    if (!rust_search(data, spans, r0, 1, cnt, key, klen, &j)) return 0;
    if (rec) *rec = r0 + j;
    return 1;
}

/* src/sstable/manager.rs:199-234. */
int hgo_compact(uint32_t ntables, const uint8_t* const* datas,
                const hg_span* const* spans, const uint64_t* counts,
                uint32_t* out_table, uint64_t* out_rec, uint64_t cap,
                uint64_t* n_out) {
    uint64_t* head = (uint64_t*)calloc(ntables ? ntables : 1, sizeof(uint64_t));
    uint64_t n = 0;
    int any = 0;
    for (uint32_t t = 0; t < ntables; ++t) any |= counts[t] > 0;
    if (!any) { free(head); if (n_out) *n_out = 0; return HG_ERR_EMPTY_MERGE; } /* :213 unwrap on None */
    for (;;) {
        /* :209-215 min_by_key over Some candidates: the FIRST minimum in
         * iteration order wins, i.e. the newest table. */
        int32_t best = -1;
        const uint8_t* bk = NULL;
        uint64_t bl = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            if (head[t] >= counts[t]) continue;
            const hg_span* s = &spans[t][head[t]];
            const uint8_t* k = datas[t] + s->off + 16;
            if (best < 0 || key_cmp(k, s->klen, bk, bl) < 0) {
                best = (int32_t)t; bk = k; bl = s->klen;
            }
        }
        /* :216-217 push min pair */
        if (n < cap) { out_table[n] = (uint32_t)best; out_rec[n] = head[best]; }
        ++n;
        /* :218-227 advance every iterator whose head key == min_key */
        const uint8_t* mk = bk;
        uint64_t ml = bl;
        int remaining = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            if (head[t] >= counts[t]) continue;
            const hg_span* s = &spans[t][head[t]];
            if (key_cmp(datas[t] + s->off + 16, s->klen, mk, ml) == 0) ++head[t];
        }
        /* :228-230 stop when every candidate is None */
        for (uint32_t t = 0; t < ntables; ++t) remaining |= head[t] < counts[t];
        if (!remaining) break;
    }
    free(head);
    if (n_out) *n_out = n;
    return n > cap ? HG_ERR_CAPACITY : HG_OK;
}

uint64_t hgo_payload_size(const hg_span* spans, uint64_t n) {
    uint64_t s = 0;
    for (uint64_t i = 0; i < n; ++i) s += (uint64_t)spans[i].klen + spans[i].vlen;
    return s;
}

/* ---- CPU baselines with the reference's ownership pattern ---------------- */

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct { uint8_t* key; uint64_t klen; uint8_t* val; uint64_t vlen; } owned_pair;

uint64_t hgo_bench_decode_owned(const uint8_t* bytes, uint64_t len,
                                double* seconds_decode) {
    double t0 = now_s();
    uint64_t n = 0, capv = 0, pos = 0;
    owned_pair* v = NULL; /* let mut pairs = vec![] */
    int bad = 0;
    while (pos < len) {
        uint8_t* lb = (uint8_t*)calloc(16, 1);               /* vec![0; 16] */
        if (len - pos < 16) { free(lb); bad = 1; break; }
        memcpy(lb, bytes + pos, 16);                          /* read_exact */
        uint64_t k = rd_le64(lb), vl = rd_le64(lb + 8);
        if (k > UINT64_MAX - vl || k + vl > len - pos - 16) { free(lb); bad = 1; break; }
        uint8_t* cb = (uint8_t*)calloc(k + vl ? k + vl : 1, 1); /* vec![0; k+v] */
        memcpy(cb, bytes + pos + 16, k + vl);                   /* read_exact */
        owned_pair p;
        p.klen = k; p.key = (uint8_t*)malloc(k ? k : 1); memcpy(p.key, cb, k); /* to_vec */
        p.vlen = vl; p.val = NULL;
        if (vl) { p.val = (uint8_t*)malloc(vl); memcpy(p.val, cb + k, vl); }
        free(cb); free(lb);
        if (n == capv) { capv = capv ? 2 * capv : 4; v = (owned_pair*)realloc(v, capv * sizeof *v); }
        v[n++] = p;                                           /* pairs.push */
        pos += 16 + k + vl;
    }
    double t1 = now_s();
    for (uint64_t i = 0; i < n; ++i) { free(v[i].key); free(v[i].val); }
    free(v);
    if (seconds_decode) *seconds_decode = t1 - t0;
    return bad ? (uint64_t)-1 : n;
}

uint64_t hgo_bench_encode_owned(const uint8_t* arena, const hg_pair* pairs,
                                uint64_t n, double* seconds) {
    double t0 = now_s();
    uint8_t* out = NULL;
    uint64_t olen = 0, ocap = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const hg_pair* p = &pairs[i];
        uint8_t* kl = (uint8_t*)malloc(8); wr_le64(kl, p->klen);   /* serialize(&len) */
        uint8_t* vl = (uint8_t*)malloc(8); wr_le64(vl, p->vlen);   /* or vec![0; 8] */
        uint8_t* kc = (uint8_t*)malloc(p->klen ? p->klen : 1);     /* key.clone() */
        memcpy(kc, arena + p->key_off, p->klen);
        uint8_t* vc = NULL;
        if (p->vlen) { vc = (uint8_t*)malloc(p->vlen); memcpy(vc, arena + p->val_off, p->vlen); }
        uint64_t rl = 16 + (uint64_t)p->klen + p->vlen, bl = 0, bc = 0;
        uint8_t* buf = NULL;                                        /* Vec::new + appends */
        const uint8_t* parts[4] = {kl, vl, kc, vc};
        uint64_t plen[4] = {8, 8, p->klen, p->vlen};
        for (int j = 0; j < 4; ++j) {
            if (!plen[j]) continue;
            while (bl + plen[j] > bc) { bc = bc ? 2 * bc : 8; buf = (uint8_t*)realloc(buf, bc); }
            memcpy(buf + bl, parts[j], plen[j]); bl += plen[j];
        }
        while (olen + rl > ocap) { ocap = ocap ? 2 * ocap : 64; out = (uint8_t*)realloc(out, ocap); }
        memcpy(out + olen, buf, rl); olen += rl;                    /* flat_map().collect() */
        free(buf); free(kl); free(vl); free(kc); free(vc);
    }
    double t1 = now_s();
    free(out);
    if (seconds) *seconds = t1 - t0;
    return olen;
}
