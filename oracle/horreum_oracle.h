/*
 * horreum_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ikanago/horreum's SSTable record codec, used as the
 * parity checker for the HIP engine.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path
 * (horreum_amd/, libhorreum_gpu.so) never links or calls it.
 *
 * The reference is Rust and cannot be built here (no cargo/rustc, crates not
 * vendored).  This restatement is pinned by the
 * known-answer vectors of the reference's own tests (tests/golden/).
 * Struct layouts are shared with the product ABI (include/horreum_gpu.h).
 */
#ifndef HORREUM_ORACLE_H
#define HORREUM_ORACLE_H

#include "../include/horreum_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* InternalPair::deserialize_from_bytes (src/format.rs:50-77). */
int hgo_decode(const uint8_t* bytes, uint64_t len, hg_span* spans,
               uint64_t cap, uint64_t* n_out, hg_err* err);

/* InternalPair::serialize / serialize_flatten (src/format.rs:23-42) plus
 * Index::new block positions/lengths (src/sstable/index.rs:55-67). */
int hgo_encode(const uint8_t* arena, const hg_pair* pairs, uint64_t n,
               uint8_t* out, uint64_t cap, uint64_t* rec_off,
               uint32_t block_stride, hg_block* blocks, uint64_t* out_len);

/* Index::get (src/sstable/index.rs:72-78).  Block first keys are given as
 * (arena, pairs[blocks[b].first_rec]).  Returns 1 and fills *pos and *len when a
 * block is selected, 0 for None. */
int hgo_index_get(const hg_block* blocks, uint64_t nblocks,
                  const uint8_t* arena, const hg_pair* pairs,
                  const uint8_t* key, uint64_t klen,
                  uint64_t* pos, uint64_t* len);

/* SSTableManager::compact_inner (src/sstable/manager.rs:199-234).  Tables
 * are given in iterator order (compact() passes the newest table first,
 * :148-151); on equal keys the FIRST iterator wins.  Writes the chosen
 * (table, record) pairs in output order. */
int hgo_compact(uint32_t ntables, const uint8_t* const* datas,
                const hg_span* const* spans, const uint64_t* counts,
                uint32_t* out_table, uint64_t* out_rec, uint64_t cap,
                uint64_t* n_out);

/* SSTable::open size accounting: sum(klen + vlen) (src/sstable/table.rs:36-45). */
/* src/sstable/table.rs:54-70: SSTable::get on a decoded table. */
int hgo_table_get(const uint8_t* data, const hg_span* spans, uint64_t n, uint32_t stride,
                  const uint8_t* key, uint64_t klen, uint64_t* rec);

uint64_t hgo_payload_size(const hg_span* spans, uint64_t n);

/* CPU baselines.  Decode with the reference's per-record ownership pattern
 * (16-byte header Vec, zeroed content Vec, key/value to_vec copies, pushed
 * into a growing Vec; src/format.rs:63-77).  Returns records decoded, or
 * (uint64_t)-1 on a format error.  Everything allocated is freed before
 * returning; *seconds_decode excludes the final drop. */
uint64_t hgo_bench_decode_owned(const uint8_t* bytes, uint64_t len,
                                double* seconds_decode);
/* Encode with the reference's per-pair temporaries (src/format.rs:23-42). */
uint64_t hgo_bench_encode_owned(const uint8_t* arena, const hg_pair* pairs,
                                uint64_t n, double* seconds);

/* Optimised multi-threaded CPU codec (cpu_opt.c; bench.py's cpu_baseline):
 * decode into spans over `nthreads` byte ranges with guessed entries handed
 * over in order (scratch: len/16 + 2*nthreads + 2 spans); records decoded,
 * UINT64_MAX on a format error.  Encode: sizes, prefix, copy on `nthreads`
 * threads; returns bytes written.  *seconds = wall time of the call. */
uint64_t hgo_mt_decode(const uint8_t* bytes, uint64_t len, hg_span* spans, uint64_t cap,
                       hg_span* scratch, uint32_t nthreads, double* seconds);
void hgo_mt_memcpy(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t nthreads,
                   double* seconds);
uint64_t hgo_mt_encode(const uint8_t* arena, const hg_pair* pairs, uint64_t n, uint8_t* out,
                       uint32_t nthreads, double* seconds);

#ifdef __cplusplus
}
#endif
#endif
