/*
 * horreum_gpu.h — C ABI of the MI355X SSTable record codec.
 *
 * This is the drop-in boundary for horreum's record codec and SSTable
 * writer/reader (reference: ikanago/horreum, Rust).  The reference has no FFI
 * of its own; each entry point below names the Rust function it replaces
 * (file:line in the reference tree).  A Rust caller binds these with plain
 * `extern "C"` declarations.
 *
 * On-disk record format (src/format.rs:23-37):
 *     [u64 LE key_len][u64 LE value_len][key bytes][value bytes]
 * value_len == 0 means "no value" (a deletion / tombstone): `Some(b"")` and
 * `None` encode identically and decode as `None` (src/format.rs:25-28, 71-75).
 *
 * Conventions
 *   - Every buffer is caller-owned.  The library never allocates output.
 *   - `_dev` entry points take device (HBM) pointers; `_host` entry points take
 *     host pointers and stage through pinned memory.
 *   - `_async` entry points enqueue work on the context's stream and return
 *     immediately; their result struct lives in device memory and is valid
 *     after the stream is synchronised.
 *   - Return value: HG_OK (0) or a status code.  Data-format errors are
 *     returned (never aborted on), unlike the reference, which unwrap()s them
 *     (src/sstable/storage.rs:64-66, src/sstable/table.rs:62-64).
 *   - One context = one GPU + one HIP stream.  Distinct contexts may be used
 *     from distinct threads; one context must not be used concurrently.
 */
#ifndef HORREUM_GPU_H
#define HORREUM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_ABI_VERSION 6

/* Status codes: return values, and the `kind` field of hg_err / results. */
enum hg_status {
    HG_OK = 0,
    /* Fewer than 16 bytes remain at a record start: the reference's
     * read_exact of the 16-byte length header fails (src/format.rs:64-65). */
    HG_ERR_TRUNCATED_HEADER = 1,
    /* Header read, but offset+16+key_len+value_len runs past the end: the
     * reference's read_exact of the body fails (src/format.rs:68-69). */
    HG_ERR_TRUNCATED_BODY = 2,
    /* key_len + value_len overflows u64 (src/format.rs:68; the reference
     * panics or wraps here). */
    HG_ERR_LEN_OVERFLOW = 3,
    /* A well-formed record whose key_len or value_len is >= 2^32 does not fit
     * the 16-byte hg_span; engine limit, documented in DESIGN.md. */
    HG_ERR_SPAN_RANGE = 4,
    /* Output buffer too small.  The required count/size is still reported. */
    HG_ERR_CAPACITY = 5,
    HG_ERR_INVALID_ARG = -1,
    HG_ERR_HIP = -2,
    HG_ERR_TOO_LARGE = -3,  /* input length >= 2^40 bytes, or a merge of >= 2^31
                               records (engine limits) */
    HG_ERR_INTERNAL = -4,   /* e.g. a bounded device spin timed out */
    HG_ERR_EMPTY_MERGE = -5, /* merge of zero records; the reference panics (src/sstable/manager.rs:213) */
    /* Retired (ABI <= 3 returned it for a merge input that was not strictly
     * increasing).  Since ABI 4 the merge follows the reference loop on any
     * input, so no entry point returns it. */
    HG_ERR_UNSORTED = -6
};

/* One decoded record: key at off+16, value at off+16+klen.
 * vlen == 0 <=> tombstone (value None).  16 bytes, 8-byte aligned. */
typedef struct hg_span {
    uint64_t off;
    uint32_t klen;
    uint32_t vlen;
} hg_span;

/* One record to encode, as offsets into a caller arena.  vlen == 0 encodes a
 * tombstone (InternalPair{value: None}, src/format.rs:6-11). */
typedef struct hg_pair {
    uint64_t key_off;
    uint64_t val_off;
    uint32_t klen;
    uint32_t vlen;
} hg_pair;

/* One block of the in-memory SSTable index (src/sstable/index.rs:6-15):
 * first key = key of record `first_rec`; bytes [position, position+length). */
typedef struct hg_block {
    uint64_t first_rec;
    uint64_t position;
    uint64_t length;
} hg_block;

/* Error detail: kind (enum hg_status) and the byte offset of the failing
 * record start (the position of the reference's cursor when it failed). */
typedef struct hg_err {
    int32_t kind;
    uint32_t reserved;
    uint64_t offset;
} hg_err;

/* Device-resident result of an async decode. */
typedef struct hg_decode_result {
    uint64_t n_records;  /* records decoded (before the error, if any) */
    int32_t kind;        /* enum hg_status */
    uint32_t reserved;
    uint64_t err_offset; /* failing record start when kind != HG_OK */
} hg_decode_result;

/* Device-resident result of an async encode. */
typedef struct hg_encode_result {
    uint64_t out_len; /* total encoded bytes, sum(16 + klen + vlen) */
    int32_t kind;     /* HG_OK or HG_ERR_CAPACITY */
    uint32_t reserved;
} hg_encode_result;

/* Result of a merge / compaction.  kind: HG_OK, HG_ERR_CAPACITY,
 * HG_ERR_EMPTY_MERGE, or a decode error of an input table (table, index =
 * failing byte offset).  On HG_OK, table says how the reference loop
 * (manager.rs:199-234) was followed: 0 the parallel newest-wins merge
 * (every table strictly increasing); for input that is not, 1 the serial
 * loop on the device (hg_merge_dev_async, or many disorder points), 2 epochs
 * of the parallel merge cut at the tables' disorder points (the synchronous
 * entry points; index = the number of epochs), 3 the parallel merge redone
 * after a look-back wait ran over its budget (a stalled grid; synchronous
 * entry points; index = the merges run after the first, >= 1). */
typedef struct hg_merge_result {
    uint64_t n_out;  /* merged records (tombstones included) */
    int32_t kind;
    uint32_t table;
    uint64_t index;
} hg_merge_result;

/* A lookup key: bytes [off, off+len) of a caller key arena. */
typedef struct hg_key {
    uint64_t off;
    uint32_t len;
    uint32_t reserved;
} hg_key;

/* Result of one point lookup.  found = 1: record `rec` holds the key (value
 * at table byte val_off, vlen bytes; vlen == 0 is a tombstone, i.e. the
 * reference's Some(InternalPair{value: None})).  found = 0: absent. */
typedef struct hg_lookup_result {
    uint64_t rec;
    uint64_t val_off;
    uint32_t vlen;
    int32_t found;
} hg_lookup_result;

typedef struct hg_ctx hg_ctx;

/* ---- library / context ---------------------------------------------- */
int hg_abi_version(void);
const char* hg_status_string(int status);
/* Where the most recent HG_ERR_HIP in this process came from:
 * "file:line: hipErrorName (code)", or "" if none yet.  Diagnostics only
 * (a HIP failure has no counterpart in the reference, which runs on the CPU). */
const char* hg_last_hip_error(void);

/* Knobs: batch-geometry overrides, A/B switches and test hooks (ABI 6).
 * The library reads no environment variables; these are its only run-time
 * switches, process-wide, all defaulting to the measured best (the list and
 * their meaning: DESIGN.md section 1, "No environment reads").  value < 0 clears a knob.  Returns
 * HG_ERR_INVALID_ARG for an unknown name.  hg_get_knob: -1 when unset.
 * A call reads a knob when it needs it (some calls more than once), so set
 * knobs while no call is in flight on any thread. */
int hg_set_knob(const char* name, int64_t value);
int hg_get_knob(const char* name, int64_t* value);

/* Create a context bound to HIP device `device` with its own stream. */
int hg_ctx_create(int device, hg_ctx** out);
int hg_ctx_destroy(hg_ctx* ctx);
/* Launch on a caller stream (a hipStream_t; NULL = the null stream). */
int hg_ctx_set_stream(hg_ctx* ctx, void* hip_stream);
/* Free the context's device work buffers (decode/encode/merge arenas and
 * workspaces; they grow again on demand): e.g. after SSTableManager's cold
 * open (src/sstable/manager.rs:47-55), whose batched decode sized them for a
 * whole directory.  Synchronizes the context's stream first. */
int hg_ctx_trim(hg_ctx* ctx);
/* Go back to the stream the context created for itself. */
int hg_ctx_use_own_stream(hg_ctx* ctx);
void* hg_ctx_stream(hg_ctx* ctx);
int hg_ctx_synchronize(hg_ctx* ctx);
/* Pre-size the device workspace so later calls never allocate
 * (keeps allocation out of timed regions): the single-table
 * decode and encode for tables of up to max_sst_bytes and max_pairs records,
 * and a one-table batched decode.
 *
 * Graph capture is not supported: a context carries state from call to call
 * (which control words the previous call's kernels left clear, argument
 * staging), so every stream-ordered entry point returns HG_ERR_INVALID_ARG
 * on a stream that is being captured and enqueues nothing. */
int hg_ctx_reserve(hg_ctx* ctx, uint64_t max_sst_bytes, uint64_t max_pairs);

/* ---- decode ----------------------------------------------------------
 * Replaces InternalPair::deserialize_from_bytes (src/format.rs:50-59) and
 * deserialize_inner (src/format.rs:63-77), i.e. the decode behind
 * PersistedFile::read_all (src/sstable/storage.rs:60-67), SSTable::open /
 * get / get_all (src/sstable/table.rs:33-75) and compaction's table reads
 * (src/sstable/manager.rs:148-151).
 *
 * Finds every record boundary of `len` bytes of SSTable data and writes one
 * hg_span per record, in file order, to spans[0..n).  If n > cap, only the
 * first `cap` spans are written and HG_ERR_CAPACITY is returned with *n_out =
 * n.  On a format error, spans[0..n_out) hold the records before the failing
 * one and err->offset is the failing record's start. */
int hg_decode_dev(hg_ctx* ctx, const uint8_t* d_sst, uint64_t len,
                  hg_span* d_spans, uint64_t cap,
                  uint64_t* n_out, hg_err* err);
/* Same, enqueued on the context stream; result lands in *d_result. */
int hg_decode_dev_async(hg_ctx* ctx, const uint8_t* d_sst, uint64_t len,
                        hg_span* d_spans, uint64_t cap,
                        hg_decode_result* d_result);
/* Many independent tables at once (the batched multi-table decode of
 * BASELINE config 4; SSTableManager::new opens every table of a directory,
 * src/sstable/manager.rs:47-55).  Table i: d_tables[i] (device), lens[i]
 * bytes, spans to d_spans[i] (capacity caps[i]), result to d_results[i]
 * (device array).  The host arrays are read during the call.  Tables decode
 * concurrently on auxiliary streams forked from and joined back into the
 * context stream; nothing is synchronised. */
int hg_decode_batch_dev_async(hg_ctx* ctx, uint32_t ntables,
                              const uint8_t* const* d_tables, const uint64_t* lens,
                              hg_span* const* d_spans, const uint64_t* caps,
                              hg_decode_result* d_results);
/* Host-memory in and out (pinned staging, H2D -> decode -> D2H). */
int hg_decode_host(hg_ctx* ctx, const uint8_t* h_sst, uint64_t len,
                   hg_span* h_spans, uint64_t cap,
                   uint64_t* n_out, hg_err* err);

/* ---- range decode ------------------------------------------------------
 * A table decoded in byte ranges: a single huge table split over devices
 * (the entry handoff is one u64 per split, no collective), or
 * decoded in chunks as its bytes arrive.  d_sst is the table's first byte;
 * bytes [begin, min(len, stop + 16)) must be valid device memory.  Decodes
 * the records that START in [entry, stop) -- `entry` must be the exact start
 * of a record (0 for the first range, else the exit of the previous range;
 * begin <= entry) -- with absolute offsets in the spans.  Records may end
 * past `stop` (up to len).  On HG_OK *exit is the first record start at or
 * after `stop` (the next range's entry; len at the table's end); the async
 * form stores it in d_result->err_offset.  Format errors are reported as by
 * hg_decode_dev (absolute offset), exactly where the reference's cursor walk
 * (src/format.rs:54-58) would fail inside the range. */
int hg_decode_range_dev_async(hg_ctx* ctx, const uint8_t* d_sst, uint64_t len,
                              uint64_t begin, uint64_t stop, uint64_t entry,
                              hg_span* d_spans, uint64_t cap,
                              hg_decode_result* d_result);
int hg_decode_range_dev(hg_ctx* ctx, const uint8_t* d_sst, uint64_t len,
                        uint64_t begin, uint64_t stop, uint64_t entry,
                        hg_span* d_spans, uint64_t cap, uint64_t* n_out,
                        uint64_t* exit, hg_err* err);
/* A GUESS of the first record start at or after `stop`: the 16 KiB before it
 * are walked from a guessed entry (the decode engine's lead-in); the walk's
 * exit is the guess.  Verify it against the exact exit of the previous range
 * and decode again from that exit when they differ.  *entry = UINT64_MAX
 * when nothing was found, len when stop >= len.  Bytes [stop - 16384 (or 0),
 * min(len, stop + 16)) must be valid device memory. */
int hg_decode_guess_entry_dev(hg_ctx* ctx, const uint8_t* d_sst, uint64_t len,
                              uint64_t stop, uint64_t* entry);

/* ---- encode ----------------------------------------------------------
 * Replaces InternalPair::serialize (src/format.rs:23-37) and
 * serialize_flatten (src/format.rs:40-42) as used by PersistedFile::new
 * (src/sstable/storage.rs:21-38), and Index::new's second encode that only
 * learns block lengths (src/sstable/index.rs:55-67).
 *
 * Packs pairs[0..n) (offsets into `arena`) into out[0..L), L = sum(16 + klen
 * + vlen), in the given order.  Optional outputs: rec_off[i] = byte offset of
 * record i; blocks[b] for every `block_stride` records (block_stride == 0
 * with a non-NULL blocks is HG_ERR_INVALID_ARG: the reference panics,
 * slice::chunks(0)).  If L > cap nothing is written past cap and
 * HG_ERR_CAPACITY is returned with *out_len = L. */
int hg_encode_dev(hg_ctx* ctx, const uint8_t* d_arena, const hg_pair* d_pairs,
                  uint64_t n, uint8_t* d_out, uint64_t cap,
                  uint64_t* d_rec_off, uint32_t block_stride,
                  hg_block* d_blocks, uint64_t* out_len);
int hg_encode_dev_async(hg_ctx* ctx, const uint8_t* d_arena,
                        const hg_pair* d_pairs, uint64_t n, uint8_t* d_out,
                        uint64_t cap, uint64_t* d_rec_off,
                        uint32_t block_stride, hg_block* d_blocks,
                        hg_encode_result* d_result);
int hg_encode_host(hg_ctx* ctx, const uint8_t* h_arena, uint64_t arena_len,
                   const hg_pair* h_pairs, uint64_t n, uint8_t* h_out,
                   uint64_t cap, uint64_t* h_rec_off, uint32_t block_stride,
                   hg_block* h_blocks, uint64_t* out_len);
/* Bytes serialize_flatten would produce for pairs[0..n) (src/format.rs:40-42):
 * sum(16 + klen + vlen).  `pairs` may be host or device memory (device: one
 * reduction on the context stream, synchronised). */
int hg_encoded_size(hg_ctx* ctx, const hg_pair* pairs, uint64_t n, uint64_t* bytes);

/* ---- merge (compaction) ------------------------------------------------
 * Replaces SSTableManager::compact_inner (src/sstable/manager.rs:199-234),
 * the k-way merge of SSTableManager::compact (:137-159).  ntables tables of
 * decoded records live in one device arena: table t's bytes start at
 * table_off[t] and its spans (offsets relative to that start) are
 * d_spans[t][0..counts[t]).  Tables are in priority order: on equal keys the
 * lowest t wins (compact() passes them newest first, :146-149).  Output:
 * one hg_pair per distinct key, ascending, pointing into the arena
 * (key_off/val_off relative to d_arena), tombstones kept -- ready for
 * hg_encode_* to write the compacted table.  table_off, d_spans (an array of
 * device pointers) and counts are host arrays.  Tables that are strictly
 * increasing by key (every table horreum writes) merge by parallel merge
 * path; any other input -- duplicate keys or keys out of order inside a
 * table, which SSTable::new accepts (src/sstable/table.rs:93-108) -- gets the
 * reference loop's exact output (first minimum head wins, every equal head
 * advances) from a serial device pass.  All tables empty is
 * HG_ERR_EMPTY_MERGE (the reference panics, manager.rs:213). */
int hg_merge_dev(hg_ctx* ctx, uint32_t ntables, const uint8_t* d_arena,
                 uint64_t arena_len, const uint64_t* table_off,
                 const hg_span* const* d_spans, const uint64_t* counts,
                 hg_pair* d_out, uint64_t cap, hg_merge_result* result);
int hg_merge_dev_async(hg_ctx* ctx, uint32_t ntables, const uint8_t* d_arena,
                       uint64_t arena_len, const uint64_t* table_off,
                       const hg_span* const* d_spans, const uint64_t* counts,
                       hg_pair* d_out, uint64_t cap,
                       hg_merge_result* d_result);
/* The byte work of SSTableManager::compact (manager.rs:137-159) from host
 * buffers: decode every table, merge (as hg_merge_dev), encode the merged
 * records into h_out (the compacted SSTable, byte-identical to the
 * reference's serialize_flatten of compact_inner's output) and its index
 * blocks (optional, as hg_encode_host).  *out_len = encoded bytes; the
 * compacted table's payload size (table.rs:36-45) is
 * *out_len - 16 * result->n_out. */
int hg_compact_host(hg_ctx* ctx, uint32_t ntables, const uint8_t* const* h_tables,
                    const uint64_t* lens, uint8_t* h_out, uint64_t cap,
                    uint64_t* out_len, uint32_t block_stride, hg_block* h_blocks,
                    hg_merge_result* result);
/* hg_compact_host on tables already in device memory: table t is
 * d_arena[table_off[t], +lens[t]) (one allocation, so a key read never leaves
 * it); the compacted table goes to d_out (cap bytes) and its index blocks,
 * when d_blocks is given, to d_blocks (hg_block_count(result->n_out,
 * block_stride) entries).  Synchronous: one host sync for the decoded record
 * counts (the merge is launched from them), merge and encode back to back
 * (the encode reads the merge's output count on the device), one sync for the
 * results. */
int hg_compact_dev(hg_ctx* ctx, uint32_t ntables, const uint8_t* d_arena,
                   uint64_t arena_len, const uint64_t* table_off, const uint64_t* lens,
                   uint8_t* d_out, uint64_t cap, uint64_t* out_len, uint32_t block_stride,
                   hg_block* d_blocks, hg_merge_result* result);

/* ---- point lookups ----------------------------------------------------
 * Replaces SSTable::get (src/sstable/table.rs:54-70) for a batch of keys:
 * Index::get (src/sstable/index.rs:72-78) binary-searches the first keys of
 * the blocks of `block_stride` records (0: the whole table is one block),
 * then binary_search_by_key searches that block.  Both follow Rust's
 * slice::binary_search_by (std 1.52-1.81: mid = left + (right - left) / 2,
 * the first probe that compares Equal wins), so on any table -- duplicate or
 * unordered keys included (legal, table.rs:93-108) -- the record found is
 * the reference's.  First build the key index once per decoded table (d_spans,
 * n records; 32 * n bytes of device memory at d_index), then look up any
 * number of batches. */
uint64_t hg_keyindex_bytes(uint64_t n);
int hg_keyindex_build_dev_async(hg_ctx* ctx, const uint8_t* d_table, uint64_t len,
                                const hg_span* d_spans, uint64_t n, void* d_index);
int hg_lookup_dev_async(hg_ctx* ctx, const uint8_t* d_table, const hg_span* d_spans,
                        const void* d_index, uint64_t n, uint32_t block_stride,
                        const uint8_t* d_keys, const hg_key* d_queries, uint64_t nq,
                        hg_lookup_result* d_results);
/* Host table bytes and host keys: decode, index, look up, copy back. */
int hg_lookup_host(hg_ctx* ctx, const uint8_t* h_table, uint64_t len, uint32_t block_stride,
                   const uint8_t* h_keys, uint64_t keys_len, const hg_key* h_queries,
                   uint64_t nq, hg_lookup_result* h_results);

/* ---- host memory ------------------------------------------------------
 * The `_host` entry points DMA straight from / to page-locked host memory
 * and stage pageable memory through two pinned 64 MiB buffers (CPU copies
 * split over host threads, overlapped with the DMA).  A caller that keeps an
 * SSTable file mmap'd (PersistedFile, src/sstable/storage.rs:21-67) or a
 * memtable arena alive registers it once so every later call skips the CPU
 * copy.  hg_host_register pins [h_ptr, h_ptr+len) (hipHostRegister);
 * hg_host_unregister takes the base pointer passed to register;
 * hg_host_is_pinned returns 1 for page-locked host memory, else 0. */
int hg_host_register(const void* h_ptr, uint64_t len);
int hg_host_unregister(const void* h_ptr);
int hg_host_is_pinned(const void* h_ptr);

/* ---- several contexts: one host thread per context, no collectives -------
 * ctxs[0..nctx) may be on different devices or on the same one; each is used
 * by exactly one thread for the duration of the call.
 *
 * Many tables (SSTableManager::new opening a directory, manager.rs:47-55;
 * BASELINE config 4): table i goes to context i % nctx; each context uploads
 * its tables and decodes them in one batched launch chain per group of tables
 * under a device byte budget (knob HG_DECODE_GROUP_BYTES, default 40 % of the free
 * device memory; tables plus span capacity), so a directory larger than HBM
 * opens group by group.  spans of table i
 * to h_spans[i] (capacity caps[i]), n_out[i] records, errs[i] its format
 * error (kind HG_OK if none; errs may be NULL).  Returns HG_OK unless a
 * runtime error occurred. */
int hg_multi_decode_host(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                         const uint8_t* const* h_tables, const uint64_t* lens,
                         hg_span* const* h_spans, const uint64_t* caps,
                         uint64_t* n_out, hg_err* errs);
/* One table cut into nctx byte ranges (16 KiB-aligned cuts): every context
 * guesses its range's entry (hg_decode_guess_entry_dev), decodes the range
 * from it, then the host hands the exact entry over in order (the previous
 * range's exit) and a range entered off its guess is decoded again.  The
 * result equals hg_decode_host's (spans, n_out, error kind and offset). */
int hg_multi_decode_file_host(hg_ctx* const* ctxs, uint32_t nctx,
                              const uint8_t* h_sst, uint64_t len,
                              hg_span* h_spans, uint64_t cap,
                              uint64_t* n_out, hg_err* err);
/* SSTableManager::compact (manager.rs:137-159) split by key range: every
 * table is uploaded once, to context i % nctx, decoded there and its keys
 * sampled; nctx-1 splitter keys are taken from the samples (the reference's
 * block first keys are every block_stride-th key, index.rs:55-67); context g
 * gathers the slice of every table inside key range g -- bytes and decoded
 * spans, copied device to device from the table's context (xGMI peer copies
 * across GPUs): nothing is uploaded or decoded twice -- merges and encodes
 * it; the output is the concatenation in key order with its block index --
 * byte-identical to hg_compact_host.  Input that is not strictly increasing
 * (found by a slice's merge or at a cut) and tables that do not decode are
 * compacted by hg_compact_host on ctxs[0], which follows the reference loop
 * exactly. */
int hg_multi_compact_host(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                          const uint8_t* const* h_tables, const uint64_t* lens,
                          uint8_t* h_out, uint64_t cap, uint64_t* out_len,
                          uint32_t block_stride, hg_block* h_blocks,
                          hg_merge_result* result);

/* The same split compaction on tables already in device memory: table t is
 * d_tables[t] (lens[t] bytes) on the device of ctxs[owner[t]], decoded there
 * in place; range g is merged and encoded on ctxs[g] into d_outs[g] (caps[g]
 * bytes on that context's device; out_lens[g] bytes, out_recs[g] records;
 * ranges past the splitters found are empty).  The compacted table is the
 * concatenation of the slices g = 0 .. nctx-1, byte-identical to
 * hg_compact_dev.  Input that is not range-separable, and tables that do not
 * decode, are gathered on ctxs[0] and compacted there by hg_compact_dev
 * (the reference loop; the whole output, or the error, in slice 0: size
 * caps[0] for it).  result->n_out = records in all slices. */
int hg_multi_compact_dev(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                         const uint32_t* owner, const uint8_t* const* d_tables,
                         const uint64_t* lens, uint8_t* const* d_outs, const uint64_t* caps,
                         uint64_t* out_lens, uint64_t* out_recs, hg_merge_result* result);

/* Number of blocks Index::new produces for n pairs: ceil(n / stride). */
uint64_t hg_block_count(uint64_t n, uint32_t block_stride);

#ifdef __cplusplus
}
#endif
#endif /* HORREUM_GPU_H */
