/*
 * fsehip.h -- C ABI of the MI355X-native FSE (tANS) entropy coder.
 *
 * Drop-in boundary for the hot path of Cognoscan/entropy_coders (a Rust
 * crate).  Two layers:
 *
 *  (1) Reference-shaped entry points (host pointers, one block per call),
 *      one per public function of the crate on this path.  They keep the
 *      crate's argument meaning and its "append to dst" convention; Rust
 *      panics / None / Err become negative status codes (fse_status.h).
 *      Compute runs on the GPU; there is no CPU fallback.  These are what a
 *      Rust FFI shim binds.
 *
 *  (2) Batched device entry points (fsehip_*): all pointers are device
 *      pointers, calls are asynchronous on `stream` and report a status per
 *      block.  This is the throughput path (bench.py, multi-GPU sharding).
 *
 * Every compressed block is byte-identical to the crate's fse_compress2
 * output for the same input (lib.rs:146-183).
 */
#ifndef FSEHIP_H
#define FSEHIP_H

#include <stddef.h>
#include <stdint.h>

#include "fse_status.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fsehip_stream_t; /* hipStream_t; NULL = the null stream */

/* ------------------------------------------------------------------------
 * (1) Reference-shaped entry points
 * ------------------------------------------------------------------------ */

/* Replaces `pub fn fse_compress2(src: &[u8], dst: &mut Vec<u8>) -> usize`
 * (lib.rs:146).  Appends header||payload at dst[*dst_len], advances
 * *dst_len, and stores the Rust return value (payload bits incl. marker) in
 * *payload_bits.  Errors: EMPTY, TOO_SHORT, ALL_ZERO_SYMBOL0 (reference
 * panics), DST_TOO_SMALL (the reference grows its Vec), UNSUPPORTED (n >
 * 2^28), ENCODER_INIT (the tableLog-15 panic of new_first_symbol). */
int fse_compress2(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                  uint64_t* payload_bits);

/* `Histogram::new(src).normalize(table_log)` followed by the fse_compress2
 * body (histogram.rs:95 + lib.rs:149-182): the tableLog sweep entry point.
 * table_log is clamped to 5..15 as normalize does (0 acts as 5). */
int fse_compress2_log(const uint8_t* src, size_t n, uint32_t table_log, uint8_t* dst, size_t dst_cap,
                      size_t* dst_len, uint64_t* payload_bits);

/* Replaces `pub fn fse_decompress2(src: &[u8], dst: &mut Vec<u8>)
 * -> Option<usize>` (lib.rs:215).  Appends the decoded bytes at
 * dst[*dst_len] and advances *dst_len.  None -> BAD_HEADER / NO_MARKER;
 * the state-read panic -> TOO_SHORT; the never-terminating single-symbol
 * case -> SINGLE_SYMBOL; output beyond dst_cap -> DST_TOO_SMALL (the
 * reference grows its Vec).
 *
 * The host entry points of this section are synchronous on the default
 * stream and stage through per-thread buffers the library keeps: pinned host
 * memory (the input, and up to 4 MiB of the result; larger results come back
 * by a plain device-to-host copy) and device memory (input, output up to
 * dst_cap - *dst_len, tables).  fsehip_release_workspace frees them.  A lone
 * stream decodes as one serial chain (~1.4 ms per 64 KiB call on MI355X,
 * slower than one host core); many streams belong on fse_decompress2_many
 * (host buffers) or fsehip_decompress_streams (device buffers). */
int fse_decompress2(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len);

/* The 1-state format: replaces `pub fn fse_compress(src, dst) -> (NormHistogram, usize)`
 * (lib.rs:112; the returned NormHistogram is the block's own header) and
 * `pub fn fse_decompress(src, dst) -> Option<usize>` (lib.rs:187), same
 * conventions as the 2-state pair above. */
int fse_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len, uint64_t* payload_bits);
int fse_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len);

/* Many fse_decompress2 / fse_decompress calls in one (lib.rs:215-248 /
 * 187-211 per stream): the drop-in for a caller's loop over many crate
 * streams.  Stream i (srcs[i], src_lens[i] bytes) decodes into
 * dst + i * dst_stride with at most dst_stride bytes; dst_lens[i] = bytes
 * decoded and statuses[i] = its status, as the single call would return it
 * (EMPTY, BAD_HEADER, NO_MARKER, TOO_SHORT, SINGLE_SYMBOL, DST_TOO_SMALL,
 * UNSUPPORTED above 2^28 bytes; a null srcs[i] with src_lens[i] > 0 is
 * BAD_ARG).  Returns FSE_OK when the batch ran (look at statuses), or a
 * call-level error (BAD_ARG, NO_DEVICE, HIP).  Streams up to 4 MiB are
 * batched, grouped by the table log in their header (<= 11, 12, 13..15: each
 * group runs the kernels and decode-table stride of its class, so one large
 * or corrupt log does not move the others), in groups of at most 512 MiB of
 * staging each way and 512 MiB of decode tables; longer streams, a log
 * nibble above 15 (a header the crate rejects) and dst_stride above 128 MiB
 * take the single-stream path one by one.
 *
 * Where the GPU pays.  A lone stream is one serial chain: fse_decompress2
 * takes ~1.4 ms per 64 KiB call on MI355X against ~0.14-0.4 ms on one host
 * core, so the per-call path never beats a CPU core.  This call stages all
 * streams through pinned memory in one copy each way and decodes them as
 * thousands of chains at once (fsehip_decompress_streams): 2.6 ms for 16
 * 64 KiB streams, 3.7 ms for 256, 6.3 ms for 1,000 (9.7 GiB/s), 16.5 ms for
 * 4,000 (14.8 GiB/s), PCIe included, so it beats one host core from ~16
 * streams and 16 cores from ~256 (tools/many_streams.py; bench.py's
 * host_call_latency reports 1,000 streams).  One or two streams take the
 * single-stream path; batches of up to 32 streams at table log <= 11 run
 * the single-stream kernel once per stream in one launch (3 streams 1.5 ms,
 * 16 streams 2.1 ms; 1-state 16 streams 2.0 ms, tools/many_ab.py).
 * Synchronous on the default stream; the staging buffers are per thread
 * (grow-only, freed by fsehip_release_workspace). */
int fse_decompress2_many(const uint8_t* const* srcs, const size_t* src_lens, size_t n_streams, uint8_t* dst,
                         size_t dst_stride, size_t* dst_lens, int32_t* statuses);
int fse_decompress_many(const uint8_t* const* srcs, const size_t* src_lens, size_t n_streams, uint8_t* dst,
                        size_t dst_stride, size_t* dst_lens, int32_t* statuses);

/* Replaces `Histogram::new(data)` (histogram.rs:18-66) -- the north star's
 * `histogram::count`: counts[256], table_len = 1 + largest symbol. */
int histogram_count(const uint8_t* src, size_t n, uint32_t counts[256], uint32_t* table_len);

/* ------------------------------------------------------------------------
 * (1b) The crate's building blocks, as plain-data structs (repr(C) twins of
 * the Rust types; every table has room for the largest log, 15) and calls
 * that run on the GPU.  Same argument meaning and panics-as-statuses as
 * above; host pointers.
 * ------------------------------------------------------------------------ */

/* Histogram (histogram.rs:9-14): counts, size = input length, table_len =
 * 1 + the largest symbol (1 when empty). */
typedef struct {
    uint32_t counts[256];
    uint32_t size;
    uint32_t table_len;
} fse_histogram;

/* NormHistogram (histogram.rs:289-294): norm[s] in {-1, 0, 1..2^log2}. */
typedef struct {
    int32_t norm[256];
    uint32_t log2;
    uint32_t table_len;
} fse_norm_histogram;

/* EncodeTable (fse.rs:72-84): stateTable (`table`, 2^table_log used),
 * the spread (`symbols`) and the symbol transforms. */
typedef struct {
    uint32_t bits;      /* deltaNbBits */
    int32_t find_state; /* deltaFindState */
} fse_symbol_transform;
typedef struct {
    uint32_t table_log;
    uint16_t table[1u << 15];
    uint8_t symbols[1u << 15];
    fse_symbol_transform symbol_tt[256];
} fse_encode_table;

/* DecodeTable (fse.rs:253-265). */
typedef struct {
    uint16_t new_state;
    uint8_t symbol;
    uint8_t num_bits;
} fse_decode_transform;
typedef struct {
    uint32_t table_log;
    uint32_t fast_mode; /* no symbol with norm >= 2^(table_log-1) (fse.rs:302-305) */
    fse_decode_transform table[1u << 15];
} fse_decode_table;

/* Histogram::new (histogram.rs:18-66). */
int histogram_new(const uint8_t* src, size_t n, fse_histogram* out);
/* Histogram::normalize(log2) (histogram.rs:95-155): log2 is clamped to 5..15
 * and raised to ilog2(table_len - 1) + 2 as in the reference. */
int histogram_normalize(const fse_histogram* h, uint32_t log2, fse_norm_histogram* out);
/* Histogram::normalize_optimal (histogram.rs:281-284, optimal_log2 264-277). */
int histogram_normalize_optimal(const fse_histogram* h, fse_norm_histogram* out);
/* NormHistogram::new (histogram.rs:299-303). */
int norm_histogram_new(const uint8_t* src, size_t n, fse_norm_histogram* out);
/* NormHistogram::write (histogram.rs:376-431): appends the header at
 * dst[*dst_len], advances *dst_len, *bits_written = the returned bit count. */
int norm_histogram_write(const fse_norm_histogram* nh, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                         uint64_t* bits_written);
/* NormHistogram::read (histogram.rs:436-505): *consumed = header bytes (the
 * remaining slice starts there).  Errors: BAD_HEADER (TableLogTooLarge,
 * TooManySymbols, UnexpectedEof), EMPTY. */
int norm_histogram_read(const uint8_t* src, size_t n, fse_norm_histogram* out, size_t* consumed);
/* EncodeTable::new / DecodeTable::new (fse.rs:88-189, 269-338). */
int encode_table_new(const fse_norm_histogram* nh, fse_encode_table* out);
int decode_table_new(const fse_norm_histogram* nh, fse_decode_table* out);
/* fse_compress with its returned NormHistogram (lib.rs:112: the tuple's
 * first element); otherwise as fse_compress. */
int fse_compress_nh(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                    uint64_t* payload_bits, fse_norm_histogram* nh);

/* The bitstream (bitstream/mod.rs:9-15).  A field is (value, width), width
 * <= 32 (the crate's writer and readers take <= 16).
 *  bitstack_write: BitStackWriter::new(dst) + write_bits_unmasked(vals[i],
 *    nbits[i]) for each field + finish() (writer.rs:14-222): the fields
 *    LSB-first from byte *dst_len on, zero-padded to a byte; appends,
 *    advances *dst_len, *bits_written = finish()'s count.
 *  bitstack_read: BitStackReader::new(src) (None -> NO_MARKER: empty or a
 *    zero last byte, stack_reader.rs:17-92) + read(nbits[i]) per field
 *    (top down); *n_read = reads that returned Some (the first None stops
 *    them), *finished = finish() after them (stack_reader.rs:224-226).
 *  bitstream_read: BitStreamReader::new(src, total_bits) (asserts
 *    n == ceil(total_bits / 8) > 0 -> BAD_ARG) + read(nbits[i]) per field;
 *    *n_read = reads that returned Ok, *bits_left = available() after them. */
int bitstack_write(const uint32_t* vals, const uint8_t* nbits, size_t count, uint8_t* dst, size_t dst_cap,
                   size_t* dst_len, uint64_t* bits_written);
int bitstack_read(const uint8_t* src, size_t n, const uint8_t* nbits, size_t count, uint32_t* vals, size_t* n_read,
                  int* finished);
int bitstream_read(const uint8_t* src, size_t n, uint64_t total_bits, const uint8_t* nbits, size_t count,
                   uint32_t* vals, size_t* n_read, uint64_t* bits_left);
/* BitStreamReader with each field's call named (stream_reader.rs:56-119):
 * ops[i] = FSE_BITS_READ (read), FSE_BITS_PEEK (peek: value, no advance) or
 * FSE_BITS_ADVANCE (advance_by: advance, value 0).  Any of them fails past
 * total_bits (UnexpectedEof) and stops the list: *n_done = steps that
 * returned Ok, *bits_left = available() after them (finish(): the remaining
 * slice starts at byte (total_bits - *bits_left) / 8, finish_byte() at the
 * next byte boundary).  ops = NULL: all reads, as bitstream_read. */
#define FSE_BITS_READ 0
#define FSE_BITS_PEEK 1
#define FSE_BITS_ADVANCE 2
int bitstream_read_ops(const uint8_t* src, size_t n, uint64_t total_bits, const uint8_t* nbits, const uint8_t* ops,
                       size_t count, uint32_t* vals, size_t* n_done, uint64_t* bits_left);

/* ------------------------------------------------------------------------
 * (1c) The bit readers and writer as incremental cursors
 *
 * The crate's callers drive its readers one field at a time with widths
 * chosen from earlier values (NormHistogram::read, histogram.rs:453-496; the
 * decoders, fse.rs:349-385).  Each reader / writer is a plain struct the
 * caller owns (no allocation, no handle table) and every call is O(1):
 * a Rust shim wraps it as BitStackReader / BitStreamReader / BitStackWriter
 * with the same method names.  These run on the
 * caller's side of the ABI (host): one field is a few shifts.  Millions of
 * fields with known widths go through the batched device forms
 * (fsehip_bitstack_write / fsehip_bitstack_read / fsehip_bitstream_read_ops).
 * Semantics are the crate's on a 64-bit target (32-bit refills/flushes),
 * including available(), which depends on the buffer's address alignment as
 * the crate's does.  None / Err(UnexpectedEof) -> FSE_ERR_EOF; the crate's
 * debug assertions (width > 32, advance past the buffer) -> FSE_ERR_BAD_ARG.
 * ------------------------------------------------------------------------ */

/* BitStackReader (stack_reader.rs:5-227): reads the stack from the end,
 * after the marker bit. */
typedef struct {
    const uint8_t* base; /* the slice */
    const uint8_t* ptr;  /* next refill address */
    uint64_t buffer;
    uint64_t bits;       /* bits buffered: available() */
    int32_t finished;
    int32_t reserved;
} fse_bitstack_reader;
/* new (stack_reader.rs:17-92): None (empty slice, zero last byte, marker not
 * in the last byte) -> FSE_ERR_NO_MARKER */
int bitstack_reader_new(fse_bitstack_reader* r, const uint8_t* src, size_t n);
int bitstack_reader_reload(fse_bitstack_reader* r);                                        /* 97-172 */
int bitstack_reader_peek(const fse_bitstack_reader* r, uint32_t nbits, uint32_t* val);      /* 176-184 */
int bitstack_reader_read_no_reload(fse_bitstack_reader* r, uint32_t nbits, uint32_t* val); /* 193-197 */
int bitstack_reader_advance_no_reload(fse_bitstack_reader* r, uint32_t nbits);             /* 204-207 */
int bitstack_reader_read(fse_bitstack_reader* r, uint32_t nbits, uint32_t* val);           /* 211-215 */
uint64_t bitstack_reader_available(const fse_bitstack_reader* r);                          /* 218-220 */
int bitstack_reader_finish(const fse_bitstack_reader* r); /* 224-226: 1 if every bit was read */

/* BitStreamReader (stream_reader.rs:5-136): forward LSB-first reader. */
typedef struct {
    const uint8_t* src;
    uint64_t n;
    uint64_t total_bits;
    uint64_t bits_read;
} fse_bitstream_reader;
/* new (stream_reader.rs:16-49): n == 0 or n != ceil(total_bits/8) (the
 * crate's asserts) -> FSE_ERR_BAD_ARG */
int bitstream_reader_new(fse_bitstream_reader* r, const uint8_t* src, size_t n, uint64_t total_bits);
int bitstream_reader_read(fse_bitstream_reader* r, uint32_t nbits, uint32_t* val);       /* 56-60 */
int bitstream_reader_advance_by(fse_bitstream_reader* r, uint32_t nbits);                /* 67-75 */
int bitstream_reader_peek(const fse_bitstream_reader* r, uint32_t nbits, uint32_t* val); /* 82-114 */
uint64_t bitstream_reader_available(const fse_bitstream_reader* r);                      /* 117-119 */
/* finish (123-128): the remaining slice starts at src + *byte, *remaining
 * bits, *offset bits into its first byte */
int bitstream_reader_finish(const fse_bitstream_reader* r, size_t* byte, uint64_t* remaining, uint32_t* offset);
/* finish_byte (132-135): offset of the remaining bytes (next byte boundary) */
size_t bitstream_reader_finish_byte(const fse_bitstream_reader* r);

/* BitStackWriter (writer.rs:5-223) appending to dst[len..cap).  Whole bytes
 * are committed to dst as they complete; a full buffer is a sticky
 * FSE_ERR_DST_TOO_SMALL (the crate grows its Vec). */
typedef struct {
    uint8_t* dst;
    uint64_t cap;
    uint64_t len;         /* bytes committed (the Vec's length at finish) */
    uint64_t initial_len;
    uint64_t storage;     /* pending bits, LSB-first */
    uint32_t bits;
    int32_t status;
} fse_bitstack_writer;
int bitstack_writer_new(fse_bitstack_writer* w, uint8_t* dst, size_t cap, size_t len); /* 16-40 */
int bitstack_writer_flush(fse_bitstack_writer* w);                                     /* 43-110 */
/* write_bits_raw (164-180): val's bits above nbits must be zero; no flush */
int bitstack_writer_write_bits_raw(fse_bitstack_writer* w, uint32_t val, uint32_t nbits);
int bitstack_writer_write_bits_raw_unmasked(fse_bitstack_writer* w, uint32_t val, uint32_t nbits); /* 140-149 */
int bitstack_writer_write_bits(fse_bitstack_writer* w, uint32_t val, uint32_t nbits);          /* 185-188 */
int bitstack_writer_write_bits_unmasked(fse_bitstack_writer* w, uint32_t val, uint32_t nbits); /* 193-198 */
/* finish (201-222): zero-pads the last byte; *dst_len = new length of dst,
 * *bits_written = bits written since new() */
int bitstack_writer_finish(fse_bitstack_writer* w, size_t* dst_len, uint64_t* bits_written);

/* ------------------------------------------------------------------------
 * (2) Batched device entry points
 * ------------------------------------------------------------------------ */

typedef struct {
    uint32_t block_size;    /* bytes per block, <= 2^28 (u32 bit counts); multiple of 16 when >1 block; default 65536 */
    uint32_t table_log;     /* 0 = NormHistogram::new (optimal); else Histogram::normalize(L) */
    uint32_t ckpt_interval; /* steps between decode checkpoints (power of two; >= 8 for 2-state
                               pairs, >= 16 for 1-state symbols), 0 = none */
    uint32_t max_table_log; /* upper bound on L used by the blocks (5..15; kernels exist for <= 11,
                               12, 13, 14 and 15); 0 = derive (encode) / 12 (decode) */
    uint32_t nstates;       /* block format: 2 (or 0) = fse_compress2 (lib.rs:146), 1 = fse_compress (lib.rs:112) */
} fsehip_params;

/* Per-block output slot size (bytes) able to hold any block of block_size
 * bytes at tableLog <= max_table_log, and sidecar entries per block (2-state
 * blocks; the _ns variant covers both formats). */
uint64_t fsehip_slot_bytes(uint32_t block_size, uint32_t max_table_log);
uint32_t fsehip_sidecar_per_block(uint32_t block_size, uint32_t ckpt_interval);
uint32_t fsehip_sidecar_per_block_ns(uint32_t block_size, uint32_t ckpt_interval, uint32_t nstates);

/* Compress n_total bytes as ceil(n_total/block_size) independent blocks.
 * Block b's bytes go to d_out + b*slot_bytes (comp_len[b] bytes, exactly
 * fse_compress2's output); d_sidecar (optional) receives the decode
 * checkpoints: entry = bitpos(32, payload-relative) | s0<<32 | s1<<48 for
 * the decoder state before pair k*ckpt_interval.  A slot's bytes beyond
 * comp_len[b] are unspecified: at table logs 13..15 the kernels use them
 * as scratch (the spread's 2^L symbols after the first 512 bytes); slots
 * smaller than 512 + 2^L bytes make the call take a workspace buffer of
 * 2^L bytes per block instead (see fsehip_decompress_blocks). */
int fsehip_compress_blocks(const fsehip_params* p, const uint8_t* d_src, uint64_t n_total, uint8_t* d_out,
                           uint64_t slot_bytes, uint32_t* d_comp_len, uint32_t* d_payload_bits,
                           uint64_t* d_sidecar, int32_t* d_status, fsehip_stream_t stream);

/* Decompress blocks produced as above.  With d_sidecar the blocks decode in
 * parallel segments; without it (any valid fse_compress2 stream, e.g. from
 * the CPU crate) each block decodes serially, many at once (one lane per
 * block, its table compact in LDS).  Blocks at table log <= 11 (both formats) keep
 * only the u16 table entries in LDS (8 blocks per workgroup, 32 chains per
 * CU) and defer their symbols: the chains write state pairs into the
 * stream's workspace and a map kernel turns them into bytes; if that
 * workspace cannot be allocated (or the batch has 2^24 blocks or more), the
 * single-kernel decode runs (6 blocks per workgroup, 24 chains per CU).
 * n_total (> 0) gives the raw length.  slot_bytes is a multiple of 256, as
 * encoder slots are (the decode-table build requires it); d_in and d_out
 * 16-byte aligned (BAD_ARG otherwise).
 *
 * Workspace (device memory owned by the library, one per (device, stream),
 * grown on demand and kept for reuse until fsehip_release_workspace):
 *   decode tables  fsehip_dtable_bytes(max_table_log) + 4 bytes per block
 *                  (every call of fsehip_decompress_blocks / _streams /
 *                  fsehip_build_sidecar);
 *   deferred symbols (sidecar-less decode at table log <= 11 only):
 *                  2 bytes per output byte of the batch's capacity
 *                  (n_blocks x block_size) + 8 bytes per block -- 2 GiB for a
 *                  1 GiB batch.  A size that failed to allocate is remembered
 *                  (later calls of that size or more take the single-kernel
 *                  decode without retrying) until the next release;
 *   encode spread  2^L bytes per block (L the encode kernel's table log,
 *                  13..15) when the slots are smaller than 512 + 2^L bytes
 *                  (fsehip_compress_blocks);
 *   header parse   520 bytes per block (the headers parsed one per lane
 *                  before the table build: batches of >= 256 blocks at
 *                  max_table_log <= 12, fsehip_build_dtables included;
 *                  without it the tables kernel parses on its own).
 * Growing a buffer synchronises the stream before freeing the old one.
 * First table build on a device (any encode or decode call): the library
 * first runs a ~1 ms synchronous self-check on the null stream (the lane
 * order of same-address LDS atomics that its rank pass relies on; the
 * slower peer-mask ranks are used if it fails), so issue one call before
 * capturing a stream into a graph. */
int fsehip_decompress_blocks(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                             const uint32_t* d_comp_len, const uint64_t* d_sidecar, uint8_t* d_out,
                             uint64_t n_total, int32_t* d_status, fsehip_stream_t stream);

/* Decode tables, built once per block (NormHistogram::read + DecodeTable,
 * histogram.rs:436-505, fse.rs:280-338) for decode-only workloads (C3):
 * d_dtables holds fsehip_dtable_bytes(max_table_log) bytes per block (entry
 * u32 = nbBits | symbol << 8 | newState << 18 for max_table_log <= 14, and
 * newState << 17 at 15), d_dtinfo one int32 per
 * block (header bytes | tableLog << 16, or a negative status).
 * The tables go to the caller's buffers, but a batch of >= 256 blocks at
 * max_table_log <= 12 first parses its headers into the stream's workspace
 * (520 bytes per block, the header-parse entry of the workspace note at
 * fsehip_decompress_blocks): the call then holds that workspace's lock, so
 * it is serialised with the library's other calls on the same stream, and
 * growing the scratch synchronises the stream (the host blocks until the
 * stream's earlier work is done).  fsehip_release_workspace frees it. */
uint64_t fsehip_dtable_bytes(uint32_t max_table_log);
int fsehip_build_dtables(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                         const uint32_t* d_comp_len, uint32_t n_blocks, uint32_t* d_dtables, int32_t* d_dtinfo,
                         fsehip_stream_t stream);
/* Decompress with prebuilt tables, with or without the sidecar (as above;
 * here slot_bytes need only be a multiple of 32, the staging loads' chunk).
 * fsehip_build_dtables requires a multiple of 256.
 * fsehip_decompress_blocks runs fsehip_build_dtables + this into a
 * per-stream workspace. */
int fsehip_decompress_blocks_dt(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                                const uint32_t* d_comp_len, const uint64_t* d_sidecar, const uint32_t* d_dtables,
                                const int32_t* d_dtinfo, uint8_t* d_out, uint64_t n_total, int32_t* d_status,
                                fsehip_stream_t stream);

/* Serial decode that also records the sidecar index (for streams produced
 * elsewhere, e.g. by the CPU crate), so later decodes run in parallel.
 * 1-state blocks: table logs <= 12 (UNSUPPORTED above). */
int fsehip_build_sidecar(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                         const uint32_t* d_comp_len, uint8_t* d_out, uint64_t n_total, uint64_t* d_sidecar_out,
                         int32_t* d_status, fsehip_stream_t stream);

/* Batched fse_decompress2 / fse_decompress (nstates 2 / 1) in the crate's
 * own termination (lib.rs:215-248 / 187-211), for streams with no sidecar
 * and no recorded raw length, e.g. many outputs of the CPU crate.  Stream b:
 * d_comp_len[b] bytes at d_in + b * in_stride (in_stride a multiple of 256
 * and at least the largest stream; d_in 16-byte aligned); its output at d_out + b *
 * out_stride, at most out_stride bytes; d_out_len[b] = bytes decoded.
 * d_status[b]: DST_TOO_SMALL when out_stride is short, SINGLE_SYMBOL for a
 * stream the crate would decode forever, UNSUPPORTED for a table log above
 * the kernels' bound or a stream above 2^28 bytes.  The bound is
 * max_table_log (0 = 11; below 11 it is 11: the smallest kernel variant);
 * the decode-table workspace is 4 << bound bytes per stream (8 KiB at 11,
 * 16 KiB at 12, 32 / 64 / 128 KiB at 13 / 14 / 15), plus 2 * out_stride + 8
 * bytes per stream for the deferred symbols of streams at bound 11 (sized by
 * the capacity out_stride, not by the bytes decoded; see the workspace note
 * at fsehip_decompress_blocks and fsehip_release_workspace).
 * out_stride must be a multiple of 16 and d_out 16-byte aligned (the decoder
 * stores 16-byte groups; BAD_ARG otherwise).
 * Serial per stream, many streams at once. */
int fsehip_decompress_streams(uint32_t nstates, uint32_t max_table_log, const uint8_t* d_in, uint64_t in_stride,
                              const uint32_t* d_comp_len, uint32_t n_streams, uint8_t* d_out, uint32_t out_stride,
                              uint32_t* d_out_len, int32_t* d_status, fsehip_stream_t stream);

/* Free the workspace of (device, stream) -- device < 0: of every device for
 * that stream handle -- after the work already enqueued on the stream, plus
 * the calling thread's staging buffers of the host entry points.  The next
 * call allocates again.  Call it before destroying a stream the library has
 * been used on.  Returns FSE_OK, or HIP if a synchronise / free failed. */
int fsehip_release_workspace(int device, fsehip_stream_t stream);

/* Compact the slot layout into one stream (blocks back to back at the byte
 * offsets d_offsets[b], an exclusive scan of d_comp_len) and back.  Used to
 * ship compressed shards between GPUs (RCCL gather) or to the host. */

int fsehip_pack_blocks(const uint8_t* d_slots, uint64_t slot_bytes, const uint32_t* d_comp_len,
                       const uint64_t* d_offsets, uint32_t n_blocks, uint8_t* d_stream, fsehip_stream_t stream);
int fsehip_unpack_blocks(const uint8_t* d_stream, const uint64_t* d_offsets, const uint32_t* d_comp_len,
                         uint32_t n_blocks, uint8_t* d_slots, uint64_t slot_bytes, fsehip_stream_t stream);

/* Move whole blocks between packed streams: block b's d_lens[b] bytes go from
 * d_src + d_src_offsets[b] to d_dst + d_dst_offsets[b] (any byte offsets;
 * ranges must not overlap).  Selects one rank's blocks out of a packed
 * stream for the distributed scatter (entropy_coders_amd/dist.py). */
int fsehip_copy_blocks(const uint8_t* d_src, const uint64_t* d_src_offsets, const uint32_t* d_lens, uint32_t n_blocks,
                       uint8_t* d_dst, const uint64_t* d_dst_offsets, fsehip_stream_t stream);

/* The bitstream as device passes over `count` fields (a prefix scan of the
 * widths places every field; HBM-bound).
 *  fsehip_bitstack_write: fields LSB-first from bit 0 of d_out; d_out must
 *    hold 4 * ceil(total / 32) bytes (<= 4 * count) and be 4-byte aligned;
 *    *d_total_bits = the bit count.
 *  fsehip_bitstack_read / fsehip_bitstream_read: d_in readable up to
 *    roundup(n_bytes, 4); d_result[0] = reads that succeed, [1] = 1 when
 *    they consume every available bit, [2] = status (NO_MARKER for a stack
 *    without its marker). */
int fsehip_bitstack_write(const uint32_t* d_vals, const uint8_t* d_nbits, uint64_t count, uint8_t* d_out,
                          uint64_t out_cap, uint64_t* d_total_bits, fsehip_stream_t stream);
int fsehip_bitstack_read(const uint8_t* d_in, uint64_t n_bytes, const uint8_t* d_nbits, uint64_t count,
                         uint32_t* d_vals, uint64_t* d_result, fsehip_stream_t stream);
int fsehip_bitstream_read(const uint8_t* d_in, uint64_t n_bytes, uint64_t total_bits, const uint8_t* d_nbits,
                          uint64_t count, uint32_t* d_vals, uint64_t* d_result, fsehip_stream_t stream);
/* The same with per-field ops (FSE_BITS_READ / PEEK / ADVANCE, device
 * pointer; NULL = all reads). */
int fsehip_bitstream_read_ops(const uint8_t* d_in, uint64_t n_bytes, uint64_t total_bits, const uint8_t* d_nbits,
                              const uint8_t* d_ops, uint64_t count, uint32_t* d_vals, uint64_t* d_result,
                              fsehip_stream_t stream);

/* histogram::count per block: d_counts[b*256 + s], d_table_len[b]. */
int fsehip_histogram_blocks(const uint8_t* d_src, uint64_t n_total, uint32_t block_size, uint32_t* d_counts,
                            uint32_t* d_table_len, fsehip_stream_t stream);

/* Synthetic input (bench/tests): kind 0 = LUT generator of
 * benches/fse_benchmark.rs:5-20 with probability prob, 1 = geometric p=0.5,
 * 2 = uniform 0..239; counter-based splitmix64 (see oracle fo_generate). */
int fsehip_generate(int kind, double prob, uint64_t seed, uint32_t block_size, uint8_t* d_out,
                    uint64_t n_total, fsehip_stream_t stream);

/* Self-check of the table builds.  Every stateTable and decode table ranks its
 * positions with one LDS atomic per 64 positions (fse.rs:157-162, 329-337
 * order), which relies on an undocumented lane order of same-address LDS
 * atomics, so every table checks its ranks and is rebuilt with lane-matching
 * ranks when the check fails.  counts[0..2] = the rebuilds so far on `device`
 * by the batch encoder, the decode-table builds and the building-block table
 * calls (0 on a correct GPU); reset != 0 zeroes them after reading.
 * Synchronous. */
int fsehip_rank_fallbacks(int device, uint32_t counts[3], int reset);

/* Device count visible to this process (0 when HIP is unusable). */
int fsehip_device_count(void);
/* Library build identifier. */
const char* fsehip_version(void);

#ifdef __cplusplus
}
#endif
#endif
