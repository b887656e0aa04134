// fse_bits.cpp -- the crate's bit readers and writer as incremental cursors
// (include/fsehip.h section 1c).
//
// BitStackReader (stack_reader.rs:5-227), BitStreamReader
// (stream_reader.rs:5-136) and BitStackWriter (writer.rs:5-223) are small
// stateful objects the crate's own callers drive one field at a time, with a
// width that depends on values read before (NormHistogram::read,
// histogram.rs:453-496; the decoders, fse.rs:354-385).  Here each is a plain
// struct the caller owns and passes to O(1) calls.  They run where their
// caller runs, on the host: one field is a few shifts, far below the cost
// of any device round trip.  Bulk bit I/O (millions of fields with known
// widths) has the batched device forms fsehip_bitstack_write/read and
// fsehip_bitstream_read(_ops); the block codecs carry their own device
// readers and writers.
//
// Semantics follow the crate on a 64-bit target (usize = u64, so the
// "half word" refills and flushes are 32 bits), including the address
// alignment the stack reader uses to place its refills: available() after
// new() and after each reload is the reference's value for the same buffer
// address.
#include <cstdint>
#include <cstring>

#include "../../include/fsehip.h"

namespace {

constexpr uint32_t HALF_BYTES = 4, HALF_BITS = 32;

// find_mask (lib.rs:15-57): (1 << n) - 1 for n <= 32
inline uint64_t mask_of(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

inline uint64_t align_offset(const uint8_t* p, uint32_t a) {
    const uintptr_t m = reinterpret_cast<uintptr_t>(p) & (a - 1u);
    return m ? a - m : 0;
}

inline int ilog2_u64(uint64_t x) { return 63 - __builtin_clzll(x); }

// BitStackReader::reload (stack_reader.rs:97-172)
void stack_reload(fse_bitstack_reader* r) {
    if (r->finished) return;
    const uint8_t* base = r->base;
    const uint8_t* ptr = r->ptr;
    if (ptr == base) {  // final readout: the bytes below the last aligned word read
        uint32_t to_read = HALF_BYTES - (uint32_t)(reinterpret_cast<uintptr_t>(ptr) & (HALF_BYTES - 1u));
        r->finished = r->bits <= HALF_BITS;
        if (!r->finished) to_read = 0;
        uint32_t rd = 0;
        for (uint32_t i = 0; i < to_read; ++i) rd |= (uint32_t)ptr[i] << (8u * i);
        const uint32_t rb = 8u * to_read;
        r->buffer = rb ? (r->buffer << rb) | rd : r->buffer;
        r->bits += rb;
        return;
    }
    const bool will = r->bits <= HALF_BITS;
    uint32_t rd;
    std::memcpy(&rd, ptr, 4);  // aligned word inside the slice (new() placed ptr)
    if (will) {
        r->buffer = (r->buffer << HALF_BITS) | rd;
        r->bits += HALF_BITS;
    }
    const uint64_t base_off = (uint64_t)(ptr - base);
    if (base_off >= HALF_BYTES)
        r->ptr = ptr - (will ? HALF_BYTES : 0u);
    else
        r->ptr = ptr - (will ? base_off : 0u);
}

}  // namespace

extern "C" {

// BitStackReader::new (stack_reader.rs:17-92)
int bitstack_reader_new(fse_bitstack_reader* r, const uint8_t* src, size_t n) {
    if (!r || (!src && n)) return FSE_ERR_BAD_ARG;
    std::memset(r, 0, sizeof(*r));
    if (n == 0) return FSE_ERR_NO_MARKER;
    const uint8_t* ptr = src + n - 1;
    const uint64_t align = align_offset(ptr, HALF_BYTES);
    if ((uint64_t)(ptr - src) > HALF_BYTES - align)
        ptr = ptr + align - HALF_BYTES;
    else
        ptr = src;
    const uint64_t to_read = n - (uint64_t)(ptr - src);  // <= 8 (at most 5 when the pointer moved)
    uint64_t buffer = 0;
    for (uint64_t i = 0; i < to_read && i < 8; ++i) buffer |= (uint64_t)ptr[i] << (8u * i);
    r->base = src;
    r->buffer = buffer;
    r->bits = (to_read < 8 ? to_read : 8) * 8u;
    r->finished = ptr == src;
    if ((uint64_t)(ptr - src) >= HALF_BYTES)
        ptr -= HALF_BYTES;
    else
        ptr = src;
    r->ptr = ptr;
    stack_reload(r);
    if (r->buffer == 0) return FSE_ERR_NO_MARKER;
    const uint64_t highbit = (uint64_t)ilog2_u64(r->buffer);
    if (r->bits - highbit > 8) return FSE_ERR_NO_MARKER;  // marker not in the last byte
    r->bits = highbit;
    stack_reload(r);
    return FSE_OK;
}

int bitstack_reader_reload(fse_bitstack_reader* r) {
    if (!r || !r->base) return FSE_ERR_BAD_ARG;
    stack_reload(r);
    return FSE_OK;
}

// peek (stack_reader.rs:176-184): None -> FSE_ERR_EOF
int bitstack_reader_peek(const fse_bitstack_reader* r, uint32_t nbits, uint32_t* val) {
    if (!r || !r->base || nbits > 32) return FSE_ERR_BAD_ARG;
    if (nbits > r->bits) return FSE_ERR_EOF;
    const uint64_t v = nbits ? (r->buffer >> (r->bits - nbits)) & mask_of(nbits) : 0u;
    if (val) *val = (uint32_t)v;
    return FSE_OK;
}

// read_no_reload (stack_reader.rs:193-197)
int bitstack_reader_read_no_reload(fse_bitstack_reader* r, uint32_t nbits, uint32_t* val) {
    const int rc = bitstack_reader_peek(r, nbits, val);
    if (rc == FSE_OK) r->bits -= nbits;
    return rc;
}

// advance_no_reload (stack_reader.rs:204-207); more bits than buffered is
// the crate's debug assertion -> BAD_ARG
int bitstack_reader_advance_no_reload(fse_bitstack_reader* r, uint32_t nbits) {
    if (!r || !r->base) return FSE_ERR_BAD_ARG;
    if (nbits > r->bits) return FSE_ERR_BAD_ARG;
    r->bits -= nbits;
    return FSE_OK;
}

// read (stack_reader.rs:211-215): read_no_reload, then reload
int bitstack_reader_read(fse_bitstack_reader* r, uint32_t nbits, uint32_t* val) {
    const int rc = bitstack_reader_read_no_reload(r, nbits, val);
    if (rc == FSE_OK) stack_reload(r);
    return rc;
}

uint64_t bitstack_reader_available(const fse_bitstack_reader* r) { return r ? r->bits : 0u; }

// finish (stack_reader.rs:224-226)
int bitstack_reader_finish(const fse_bitstack_reader* r) { return r && r->finished && r->bits == 0 ? 1 : 0; }

// BitStreamReader::new (stream_reader.rs:16-49).  The reader's cached tail
// words give exactly the zero-extended little-endian word at every index
// it can reach, so peek reads that word directly.
int bitstream_reader_new(fse_bitstream_reader* r, const uint8_t* src, size_t n, uint64_t total_bits) {
    if (!r) return FSE_ERR_BAD_ARG;
    std::memset(r, 0, sizeof(*r));
    if (!src || n == 0 || (total_bits + 7u) / 8u != n) return FSE_ERR_BAD_ARG;  // the two asserts
    r->src = src;
    r->n = n;
    r->total_bits = total_bits;
    return FSE_OK;
}

// peek (stream_reader.rs:82-114): Err(UnexpectedEof) -> FSE_ERR_EOF
int bitstream_reader_peek(const fse_bitstream_reader* r, uint32_t nbits, uint32_t* val) {
    if (!r || !r->src || nbits > 32) return FSE_ERR_BAD_ARG;
    if (r->bits_read + nbits > r->total_bits) return FSE_ERR_EOF;
    const uint64_t idx = (r->bits_read / HALF_BITS) * HALF_BYTES;
    const uint32_t off = (uint32_t)(r->bits_read & (HALF_BITS - 1u));
    uint64_t word = 0;
    for (uint32_t i = 0; i < 8u && idx + i < r->n; ++i) word |= (uint64_t)r->src[idx + i] << (8u * i);
    if (val) *val = (uint32_t)((word >> off) & mask_of(nbits));
    return FSE_OK;
}

// advance_by (stream_reader.rs:67-75)
int bitstream_reader_advance_by(fse_bitstream_reader* r, uint32_t nbits) {
    if (!r || !r->src || nbits > 32) return FSE_ERR_BAD_ARG;
    if (r->bits_read + nbits > r->total_bits) return FSE_ERR_EOF;
    r->bits_read += nbits;
    return FSE_OK;
}

// read (stream_reader.rs:56-60)
int bitstream_reader_read(fse_bitstream_reader* r, uint32_t nbits, uint32_t* val) {
    const int rc = bitstream_reader_peek(r, nbits, val);
    return rc == FSE_OK ? bitstream_reader_advance_by(r, nbits) : rc;
}

uint64_t bitstream_reader_available(const fse_bitstream_reader* r) { return r ? r->total_bits - r->bits_read : 0u; }

// finish (stream_reader.rs:123-128): remaining slice start, bits left, bit offset
int bitstream_reader_finish(const fse_bitstream_reader* r, size_t* byte, uint64_t* remaining, uint32_t* offset) {
    if (!r || !r->src) return FSE_ERR_BAD_ARG;
    if (byte) *byte = (size_t)(r->bits_read / 8u);
    if (remaining) *remaining = r->total_bits - r->bits_read;
    if (offset) *offset = (uint32_t)(r->bits_read % 8u);
    return FSE_OK;
}

// finish_byte (stream_reader.rs:132-135): start of the remaining bytes
size_t bitstream_reader_finish_byte(const fse_bitstream_reader* r) {
    return r ? (size_t)((r->bits_read + 7u) / 8u) : 0u;
}

// BitStackWriter (writer.rs:16-222) over a caller buffer: bytes are
// committed as soon as they are whole (the crate commits 32-bit words after
// aligning; the bytes are the same, writer.rs tests at 8 offsets), so fewer
// than 8 bits stay pending after every flush.  A full buffer is sticky
// FSE_ERR_DST_TOO_SMALL (the crate grows its Vec instead).
int bitstack_writer_new(fse_bitstack_writer* w, uint8_t* dst, size_t cap, size_t len) {
    if (!w) return FSE_ERR_BAD_ARG;
    std::memset(w, 0, sizeof(*w));
    if ((!dst && cap) || len > cap) return FSE_ERR_BAD_ARG;
    w->dst = dst;
    w->cap = cap;
    w->len = len;
    w->initial_len = len;
    return FSE_OK;
}

int bitstack_writer_flush(fse_bitstack_writer* w) {
    if (!w) return FSE_ERR_BAD_ARG;
    if (w->status) return w->status;
    while (w->bits >= 8u) {
        if (w->len >= w->cap) return w->status = FSE_ERR_DST_TOO_SMALL;
        w->dst[w->len++] = (uint8_t)w->storage;
        w->storage >>= 8;
        w->bits -= 8u;
    }
    return FSE_OK;
}

// write_bits_raw (writer.rs:164-180): the value's unused bits must be zero
int bitstack_writer_write_bits_raw(fse_bitstack_writer* w, uint32_t val, uint32_t nbits) {
    if (!w || nbits > 32) return FSE_ERR_BAD_ARG;
    if (w->status) return w->status;
    if (w->bits + nbits > 64u) {  // more than the crate allows between flushes: flush first
        const int rc = bitstack_writer_flush(w);
        if (rc) return rc;
    }
    // a 0-bit write after 64 pending bits (possible without a flush) would
    // shift by 64
    if (nbits) w->storage |= (uint64_t)val << w->bits;
    w->bits += nbits;
    return FSE_OK;
}

// write_bits_raw_unmasked (writer.rs:140-149): masks the value first
int bitstack_writer_write_bits_raw_unmasked(fse_bitstack_writer* w, uint32_t val, uint32_t nbits) {
    return bitstack_writer_write_bits_raw(w, (uint32_t)(val & mask_of(nbits)), nbits);
}

// write_bits / write_bits_unmasked (writer.rs:185-198): write + flush
int bitstack_writer_write_bits(fse_bitstack_writer* w, uint32_t val, uint32_t nbits) {
    const int rc = bitstack_writer_write_bits_raw(w, val, nbits);
    return rc ? rc : bitstack_writer_flush(w);
}

int bitstack_writer_write_bits_unmasked(fse_bitstack_writer* w, uint32_t val, uint32_t nbits) {
    const int rc = bitstack_writer_write_bits_raw_unmasked(w, val, nbits);
    return rc ? rc : bitstack_writer_flush(w);
}

// finish (writer.rs:201-222): pad the last byte with zeros; *dst_len = the
// buffer's new length, *bits_written = bits written since new()
int bitstack_writer_finish(fse_bitstack_writer* w, size_t* dst_len, uint64_t* bits_written) {
    if (!w) return FSE_ERR_BAD_ARG;
    int rc = bitstack_writer_flush(w);
    if (rc) return rc;
    const uint64_t total = (uint64_t)(w->len - w->initial_len) * 8u + w->bits;
    if (w->bits) {
        if (w->len >= w->cap) return w->status = FSE_ERR_DST_TOO_SMALL;
        w->dst[w->len++] = (uint8_t)(w->storage & mask_of(w->bits));
        w->storage = 0;
        w->bits = 0;
    }
    if (dst_len) *dst_len = w->len;
    if (bits_written) *bits_written = total;
    return FSE_OK;
}

}  // extern "C"
