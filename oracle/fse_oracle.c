/*
 * fse_oracle.c -- CPU restatement of Cognoscan/entropy_coders (parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY (see fse_oracle.h).  Restates the reference's
 * algorithm; it is not a translation of its code: the reference's pointer-
 * alignment-driven BitStackWriter/BitStackReader are restated by their
 * observable semantics (an exact LSB-first bit stack), which the reference's
 * own tests pin at all 8 byte offsets (bitstream/mod.rs:112-165).
 */
#include "fse_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t ilog2_u32(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
static inline uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
static inline uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }

/* ======================================================================
 * Bit I/O
 * ====================================================================== */

/* BitStackWriter (writer.rs:5-223): bits are appended LSB-first into a
 * 64-bit accumulator and flushed 32 bits at a time (writer.rs:43-110); byte
 * k of the output holds stream bits 8k..8k+7; finish() zero-pads the last
 * byte (writer.rs:201-222).  Every writer in the codec starts on a byte
 * boundary (the payload writer starts after the padded header, lib.rs:151). */
typedef struct {
    uint8_t* buf;
    size_t cap;
    size_t byte;   /* next byte to store */
    uint64_t acc;  /* pending bits, LSB = next stream bit */
    unsigned nacc; /* number of pending bits (< 32 between puts) */
    int overflow;
} bw_t;

static void bw_init(bw_t* w, uint8_t* buf, size_t cap, size_t byte_start) {
    w->buf = buf;
    w->cap = cap;
    w->byte = byte_start;
    w->acc = 0;
    w->nacc = 0;
    w->overflow = 0;
}

/* write_bits_raw(_unmasked) (writer.rs:140-180): value masked to nbits<=16,
 * then a flush of one 32-bit word when >= 32 bits are pending.            */
static inline void bw_put(bw_t* w, uint64_t val, unsigned nbits) {
    val &= (1ull << nbits) - 1ull;
    w->acc |= val << w->nacc;
    w->nacc += nbits;
    if (w->nacc >= 32) {
        if (w->byte + 4 <= w->cap) {
            uint32_t word = (uint32_t)w->acc;
            memcpy(w->buf + w->byte, &word, 4); /* little-endian host */
        } else {
            w->overflow = 1;
        }
        w->byte += 4;
        w->acc >>= 32;
        w->nacc -= 32;
    }
}

static inline uint64_t bw_pos(const bw_t* w) { return (uint64_t)w->byte * 8u + w->nacc; }

/* finish(): store the pending bytes, total = ceil(bits/8) (writer.rs:441). */
static size_t bw_finish_bytes(bw_t* w) {
    unsigned nbytes = (w->nacc + 7u) >> 3;
    for (unsigned i = 0; i < nbytes; ++i) {
        if (w->byte + i < w->cap) w->buf[w->byte + i] = (uint8_t)(w->acc >> (8u * i));
        else w->overflow = 1;
    }
    return w->byte + nbytes;
}

/* BitStackReader (stack_reader.rs:5-227) restated as an exact stack:
 * new() fails on an empty slice or a zero last byte (18-20, 77-83); the
 * marker is the highest set bit; pop(n) returns the n most recently written
 * bits or fails iff fewer than n remain (176-197).  The reference's reload
 * discipline (buffer >= 32 bits after each reload) guarantees reads never
 * fail spuriously for n <= 16 in the codec loops (lib.rs:198-207, 227-241). */
typedef struct {
    const uint8_t* buf;
    size_t len;
    uint64_t top; /* number of bits remaining below the marker */
} sr_t;

static int sr_init(sr_t* r, const uint8_t* buf, size_t n) {
    if (n == 0) return FSE_ERR_NO_MARKER;
    uint8_t last = buf[n - 1];
    if (last == 0) return FSE_ERR_NO_MARKER;
    r->buf = buf;
    r->len = n;
    r->top = (uint64_t)(n - 1) * 8u + ilog2_u32(last);
    return FSE_OK;
}

static inline uint32_t load_le32(const uint8_t* buf, size_t len, size_t b) {
    uint32_t w = 0;
    if (b + 4 <= len) {
        memcpy(&w, buf + b, 4);
    } else {
        for (size_t i = 0; b + i < len && i < 4; ++i) w |= (uint32_t)buf[b + i] << (8u * i);
    }
    return w;
}

/* peek/read (n <= 16): value bit i = stream bit (top - n + i). */
static inline int sr_pop(sr_t* r, unsigned nbits, uint32_t* val) {
    if ((uint64_t)nbits > r->top) return 0;
    uint64_t base = r->top - nbits;
    uint32_t w = load_le32(r->buf, r->len, (size_t)(base >> 3));
    *val = (w >> (base & 7u)) & ((1u << nbits) - 1u);
    r->top = base;
    return 1;
}

/* BitStreamReader (stream_reader.rs:5-136): forward LSB-first reader over
 * total_bits = 8*len bits; a peek/advance past total_bits is UnexpectedEof
 * (70-72, 85-87).                                                           */
typedef struct {
    const uint8_t* buf;
    uint64_t total;
    uint64_t pos;
} fr_t;

static int fr_peek(const fr_t* r, unsigned nbits, uint32_t* val) {
    if (r->pos + nbits > r->total) return 0;
    uint32_t v = 0;
    for (unsigned i = 0; i < nbits; ++i) {
        uint64_t p = r->pos + i;
        v |= (uint32_t)((r->buf[p >> 3] >> (p & 7u)) & 1u) << i;
    }
    *val = v;
    return 1;
}
static int fr_advance(fr_t* r, unsigned nbits) {
    if (r->pos + nbits > r->total) return 0;
    r->pos += nbits;
    return 1;
}
static int fr_read(fr_t* r, unsigned nbits, uint32_t* val) {
    if (!fr_peek(r, nbits, val)) return 0;
    r->pos += nbits;
    return 1;
}

/* ======================================================================
 * Histogram / normalisation / header  (histogram.rs)
 * ====================================================================== */

/* Histogram::new, histogram.rs:18-66.  The 4-way privatisation (20-50) is a
 * speed device; the result is the plain count.  table_len = 1 + the largest
 * symbol seen, or 1 when the input is empty (52-59).                        */
int fo_hist_count(const uint8_t* src, size_t n, fo_hist* h) {
    if (n > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG; /* assert at 19 */
    memset(h, 0, sizeof(*h));
    for (size_t i = 0; i < n; ++i) h->counts[src[i]]++;
    uint32_t tl = 0;
    for (int s = 255; s >= 0; --s)
        if (h->counts[s]) { tl = (uint32_t)s; break; }
    h->table_len = tl + 1;
    h->size = (uint32_t)n;
    return FSE_OK;
}

/* optimal_log2, histogram.rs:264-277.  u32 `(size-1).ilog2() - 2` wraps in
 * a release build for n = 2..4 (the bench profile); ilog2(0) always panics. */
int fo_optimal_log2(const fo_hist* h, uint32_t* out) {
    if (h->size == 0) return FSE_ERR_EMPTY;             /* size.ilog2() */
    uint32_t min_bits_src = ilog2_u32(h->size) + 1u;
    if (h->table_len <= 1) return FSE_ERR_ALL_ZERO_SYMBOL0; /* (tl-1).ilog2() */
    uint32_t min_bits_sym = ilog2_u32(h->table_len - 1u) + 2u;
    uint32_t min_bits = umin32(min_bits_src, min_bits_sym);
    if (h->size == 1) return FSE_ERR_TOO_SHORT;         /* (size-1).ilog2() */
    uint32_t max_bits = ilog2_u32(h->size - 1u) - 2u;   /* wrapping u32 */
    uint32_t L = umin32(FO_LOG_DEFAULT, max_bits);
    L = umax32(L, min_bits);
    if (L < FO_LOG_MIN) L = FO_LOG_MIN;
    if (L > FO_LOG_MAX) L = FO_LOG_MAX;
    *out = L;
    return FSE_OK;
}

static const uint32_t RTB_TABLE[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};

#define UNASSIGNED (-2)

/* normalize_slow, histogram.rs:157-261 (u32 counters, u64 fixed point). */
static int normalize_slow(const fo_hist* h, uint32_t L, fo_norm* out) {
    const uint32_t tl = h->table_len;
    uint32_t low_threshold = h->size >> L;
    uint32_t low_one = (uint32_t)(h->size * 3u) >> (L + 1u); /* wrapping */
    uint32_t to_distribute = 1u << L;
    uint32_t total = h->size;
    memset(out->norm, 0, sizeof(out->norm));
    out->log2 = L;
    out->table_len = tl;

    for (uint32_t s = 0; s < tl; ++s) { /* 167-181 */
        uint32_t t = h->counts[s];
        if (t == 0) continue;
        if (t <= low_threshold) {
            out->norm[s] = -1; to_distribute -= 1; total -= t;
        } else if (t <= low_one) {
            out->norm[s] = 1; to_distribute -= 1; total -= t;
        } else {
            out->norm[s] = UNASSIGNED;
        }
    }
    if (to_distribute == 0) return FSE_OK; /* 183-189 */

    if (total / to_distribute > low_one) { /* 192-201 */
        uint32_t low = (uint32_t)(total * 3u) / (uint32_t)(to_distribute * 2u);
        for (uint32_t s = 0; s < tl; ++s) {
            uint32_t t = h->counts[s];
            if (out->norm[s] == UNASSIGNED && t <= low) {
                out->norm[s] = 1; to_distribute -= 1; total -= t;
            }
        }
    }

    if ((uint32_t)((1u << L) - to_distribute) == tl) { /* 203-220 */
        uint32_t v_max = 0, i_max = 0;
        for (uint32_t s = 0; s < 256; ++s)
            if (h->counts[s] > v_max) { v_max = h->counts[s]; i_max = s; }
        out->norm[i_max] += (int32_t)to_distribute;
        return FSE_OK;
    } else if (total == 0) { /* 221-235 */
        while (to_distribute != 0) {
            int progressed = 0;
            for (uint32_t s = 0; s < tl; ++s) {
                if (out->norm[s] > 0) {
                    out->norm[s] += 1; to_distribute -= 1; progressed = 1;
                    if (to_distribute == 0) break;
                }
            }
            if (!progressed) return FSE_ERR_CURSED; /* reference loops forever */
        }
    } else { /* 236-254 */
        uint64_t v_step_log = 62u - (uint64_t)L;
        uint64_t mid = (1ull << (v_step_log - 1u)) - 1u;
        uint64_t r_step = (((1ull << v_step_log) * (uint64_t)to_distribute) + mid) / (uint64_t)total;
        uint64_t tmp_total = mid;
        for (uint32_t s = 0; s < tl; ++s) {
            if (out->norm[s] == UNASSIGNED) {
                uint64_t end = tmp_total + (uint64_t)h->counts[s] * r_step;
                uint64_t weight = (end >> v_step_log) - (tmp_total >> v_step_log);
                if (weight < 1) return FSE_ERR_CURSED; /* panic at 248 */
                out->norm[s] = (int32_t)weight;
                tmp_total = end;
            }
        }
    }
    return FSE_OK;
}

/* Histogram::normalize, histogram.rs:95-155. */
int fo_normalize(const fo_hist* h, uint32_t log2, fo_norm* out, int* used_slow) {
    if (used_slow) *used_slow = 0;
    if (h->table_len <= 1) return FSE_ERR_ALL_ZERO_SYMBOL0; /* 98: ilog2(0) */
    if (h->size == 0) return FSE_ERR_EMPTY;                 /* 103: div by 0 */
    uint32_t L = log2 < FO_LOG_MIN ? FO_LOG_MIN : (log2 > FO_LOG_MAX ? FO_LOG_MAX : log2);
    L = umax32(L, ilog2_u32(h->table_len - 1u) + 2u);

    const uint64_t scale = 62u - (uint64_t)L;
    const uint64_t step = (1ull << 62) / (uint64_t)h->size;
    const uint64_t v_step = 1ull << (scale - 20u);
    const uint32_t low_threshold = h->size >> L;
    int32_t to_distribute = (int32_t)(1u << L);
    uint32_t largest = 0;
    int32_t largest_prob = 0;

    memset(out->norm, 0, sizeof(out->norm));
    out->log2 = L;
    out->table_len = h->table_len;

    for (uint32_t i = 0; i < h->table_len; ++i) { /* 112-141 */
        uint32_t t = h->counts[i];
        if (t == h->size) { out->norm[i] = to_distribute; return FSE_OK; }
        if (t == 0) continue;
        if (t <= low_threshold) { out->norm[i] = -1; to_distribute -= 1; continue; }
        uint64_t prob = ((uint64_t)t * step) >> scale;
        if (prob < 8) {
            uint64_t rest_to_beat = v_step * (uint64_t)RTB_TABLE[prob];
            prob += (((uint64_t)t * step - (prob << scale)) > rest_to_beat) ? 1u : 0u;
        }
        int32_t p = (int32_t)prob;
        if (p > largest_prob) { largest_prob = p; largest = i; }
        out->norm[i] = p;
        to_distribute -= p;
    }
    if (to_distribute != 0 && -to_distribute >= (largest_prob >> 1)) { /* 144-145 */
        if (used_slow) *used_slow = 1;
        return normalize_slow(h, L, out);
    }
    out->norm[largest] += to_distribute; /* 147 */
    return FSE_OK;
}

/* NormHistogram::new, histogram.rs:299-303. */
int fo_norm_new(const uint8_t* src, size_t n, fo_norm* out) {
    fo_hist h;
    int rc = fo_hist_count(src, n, &h);
    if (rc) return rc;
    uint32_t L;
    rc = fo_optimal_log2(&h, &L);
    if (rc) return rc;
    return fo_normalize(&h, L, out, NULL);
}

/* write_bound, histogram.rs:330-337 */
size_t fo_header_write_bound(const fo_norm* nh) {
    size_t m = (((size_t)nh->table_len * nh->log2) >> 3) + 3;
    return nh->table_len > 1 ? m : 512;
}

/* NormHistogram::write, histogram.rs:376-431. */
int fo_header_write(const fo_norm* nh, uint8_t* dst, size_t cap, size_t* len) {
    bw_t w;
    bw_init(&w, dst, cap, 0);
    bw_put(&w, nh->log2 - FO_LOG_MIN, 4); /* 380-381 */
    int32_t threshold = 1 << nh->log2;
    int32_t remaining = threshold + 1;
    uint32_t zero_count = 0;
    uint32_t num_bits = nh->log2 + 1u;
    for (uint32_t i = 0; i < nh->table_len; ++i) {
        int32_t s = nh->norm[i];
        if (remaining <= 1) break;
        if (zero_count != 0) { /* 391-409 */
            if (s == 0) { zero_count += 1; continue; }
            zero_count -= 1;
            while (zero_count >= 24) { bw_put(&w, 0xFFFF, 16); zero_count -= 24; }
            while (zero_count >= 3) { bw_put(&w, 0x3, 2); zero_count -= 3; }
            bw_put(&w, zero_count, 2);
        }
        int32_t max = (2 * threshold - 1) - remaining; /* 410 */
        remaining -= (s < 0 ? -s : s);
        int32_t count = s + 1;
        if (count >= threshold) count += max;
        uint32_t bits_to_write = num_bits - (count < max ? 1u : 0u);
        bw_put(&w, (uint64_t)(uint32_t)count, bits_to_write);
        zero_count = (count == 1) ? 1u : 0u;
        if (remaining < 1) return FSE_ERR_BAD_TABLE; /* panic at 420 */
        while (remaining < threshold) { num_bits -= 1; threshold >>= 1; }
    }
    if (w.overflow) return FSE_ERR_DST_TOO_SMALL;
    *len = bw_finish_bytes(&w);
    return FSE_OK;
}

/* NormHistogram::read, histogram.rs:436-505. */
int fo_header_read(const uint8_t* src, size_t n, fo_norm* out, size_t* consumed) {
    if (n == 0) return FSE_ERR_EMPTY; /* BitStreamReader::new assert */
    fr_t r = {src, (uint64_t)n * 8u, 0};
    uint32_t v;
    if (!fr_read(&r, 4, &v)) return FSE_ERR_BAD_HEADER;
    uint32_t log2 = v + FO_LOG_MIN;
    if (log2 > FO_LOG_MAX) return FSE_ERR_BAD_HEADER; /* TableLogTooLarge */
    memset(out->norm, 0, sizeof(out->norm));
    out->log2 = log2;
    uint64_t symbol = 0;
    uint64_t threshold = 1ull << log2;
    uint64_t remaining = threshold + 1;
    uint32_t nb = log2 + 1u;
    int previous0 = 0;
    while (remaining > 1 && symbol < 256) {
        if (previous0) { /* 455-465 */
            for (;;) {
                uint32_t pk;
                if (!fr_peek(&r, 16, &pk)) pk = 0;
                if (pk != 0xFFFF) break;
                if (!fr_advance(&r, 16)) return FSE_ERR_BAD_HEADER;
                symbol += 24;
            }
            for (;;) {
                uint32_t pk;
                if (!fr_peek(&r, 2, &pk)) pk = 0;
                if (pk != 3) break;
                if (!fr_advance(&r, 2)) return FSE_ERR_BAD_HEADER;
                symbol += 3;
            }
            if (!fr_read(&r, 2, &v)) return FSE_ERR_BAD_HEADER;
            symbol += v;
        }
        if (symbol >= 256) break;
        uint64_t max = (2 * threshold - 1) - remaining; /* 470 */
        uint32_t raw;
        if (!fr_peek(&r, nb, &raw) && !fr_peek(&r, nb - 1u, &raw)) return FSE_ERR_BAD_HEADER;
        uint64_t value;
        if (((uint64_t)raw & (threshold - 1)) < max) {
            if (!fr_advance(&r, nb - 1u)) return FSE_ERR_BAD_HEADER;
            value = (uint64_t)raw & (threshold - 1);
        } else {
            if (!fr_advance(&r, nb)) return FSE_ERR_BAD_HEADER;
            value = (uint64_t)raw & (2 * threshold - 1);
            if (value >= threshold) value -= max;
        }
        int32_t sv = (int32_t)value - 1;
        remaining -= (uint64_t)(sv < 0 ? -sv : sv);
        out->norm[symbol] = sv;
        symbol += 1;
        previous0 = (sv == 0);
        while (remaining < threshold) { nb -= 1; threshold >>= 1; }
    }
    if (remaining != 1) return FSE_ERR_BAD_HEADER; /* TooManySymbols */
    out->table_len = (uint32_t)symbol;
    *consumed = (size_t)((r.pos + 7u) >> 3); /* finish_byte, 132-135 */
    return FSE_OK;
}

/* ======================================================================
 * Tables (fse.rs)
 * ====================================================================== */

/* table_step, fse.rs:67-70 */
static inline uint32_t table_step(uint32_t size) { return size * 5u / 8u + 3u; }

/* Symbol spread shared by both tables (fse.rs:110-151 / 294-326).  Returns
 * the high threshold; -1 entries fill the top, others step by 5/8*size+3
 * skipping positions above the threshold.  Entries never written keep 0
 * (Vec::resize default, fse.rs:112 / 292).                                 */
static int spread_symbols(const fo_norm* nh, uint8_t* spread) {
    const uint32_t size = 1u << nh->log2;
    int64_t high_threshold = (int64_t)size - 1;
    memset(spread, 0, size);
    for (uint32_t s = 0; s < nh->table_len; ++s) {
        if (nh->norm[s] == -1 || nh->norm[s] < -1) {
            if (high_threshold >= 0) spread[high_threshold] = (uint8_t)s;
            high_threshold -= 1;
        }
    }
    uint32_t position = 0;
    const uint32_t mask = size - 1, step = table_step(size);
    for (uint32_t s = 0; s < nh->table_len; ++s) {
        for (int32_t k = 0; k < nh->norm[s]; ++k) {
            spread[position] = (uint8_t)s;
            position = (position + step) & mask;
            while ((int64_t)position > high_threshold) position = (position + step) & mask;
        }
    }
    if (position != 0) return FSE_ERR_BAD_TABLE; /* assert fse.rs:151/326 */
    return FSE_OK;
}

/* EncodeTable::update, fse.rs:101-189. */
int fo_build_ctable(const fo_norm* nh, fo_ctable* ct) {
    const uint32_t L = nh->log2;
    if (L < FO_LOG_MIN || L > FO_LOG_MAX) return FSE_ERR_TABLELOG_RANGE; /* 103-106 */
    const uint32_t size = 1u << L;
    uint32_t cumul[256];
    uint32_t acc = 0;
    for (uint32_t s = 0; s < 256; ++s) cumul[s] = 0;
    for (uint32_t s = 0; s < nh->table_len; ++s) { /* 119-129 */
        cumul[s] = acc;
        acc += (nh->norm[s] == -1) ? 1u : (uint32_t)nh->norm[s];
    }
    ct->log2 = L;
    int rc = spread_symbols(nh, ct->spread);
    if (rc) return rc;
    for (uint32_t i = 0; i < size; ++i) { /* 157-162 */
        uint8_t x = ct->spread[i];
        ct->st[cumul[x]] = (uint16_t)(size + i);
        cumul[x] += 1;
    }
    int32_t total = 0; /* 165-188 */
    for (uint32_t s = 0; s < 256; ++s) { ct->dnb[s] = 0; ct->dfs[s] = 0; }
    for (uint32_t s = 0; s < nh->table_len; ++s) {
        int32_t x = nh->norm[s];
        if (x == 0) {
            ct->dnb[s] = ((L + 1u) << 16) - (1u << L);
        } else if (x == -1 || x == 1) {
            ct->dnb[s] = (L << 16) - (1u << L);
            ct->dfs[s] = total - 1;
            total += 1;
        } else {
            uint32_t max_bits_out = L - ilog2_u32((uint32_t)(x - 1));
            uint32_t min_state_plus = (uint32_t)x << max_bits_out;
            ct->dnb[s] = (max_bits_out << 16) - min_state_plus;
            ct->dfs[s] = total - x;
            total += x;
        }
    }
    return FSE_OK;
}

/* DecodeTable::update, fse.rs:280-338. */
int fo_build_dtable(const fo_norm* nh, fo_dtable* dt) {
    const uint32_t L = nh->log2;
    if (L < FO_LOG_MIN || L > FO_LOG_MAX) return FSE_ERR_TABLELOG_RANGE; /* 282-285 */
    const uint32_t size = 1u << L;
    uint16_t symbol_next[256];
    memset(symbol_next, 0, sizeof(symbol_next));
    for (uint32_t s = 0; s < nh->table_len; ++s) /* 298-310 */
        symbol_next[s] = (nh->norm[s] <= -1) ? 1 : (uint16_t)nh->norm[s];
    dt->log2 = L;
    int rc = spread_symbols(nh, dt->sym);
    if (rc) return rc;
    for (uint32_t i = 0; i < size; ++i) { /* 329-337 */
        uint8_t s = dt->sym[i];
        uint16_t next_state = symbol_next[s]++;
        if (next_state == 0) return FSE_ERR_BAD_TABLE; /* ilog2(0) panic */
        uint32_t num_bits = L - ilog2_u32(next_state);
        dt->nb[i] = (uint8_t)num_bits;
        dt->new_state[i] = (uint16_t)(((uint32_t)next_state << num_bits) - size);
    }
    return FSE_OK;
}

/* ======================================================================
 * Coders (fse.rs:196-386)
 * ====================================================================== */

/* Encoder::new_first_symbol, fse.rs:210-218 */
/* Encoder::new_first_symbol, fse.rs:210-218, with Rust release semantics:
 * u32 wrapping arithmetic, the index formed as an i32 (wrapping add, fse.rs:
 * 215) and converted to usize, then the bounds-checked table read.  At
 * tableLog 15 the rounding constant 1 << 15 no longer covers the smallest
 * state of a symbol with norm >= 2: the subtraction wraps and the index
 * usually lands outside the table, where the reference panics (index out of
 * bounds) -> FSE_ERR_ENCODER_INIT; a power-of-two norm can instead land on
 * another symbol's state, which the reference then uses as is. */
static inline int enc_init(const fo_ctable* ct, uint8_t sym, uint32_t* out) {
    uint32_t bits = ct->dnb[sym];
    uint32_t bits_out = (bits + (1u << 15)) >> 16;
    uint32_t value = (bits_out << 16) - bits;
    int32_t idx = (int32_t)((value >> bits_out) + (uint32_t)ct->dfs[sym]);
    if (idx < 0 || (uint32_t)idx >= (1u << ct->log2)) return FSE_ERR_ENCODER_INIT;
    *out = ct->st[idx];
    return FSE_OK;
}

/* Encoder::encode_raw, fse.rs:227-239 */
static inline void enc_step(const fo_ctable* ct, uint32_t* value, uint8_t sym, bw_t* w) {
    uint32_t bits_out = (ct->dnb[sym] + *value) >> 16;
    bw_put(w, *value, bits_out);
    int64_t idx = (int64_t)(*value >> bits_out) + ct->dfs[sym];
    *value = ct->st[(size_t)idx];
}

/* Encoder::finish, fse.rs:248-250 */
static inline void enc_finish(const fo_ctable* ct, uint32_t value, bw_t* w) { bw_put(w, value, ct->log2); }

/* Decoder::decode_symbol(_no_reload), fse.rs:363-380: 0 when the reader
 * cannot supply num_bits (the loop terminator). */
static inline int dec_step(const fo_dtable* dt, uint32_t* state, sr_t* r, uint8_t* sym) {
    uint32_t bits;
    if (!sr_pop(r, dt->nb[*state], &bits)) return 0;
    *sym = dt->sym[*state];
    *state = dt->new_state[*state] + bits;
    *state &= 0xFFFFu; /* u16 state */
    return 1;
}

/* fse_compress2 body after the histogram, lib.rs:149-182 */
static int compress2_body(const uint8_t* src, size_t n, const fo_norm* nh, uint8_t* dst,
                          size_t cap, size_t* out_len, uint64_t* payload_bits) {
    if (n < 2) return FSE_ERR_TOO_SHORT; /* unwrap at lib.rs:154 / 156 */
    size_t hlen;
    int rc = fo_header_write(nh, dst, cap, &hlen);
    if (rc) return rc;
    static __thread fo_ctable ct;
    rc = fo_build_ctable(nh, &ct);
    if (rc) return rc;
    bw_t w;
    bw_init(&w, dst, cap, hlen);
    uint32_t e0, e1;
    size_t pairs; /* number of full pairs handled by the main loop */
    if (n & 1) { /* 155-160 */
        if ((rc = enc_init(&ct, src[n - 1], &e0)) || (rc = enc_init(&ct, src[n - 2], &e1))) return rc;
        enc_step(&ct, &e0, src[n - 3], &w); /* n odd and >= 2, so n >= 3 */
        pairs = (n - 3) / 2;
    } else { /* 161-165 */
        if ((rc = enc_init(&ct, src[n - 2], &e0)) || (rc = enc_init(&ct, src[n - 1], &e1))) return rc;
        pairs = n / 2 - 1;
    }
    for (size_t k = pairs; k-- > 0;) { /* 167-176 */
        enc_step(&ct, &e1, src[2 * k + 1], &w);
        enc_step(&ct, &e0, src[2 * k], &w);
    }
    enc_finish(&ct, e1, &w); /* 178 */
    enc_finish(&ct, e0, &w); /* 179 */
    bw_put(&w, 1, 1);        /* 181: marker */
    if (w.overflow) return FSE_ERR_DST_TOO_SMALL;
    *out_len = bw_finish_bytes(&w);
    if (payload_bits) *payload_bits = bw_pos(&w) - (uint64_t)hlen * 8u;
    return FSE_OK;
}

int fo_compress2(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len,
                 uint64_t* payload_bits) {
    fo_norm nh;
    int rc = fo_norm_new(src, n, &nh); /* lib.rs:148 */
    if (rc) return rc;
    return compress2_body(src, n, &nh, dst, cap, out_len, payload_bits);
}

int fo_compress2_log(const uint8_t* src, size_t n, uint32_t log2, uint8_t* dst, size_t cap,
                     size_t* out_len, uint64_t* payload_bits) {
    fo_hist h;
    int rc = fo_hist_count(src, n, &h);
    if (rc) return rc;
    if (n == 0) return FSE_ERR_EMPTY;
    fo_norm nh;
    rc = fo_normalize(&h, log2, &nh, NULL);
    if (rc) return rc;
    return compress2_body(src, n, &nh, dst, cap, out_len, payload_bits);
}

/* Shared decode of fse_decompress2, lib.rs:215-248.  When raw_len is
 * non-zero, decoding stops after exactly raw_len symbols (container mode). */
static int decompress2_impl(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                            size_t* out_len, size_t raw_len) {
    fo_norm nh;
    size_t hlen;
    int rc = fo_header_read(src, n, &nh, &hlen); /* 219 */
    if (rc) return rc;
    sr_t r;
    rc = sr_init(&r, src + hlen, n - hlen); /* 222 */
    if (rc) return rc;
    static __thread fo_dtable dt;
    rc = fo_build_dtable(&nh, &dt); /* 223 */
    if (rc) return rc;
    int single = 0;
    for (uint32_t s = 0; s < nh.table_len; ++s)
        if (nh.norm[s] == (int32_t)(1u << nh.log2)) single = 1;
    if (single && raw_len == 0) return FSE_ERR_SINGLE_SYMBOL;
    uint32_t s0, s1;
    if (!sr_pop(&r, nh.log2, &s0)) return FSE_ERR_TOO_SHORT; /* 224 unwrap */
    if (!sr_pop(&r, nh.log2, &s1)) return FSE_ERR_TOO_SHORT; /* 225 unwrap */
    size_t o = 0;
    const size_t limit = raw_len ? raw_len : cap;
#define PUSH(v)                                                            \
    do {                                                                   \
        if (o >= limit) return raw_len ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; \
        dst[o++] = (v);                                                    \
    } while (0)
    for (;;) {
        uint8_t sym;
        if (raw_len && o + 2 == raw_len) { /* container mode: finals */
            PUSH(dt.sym[s0]);
            PUSH(dt.sym[s1]);
            break;
        }
        if (raw_len && o + 1 == raw_len) {
            PUSH(dt.sym[s0]);
            break;
        }
        if (!dec_step(&dt, &s0, &r, &sym)) { /* 228, 242-243 */
            PUSH(dt.sym[s0]);
            PUSH(dt.sym[s1]);
            break;
        }
        PUSH(sym);
        if (!dec_step(&dt, &s1, &r, &sym)) { /* 233-239 */
            PUSH(dt.sym[s1]);
            PUSH(dt.sym[s0]);
            break;
        }
        PUSH(sym);
    }
#undef PUSH
    if (raw_len && o != raw_len) return FSE_ERR_LENGTH_MISMATCH;
    *out_len = o;
    return FSE_OK;
}

int fo_decompress2(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    return decompress2_impl(src, n, dst, cap, out_len, 0);
}

int fo_decompress2_n(const uint8_t* src, size_t n, uint8_t* dst, size_t raw_len) {
    size_t out_len;
    if (raw_len == 0) return FSE_ERR_BAD_ARG;
    return decompress2_impl(src, n, dst, raw_len, &out_len, raw_len);
}

/* fse_compress (1 state), lib.rs:112-143 */
int fo_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len,
                uint64_t* payload_bits) {
    fo_norm nh;
    int rc = fo_norm_new(src, n, &nh); /* 114 */
    if (rc) return rc;
    size_t hlen;
    rc = fo_header_write(&nh, dst, cap, &hlen); /* 115 */
    if (rc) return rc;
    static __thread fo_ctable ct;
    rc = fo_build_ctable(&nh, &ct);
    if (rc) return rc;
    bw_t w;
    bw_init(&w, dst, cap, hlen);
    uint32_t e;
    size_t pairs;
    if ((rc = enc_init(&ct, src[n - 1], &e))) return rc;
    if (n & 1) { /* first chunk has one byte: init only (121-123) */
        pairs = (n - 1) / 2;
    } else { /* 121-126 */
        enc_step(&ct, &e, src[n - 2], &w);
        pairs = n / 2 - 1;
    }
    for (size_t k = pairs; k-- > 0;) { /* 127-138 */
        enc_step(&ct, &e, src[2 * k + 1], &w);
        enc_step(&ct, &e, src[2 * k], &w);
    }
    enc_finish(&ct, e, &w); /* 139 */
    bw_put(&w, 1, 1);       /* 141 */
    if (w.overflow) return FSE_ERR_DST_TOO_SMALL;
    *out_len = bw_finish_bytes(&w);
    if (payload_bits) *payload_bits = bw_pos(&w) - (uint64_t)hlen * 8u;
    return FSE_OK;
}

/* fse_decompress (1 state), lib.rs:187-211 */
int fo_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    fo_norm nh;
    size_t hlen;
    int rc = fo_header_read(src, n, &nh, &hlen); /* 191 */
    if (rc) return rc;
    sr_t r;
    rc = sr_init(&r, src + hlen, n - hlen); /* 192 */
    if (rc) return rc;
    static __thread fo_dtable dt;
    rc = fo_build_dtable(&nh, &dt);
    if (rc) return rc;
    for (uint32_t s = 0; s < nh.table_len; ++s)
        if (nh.norm[s] == (int32_t)(1u << nh.log2)) return FSE_ERR_SINGLE_SYMBOL;
    uint32_t st;
    if (!sr_pop(&r, nh.log2, &st)) return FSE_ERR_TOO_SHORT; /* 197 unwrap */
    size_t o = 0;
    uint8_t sym;
    while (dec_step(&dt, &st, &r, &sym)) { /* 198-207 */
        if (o >= cap) return FSE_ERR_DST_TOO_SMALL;
        dst[o++] = sym;
        if (!dec_step(&dt, &st, &r, &sym)) break;
        if (o >= cap) return FSE_ERR_DST_TOO_SMALL;
        dst[o++] = sym;
    }
    if (o >= cap) return FSE_ERR_DST_TOO_SMALL;
    dst[o++] = dt.sym[st]; /* 208 */
    *out_len = o;
    return FSE_OK;
}

/* Decode checkpoints of a compress2 stream: the decoder state just before
 * it decodes main-loop pair p (symbols 2p, 2p+1).  Used to build/verify the
 * GPU container's sidecar index (DESIGN.md "sidecar").                      */
int fo_checkpoints2(const uint8_t* src, size_t n, uint32_t interval, uint32_t* bitpos,
                    uint16_t* s0o, uint16_t* s1o, size_t cap, size_t* count) {
    fo_norm nh;
    size_t hlen;
    int rc = fo_header_read(src, n, &nh, &hlen);
    if (rc) return rc;
    sr_t r;
    rc = sr_init(&r, src + hlen, n - hlen);
    if (rc) return rc;
    static __thread fo_dtable dt;
    rc = fo_build_dtable(&nh, &dt);
    if (rc) return rc;
    uint32_t s0, s1;
    if (!sr_pop(&r, nh.log2, &s0) || !sr_pop(&r, nh.log2, &s1)) return FSE_ERR_TOO_SHORT;
    size_t c = 0;
    for (uint64_t p = 0;; ++p) {
        if (interval && p % interval == 0) {
            if (c >= cap) return FSE_ERR_DST_TOO_SMALL;
            bitpos[c] = (uint32_t)r.top;
            s0o[c] = (uint16_t)s0;
            s1o[c] = (uint16_t)s1;
            c++;
        }
        uint8_t sym;
        if (!dec_step(&dt, &s0, &r, &sym)) break;
        if (!dec_step(&dt, &s1, &r, &sym)) break;
    }
    *count = c;
    return FSE_OK;
}

/* Decode checkpoints of a 1-state (fse_compress) stream: the state just
 * before it decodes symbol p (lib.rs:197-207), every `interval` symbols.    */
int fo_checkpoints1(const uint8_t* src, size_t n, uint32_t interval, uint32_t* bitpos, uint16_t* s0o,
                    size_t cap, size_t* count) {
    fo_norm nh;
    size_t hlen;
    int rc = fo_header_read(src, n, &nh, &hlen);
    if (rc) return rc;
    sr_t r;
    rc = sr_init(&r, src + hlen, n - hlen);
    if (rc) return rc;
    static __thread fo_dtable dt;
    rc = fo_build_dtable(&nh, &dt);
    if (rc) return rc;
    uint32_t st;
    if (!sr_pop(&r, nh.log2, &st)) return FSE_ERR_TOO_SHORT;
    size_t c = 0;
    for (uint64_t p = 0;; ++p) {
        if (interval && p % interval == 0) {
            if (c >= cap) return FSE_ERR_DST_TOO_SMALL;
            bitpos[c] = (uint32_t)r.top;
            s0o[c] = (uint16_t)st;
            c++;
        }
        uint8_t sym;
        if (!dec_step(&dt, &st, &r, &sym)) break;
    }
    *count = c;
    return FSE_OK;
}

/* ======================================================================
 * Bitstream property helpers (bitstream/mod.rs:29-110)
 * ====================================================================== */
size_t fo_bits_write(const uint64_t* vals, const uint8_t* bits, size_t count, int mark,
                     uint8_t* dst, size_t cap, uint64_t* written_bits) {
    bw_t w;
    bw_init(&w, dst, cap, 0);
    for (size_t i = 0; i < count; ++i) bw_put(&w, vals[i], bits[i]);
    if (written_bits) *written_bits = bw_pos(&w);
    if (mark) bw_put(&w, 1, 1);
    if (w.overflow) return 0;
    return bw_finish_bytes(&w);
}

int fo_bits_read_stack(const uint8_t* src, size_t n, const uint8_t* bits, size_t count,
                       uint64_t* vals_out, size_t* bits_left) {
    sr_t r;
    int rc = sr_init(&r, src, n);
    if (rc) return rc;
    for (size_t i = count; i-- > 0;) {
        uint32_t v;
        if (!sr_pop(&r, bits[i], &v)) return FSE_ERR_TOO_SHORT;
        vals_out[i] = v;
    }
    if (bits_left) *bits_left = (size_t)r.top;
    return FSE_OK;
}

/* ======================================================================
 * Synthetic generators
 * ====================================================================== */
#define GOLDEN 0x9E3779B97F4A7C15ull

uint64_t fo_splitmix64_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* gen_sequence LUT, benches/fse_benchmark.rs:5-20 (u8 symbol counter wraps
 * as in a release build). */
int fo_build_lut(double prob, uint8_t lut[4096]) {
    if (prob < 0.005) prob = 0.005;
    if (prob > 0.995) prob = 0.995;
    size_t remaining = 4096, idx = 0;
    uint8_t s = 0;
    while (remaining > 0) {
        size_t n = (size_t)((double)remaining * prob);
        if (n < 1) n = 1;
        for (size_t k = 0; k < n; ++k) lut[idx++] = s;
        s = (uint8_t)(s + 1);
        remaining -= n;
    }
    return FSE_OK;
}

void fo_generate(int kind, double prob, uint64_t seed, uint64_t block_index, uint8_t* out, size_t n) {
    uint8_t lut[4096];
    if (kind == 0) fo_build_lut(prob, lut);
    const uint64_t sb = seed ^ (block_index * GOLDEN);
    for (size_t i = 0; i < n; ++i) {
        uint64_t r = fo_splitmix64_mix(sb + (uint64_t)(i + 1) * GOLDEN);
        uint8_t v;
        if (kind == 0) {
            v = lut[r & 4095u];
        } else if (kind == 1) {
            uint64_t x = r | (1ull << 63);
            unsigned c = (unsigned)__builtin_ctzll(x);
            v = (uint8_t)(c > 255 ? 255 : c);
        } else {
            v = (uint8_t)(((r >> 32) * 240u) >> 32);
        }
        out[i] = v;
    }
}

/* ======================================================================
 * Multi-threaded block baseline (CPU-N in BASELINE.md)
 * ====================================================================== */
typedef struct {
    const uint8_t* src;
    uint8_t* dst;
    size_t n_total, block, slot, b0, b1;
    const uint32_t* lens_in;
    uint32_t* lens_out;
    int rc;
} job_t;

static void* comp_worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (size_t b = j->b0; b < j->b1; ++b) {
        size_t off = b * j->block;
        size_t n = j->n_total - off < j->block ? j->n_total - off : j->block;
        size_t len = 0;
        int rc = fo_compress2(j->src + off, n, j->dst + b * j->slot, j->slot, &len, NULL);
        if (rc) { j->rc = rc; j->lens_out[b] = 0; } else j->lens_out[b] = (uint32_t)len;
    }
    return NULL;
}

static void* decomp_worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (size_t b = j->b0; b < j->b1; ++b) {
        size_t off = b * j->block;
        size_t n = j->n_total - off < j->block ? j->n_total - off : j->block;
        int rc = fo_decompress2_n(j->src + b * j->slot, j->lens_in[b], j->dst + off, n);
        if (rc) j->rc = rc;
    }
    return NULL;
}

static int run_jobs(void* (*fn)(void*), job_t* proto, size_t n_blocks, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    job_t jobs[256];
    size_t per = (n_blocks + (size_t)threads - 1) / (size_t)threads;
    int rc = FSE_OK;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = *proto;
        jobs[t].b0 = (size_t)t * per < n_blocks ? (size_t)t * per : n_blocks;
        jobs[t].b1 = jobs[t].b0 + per < n_blocks ? jobs[t].b0 + per : n_blocks;
        jobs[t].rc = FSE_OK;
        pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}

int fo_compress2_blocks(const uint8_t* src, size_t n_total, size_t block, uint8_t* dst, size_t slot,
                        uint32_t* lens, int threads) {
    size_t n_blocks = (n_total + block - 1) / block;
    job_t proto = {src, dst, n_total, block, slot, 0, 0, NULL, lens, 0};
    return run_jobs(comp_worker, &proto, n_blocks, threads);
}

int fo_decompress2_blocks(const uint8_t* src, size_t slot, const uint32_t* lens, size_t n_blocks,
                          uint8_t* dst, size_t block, size_t n_total, int threads) {
    job_t proto = {src, dst, n_total, block, slot, 0, 0, lens, NULL, 0};
    return run_jobs(decomp_worker, &proto, n_blocks, threads);
}
