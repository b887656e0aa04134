// Round-trip fuzz of the host bit cursors (entropy_coders_amd/csrc/fse_bits.cpp,
// include/fsehip.h section 1c), built by tests/test_bits_native.py with
// AddressSanitizer + UBSan: random field sequences (widths 0..32) go through
// the BitStackWriter cursor plus the marker bit (as the encoders write it,
// lib.rs:178-181), are read back newest-first with the BitStackReader cursor
// and oldest-first with the BitStreamReader cursor, from buffers allocated to
// their exact size at every address alignment, so a read or write past a
// buffer, or an undefined shift, stops the run.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/fsehip.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d case %d: %s\n", __FILE__, __LINE__, \
                         cs, #c);                                              \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int cases = argc > 1 ? std::atoi(argv[1]) : 2000;
    for (int cs = 0; cs < cases; ++cs) {
        const size_t k = (size_t)(next_u64() % (cs < 200 ? 12u : 1500u));
        std::vector<uint32_t> val(k), nb(k);
        uint64_t total = 0;
        for (size_t i = 0; i < k; ++i) {
            nb[i] = (uint32_t)(next_u64() % 33u);
            const uint64_t r = next_u64();
            val[i] = nb[i] == 32 ? (uint32_t)r : (uint32_t)(r & ((1ull << nb[i]) - 1ull));
            total += nb[i];
        }
        // writer: exact capacity (+ the marker bit), at a random offset
        const size_t pre = (size_t)(next_u64() % 5u);
        const size_t cap = pre + (size_t)((total + 1 + 7) / 8);
        uint8_t* wbuf = new uint8_t[cap ? cap : 1];
        std::memset(wbuf, 0xEE, cap);
        fse_bitstack_writer w;
        CHECK(bitstack_writer_new(&w, wbuf, cap, pre) == FSE_OK);
        for (size_t i = 0; i < k; ++i) {
            const uint32_t mode = (uint32_t)(next_u64() % 4u);
            int rc;
            if (mode == 0) rc = bitstack_writer_write_bits(&w, val[i], nb[i]);
            else if (mode == 1) rc = bitstack_writer_write_bits_unmasked(&w, val[i] | (uint32_t)(next_u64() << nb[i] % 32u) * (nb[i] < 32), nb[i]);
            else if (mode == 2) rc = bitstack_writer_write_bits_raw(&w, val[i], nb[i]);
            else rc = bitstack_writer_write_bits_raw_unmasked(&w, val[i], nb[i]);
            CHECK(rc == FSE_OK);
        }
        CHECK(bitstack_writer_write_bits(&w, 1u, 1u) == FSE_OK);  // marker
        size_t len = 0;
        uint64_t bits = 0;
        CHECK(bitstack_writer_finish(&w, &len, &bits) == FSE_OK);
        CHECK(bits == total + 1);
        CHECK(len == cap);
        // one byte less must be DST_TOO_SMALL, never a write past the buffer
        if (cap > pre) {
            uint8_t* sbuf = new uint8_t[cap - 1 ? cap - 1 : 1];
            fse_bitstack_writer s;
            CHECK(bitstack_writer_new(&s, sbuf, cap - 1, pre) == FSE_OK);
            int rc = FSE_OK;
            for (size_t i = 0; i < k && rc == FSE_OK; ++i) rc = bitstack_writer_write_bits(&s, val[i], nb[i]);
            if (rc == FSE_OK) rc = bitstack_writer_write_bits(&s, 1u, 1u);
            if (rc == FSE_OK) rc = bitstack_writer_finish(&s, &len, &bits);
            CHECK(rc == FSE_ERR_DST_TOO_SMALL);
            delete[] sbuf;
        }
        const size_t n = cap - pre;
        // stack reader over an exact-size copy at each alignment
        for (uint32_t a = 0; a < 4; ++a) {
            uint8_t* raw = new uint8_t[n + a];
            std::memcpy(raw + a, wbuf + pre, n);
            fse_bitstack_reader r;
            CHECK(bitstack_reader_new(&r, raw + a, n) == FSE_OK);
            for (size_t i = k; i-- > 0;) {
                uint32_t v = 0xDEADBEEF, pv = 0;
                CHECK(bitstack_reader_peek(&r, nb[i], &pv) == FSE_OK);
                CHECK(bitstack_reader_read(&r, nb[i], &v) == FSE_OK);
                CHECK(v == val[i] && pv == v);
            }
            CHECK(bitstack_reader_available(&r) == 0);
            CHECK(bitstack_reader_finish(&r) == 1);
            uint32_t v;
            CHECK(bitstack_reader_read(&r, 1, &v) == FSE_ERR_EOF);
            delete[] raw;
        }
        // stream reader, oldest first, over the payload bytes (marker included)
        if (n) {
            uint8_t* raw = new uint8_t[n];
            std::memcpy(raw, wbuf + pre, n);
            fse_bitstream_reader s;
            CHECK(bitstream_reader_new(&s, raw, n, total + 1) == FSE_OK);
            for (size_t i = 0; i < k; ++i) {
                uint32_t v = 0xDEADBEEF;
                if (next_u64() & 1u) {
                    CHECK(bitstream_reader_peek(&s, nb[i], &v) == FSE_OK);
                    CHECK(bitstream_reader_advance_by(&s, nb[i]) == FSE_OK);
                } else {
                    CHECK(bitstream_reader_read(&s, nb[i], &v) == FSE_OK);
                }
                CHECK(v == val[i]);
            }
            uint32_t v;
            CHECK(bitstream_reader_read(&s, 1, &v) == FSE_OK && v == 1u);
            CHECK(bitstream_reader_available(&s) == 0);
            CHECK(bitstream_reader_peek(&s, 1, &v) == FSE_ERR_EOF);
            CHECK(bitstream_reader_finish_byte(&s) == n);
            delete[] raw;
        }
        // corrupt / short inputs never read outside their buffer
        for (size_t m = 0; m < 6 && m <= n; ++m) {
            uint8_t* raw = new uint8_t[m ? m : 1];
            for (size_t i = 0; i < m; ++i) raw[i] = (uint8_t)next_u64();
            fse_bitstack_reader r;
            if (bitstack_reader_new(&r, m ? raw : nullptr, m) == FSE_OK) {
                uint32_t v;
                for (int t = 0; t < 64 && bitstack_reader_read(&r, (uint32_t)(next_u64() % 33u), &v) == FSE_OK; ++t) {
                }
            }
            delete[] raw;
        }
        delete[] wbuf;
    }
    std::printf("ok %d cases\n", cases);
    return 0;
}
