/* The oracle (oracle/fse_oracle.c, test infrastructure) under AddressSanitizer
 * + UBSan, built by tests/test_bits_native.py: random blocks of several
 * distributions through fo_compress2 / fo_compress2_log / fo_compress and
 * back, from exact-size copies of the compressed bytes, plus truncated and
 * corrupted streams, which must end in a status without touching memory
 * outside their buffers. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/fse_oracle.h"

static uint64_t st = 0x243F6A8885A308D3ull;
static uint64_t rnd(void) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void fill(uint8_t* b, size_t n) {
    const int kind = (int)(rnd() % 5u);
    if (kind == 0) {
        fo_generate(0, 0.03 + (double)(rnd() % 1000u) / 1100.0, rnd(), 0, b, n);
    } else if (kind == 1) {  /* a few symbols */
        const uint32_t k = 2u + (uint32_t)(rnd() % 7u);
        uint8_t a[8];
        for (uint32_t i = 0; i < k; ++i) a[i] = (uint8_t)rnd();
        for (size_t i = 0; i < n; ++i) b[i] = a[(rnd() % 97u) % k ? rnd() % k : 0];
    } else if (kind == 2) {
        for (size_t i = 0; i < n; ++i) b[i] = (uint8_t)rnd();
    } else if (kind == 3) {
        memset(b, (int)(rnd() % 3u), n);
    } else {
        for (size_t i = 0; i < n; ++i) b[i] = (uint8_t)(rnd() % 64u == 0 ? rnd() : 7u);
    }
}

static uint8_t* dup(const uint8_t* p, size_t n) {
    uint8_t* q = (uint8_t*)malloc(n ? n : 1);
    memcpy(q, p, n);
    return q;
}

int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 400;
    for (int cs = 0; cs < cases; ++cs) {
        const size_t n = 1 + (size_t)(rnd() % (cs % 8 == 0 ? 200000u : 9000u));
        uint8_t* src = (uint8_t*)malloc(n);
        fill(src, n);
        const size_t cap = 512 + (n * 15 + 7) / 8 + 16;
        uint8_t* c = (uint8_t*)malloc(cap);
        uint8_t* d = (uint8_t*)malloc(n);
        for (int fmt = 0; fmt < 3; ++fmt) {
            size_t clen = 0, dlen = 0;
            uint64_t pbits = 0;
            const uint32_t L = (uint32_t)(rnd() % 21u);
            int rc = fmt == 0 ? fo_compress2(src, n, c, cap, &clen, &pbits)
                   : fmt == 1 ? fo_compress2_log(src, n, L, c, cap, &clen, &pbits)
                              : fo_compress(src, n, c, cap, &clen, &pbits);
            if (rc != 0) continue;
            if (clen > cap) { fprintf(stderr, "FAIL case %d: clen > cap\n", cs); return 1; }
            uint8_t* x = dup(c, clen);
            if (fmt < 2) {
                rc = fo_decompress2_n(x, clen, d, n);
                if (rc == 0 && L != 15 && fmt == 0 && memcmp(d, src, n) != 0) {
                    fprintf(stderr, "FAIL case %d: round trip\n", cs);
                    return 1;
                }
                (void)fo_decompress2(x, clen, d, n, &dlen);
            } else {
                (void)fo_decompress(x, clen, d, n, &dlen);
            }
            /* truncated and corrupted copies */
            for (int t = 0; t < 4; ++t) {
                const size_t m = t == 0 ? clen / 2 : clen;
                uint8_t* y = dup(c, m);
                if (t > 0 && m) y[rnd() % m] ^= (uint8_t)(1u + rnd() % 255u);
                if (fmt < 2) {
                    (void)fo_decompress2_n(y, m, d, n);
                    (void)fo_decompress2(y, m, d, n, &dlen);
                } else {
                    (void)fo_decompress(y, m, d, n, &dlen);
                }
                fo_norm h;
                size_t used = 0;
                (void)fo_header_read(y, m, &h, &used);
                free(y);
            }
            free(x);
        }
        free(src);
        free(c);
        free(d);
    }
    printf("ok %d cases\n", cases);
    return 0;
}
