/* cpu_fast.c -- "optimised CPU" baselines for bench.py (report one beside the
 * Java-faithful port so GPU speedups are honest).  Test / baseline infrastructure only: never
 * linked into libjrq.so, never called by the product path.
 *
 *  jo_fast_crc64_batch   CRC-64/ECMA-182 as CRC64.update (jraft-core/.../util/CRC64.java:100-110)
 *                        but slice-by-8: 8 bytes per step, T_j[i] = i * x^(8j+64) mod P.
 *  jo_fast_quorum_epoch  the closed form of one BallotBox.commitAt epoch per group
 *                        (JC/core/BallotBox.java:96-139): q-th largest
 *                        match over each conf mask, no per-entry Ballot objects.  One conf per
 *                        group (no run table), as in the C3 workload.
 * Both are checked against the oracle (jraft_oracle.c) in tests/test_oracle_golden.py. */
#include <stdint.h>
#include <string.h>

#include "jraft_oracle.h"

static uint64_t T8[8][256];
static int t8_ready;

static void t8_init(void) {
    const uint64_t *t = jo_crc64_table();
    for (int i = 0; i < 256; ++i) T8[0][i] = t[i];
    for (int j = 1; j < 8; ++j)
        for (int i = 0; i < 256; ++i) {
            const uint64_t v = T8[j - 1][i];
            T8[j][i] = t[v >> 56] ^ (v << 8);
        }
    t8_ready = 1;
}

/* Build both the oracle's table and the slice tables when the library loads, before any
 * baseline thread runs (their lazy initialisation is otherwise a benign but real race). */
__attribute__((constructor)) static void tables_at_load(void) {
    (void)jo_crc64_table();
    t8_init();
}

uint64_t jo_fast_crc64_update(uint64_t crc, const uint8_t *p, size_t n) {
    if (!t8_ready) t8_init();
    const uint64_t *t = T8[0];
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        const uint64_t v = crc ^ __builtin_bswap64(w);  /* bytes in stream order, MSB first */
        crc = T8[7][v >> 56] ^ T8[6][(v >> 48) & 0xFF] ^ T8[5][(v >> 40) & 0xFF] ^
              T8[4][(v >> 32) & 0xFF] ^ T8[3][(v >> 24) & 0xFF] ^ T8[2][(v >> 16) & 0xFF] ^
              T8[1][(v >> 8) & 0xFF] ^ T8[0][v & 0xFF];
        p += 8;
        n -= 8;
    }
    while (n--) crc = t[((crc >> 56) ^ *p++) & 0xFF] ^ (crc << 8);
    return crc;
}

void jo_fast_crc64_batch(const uint8_t *payload, const uint64_t *offsets, uint32_t n, uint64_t *out) {
    for (uint32_t i = 0; i < n; ++i)
        out[i] = jo_fast_crc64_update(0, payload + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}

/* q-th largest of match[p] over the slots in mask; INT64_MIN when fewer than q members or
 * q == 0 with a non-empty requirement (never granted). */
static int64_t kth_largest(const int64_t *m, uint32_t P, uint32_t mask, uint32_t q) {
    int64_t best = INT64_MIN;
    for (uint32_t a = 0; a < P; ++a) {
        if (!((mask >> a) & 1u)) continue;
        uint32_t ge = 0;
        for (uint32_t b = 0; b < P; ++b) ge += ((mask >> b) & 1u) && m[b] >= m[a];
        if (ge >= q && m[a] > best) best = m[a];
    }
    return best;
}

void jo_fast_quorum_epoch(uint32_t P, uint32_t G, uint64_t ld, const int64_t *match,
                          const int64_t *pending, const int64_t *last_appended,
                          const int64_t *last_committed, const uint64_t *conf,
                          int64_t *committed, uint8_t *status) {
    int64_t m[16];
    for (uint32_t g = 0; g < G; ++g) {
        const int64_t pi = pending[g], la = last_appended[g], lc = last_committed[g];
        uint8_t st = 0;
        int64_t c = lc;
        for (uint32_t p = 0; p < P; ++p) {
            m[p] = match[(uint64_t)p * ld + g];
            if (m[p] > la) st |= 2; /* OUT_OF_RANGE */
        }
        if (pi == 0) {
            st |= 1; /* NOT_LEADER: commitAt returns false, nothing changes */
        } else if (!(st & 2)) {
            const uint64_t w = conf[g];
            const uint32_t nm = (uint32_t)(w & 0xFFFF), om = (uint32_t)((w >> 16) & 0xFFFF);
            const uint32_t nq = (uint32_t)((w >> 32) & 0xFF), oq = (uint32_t)((w >> 40) & 0xFF);
            if (nm == 0 || (oq && om == 0)) st |= 4; /* EMPTY_CONF */
            int64_t cand = kth_largest(m, P, nm, nq);
            if (oq) {
                const int64_t ko = kth_largest(m, P, om, oq);
                if (ko < cand) cand = ko;
            }
            if (la < cand) cand = la;
            if (cand >= pi && cand > c) c = cand;
        }
        committed[g] = c;
        status[g] = st;
    }
}
