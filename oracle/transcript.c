/*
 * oracle/transcript.c — Merlin v1.0 transcript over STROBE-128/Keccak-f[1600]
 * plus the ark-serialize encodings used by the prover.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Restates lib/PLONK/src/transcript/strobe.{h,cpp} (STROBE_R = 166,
 * "STROBEv1.0.2" init, meta_ad/ad/prf with begin_op framing),
 * transcript/transcript.cuh:21-73 (append_message = meta_ad(label) +
 * meta_ad(len u32 LE, more) + ad(msg); challenge_bytes likewise with prf),
 * serialize.cuh:32-84 (scalar = 32 B canonical LE; G1 = 48 B canonical x LE,
 * flags in the top byte: bit 6 infinity, bit 7 "y > -y"; public inputs =
 * BTreeMap {len u64, pos u64, value 32 B}) and flags.hpp:4-44.
 * challenge_scalar (transcript.cuh:66-72): 31 bytes LE, zero-extended,
 * converted to Montgomery.
 */
#include "oracle_internal.h"

#define STROBE_R 166
#define FLAG_I 1
#define FLAG_A 2
#define FLAG_C 4
#define FLAG_T 8
#define FLAG_M 16
#define FLAG_K 32

static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int RHO[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                            27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
static const int PI_[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                            15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};

static inline uint64_t rotl(uint64_t v, int n) { return (v << n) | (v >> (64 - n)); }

void or_keccak_f1600(uint64_t st[25]) {
    for (int round = 0; round < 24; round++) {
        uint64_t c[5];
        for (int x = 0; x < 5; x++) c[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
        for (int x = 0; x < 5; x++) {
            uint64_t d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
            for (int y = 0; y < 25; y += 5) st[y + x] ^= d;
        }
        uint64_t last = st[1];
        for (int i = 0; i < 24; i++) {
            uint64_t tmp = st[PI_[i]];
            st[PI_[i]] = rotl(last, RHO[i]);
            last = tmp;
        }
        for (int y = 0; y < 25; y += 5) {
            uint64_t a[5];
            for (int x = 0; x < 5; x++) a[x] = st[y + x];
            for (int x = 0; x < 5; x++) st[y + x] = a[x] ^ (~a[(x + 1) % 5] & a[(x + 2) % 5]);
        }
        st[0] ^= RC[round];
    }
}

struct or_transcript {
    uint8_t st[200];
    int pos, pos_begin, cur_flags;
};

static void run_f(or_transcript *t) {
    t->st[t->pos] ^= (uint8_t)t->pos_begin;
    t->st[t->pos + 1] ^= 0x04;
    t->st[STROBE_R + 1] ^= 0x80;
    uint64_t s[25];
    memcpy(s, t->st, 200);  /* little-endian host, as transmute_state */
    or_keccak_f1600(s);
    memcpy(t->st, s, 200);
    t->pos = 0;
    t->pos_begin = 0;
}
static void absorb(or_transcript *t, const uint8_t *d, size_t len) {
    for (size_t i = 0; i < len; i++) {
        t->st[t->pos] ^= d[i];
        t->pos++;
        if (t->pos == STROBE_R) run_f(t);
    }
}
static void squeeze(or_transcript *t, uint8_t *d, size_t len) {
    for (size_t i = 0; i < len; i++) {
        d[i] = t->st[t->pos];
        t->st[t->pos] = 0;
        t->pos++;
        if (t->pos == STROBE_R) run_f(t);
    }
}
static void begin_op(or_transcript *t, int flags, int more) {
    if (more) return;  /* flags unchanged by construction */
    int old_begin = t->pos_begin;
    t->pos_begin = t->pos + 1;
    t->cur_flags = flags;
    uint8_t d[2] = {(uint8_t)old_begin, (uint8_t)flags};
    absorb(t, d, 2);
    if ((flags & (FLAG_C | FLAG_K)) != 0 && t->pos != 0) run_f(t);
}
static void meta_ad(or_transcript *t, const uint8_t *d, size_t len, int more) {
    begin_op(t, FLAG_M | FLAG_A, more);
    absorb(t, d, len);
}
static void ad(or_transcript *t, const uint8_t *d, size_t len, int more) {
    begin_op(t, FLAG_A, more);
    absorb(t, d, len);
}
static void prf(or_transcript *t, uint8_t *d, size_t len, int more) {
    begin_op(t, FLAG_I | FLAG_A | FLAG_C, more);
    squeeze(t, d, len);
}

void or_transcript_append_message(or_transcript *t, const char *label,
                                  const uint8_t *msg, size_t len) {
    uint8_t l4[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    meta_ad(t, (const uint8_t *)label, strlen(label), 0);
    meta_ad(t, l4, 4, 1);
    ad(t, msg, len, 0);
}

or_transcript *or_transcript_new(const char *label) {
    or_transcript *t = (or_transcript *)calloc(1, sizeof(or_transcript));
    t->st[0] = 1;
    t->st[1] = STROBE_R + 2;
    t->st[2] = 1;
    t->st[3] = 0;
    t->st[4] = 1;
    t->st[5] = 96;
    memcpy(t->st + 6, "STROBEv1.0.2", 12);
    uint64_t s[25];
    memcpy(s, t->st, 200);
    or_keccak_f1600(s);
    memcpy(t->st, s, 200);
    const char *proto = "Merlin v1.0";
    meta_ad(t, (const uint8_t *)proto, strlen(proto), 0);
    or_transcript_append_message(t, "dom-sep", (const uint8_t *)label, strlen(label));
    return t;
}
void or_transcript_free(or_transcript *t) { free(t); }

void or_transcript_state(const or_transcript *t, uint8_t st[200], int meta[3]) {
    memcpy(st, t->st, 200);
    meta[0] = t->pos;
    meta[1] = t->pos_begin;
    meta[2] = t->cur_flags;
}

void or_transcript_challenge_bytes(or_transcript *t, const char *label, uint8_t *out, size_t len) {
    uint8_t l4[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    meta_ad(t, (const uint8_t *)label, strlen(label), 0);
    meta_ad(t, l4, 4, 1);
    prf(t, out, len, 0);
}

void or_transcript_challenge_scalar(or_transcript *t, const char *label, uint64_t out_mont[4]) {
    uint8_t buf[32] = {0};
    or_transcript_challenge_bytes(t, label, buf, 31);  /* MODULUS_BITS / 8 */
    uint64_t c[4];
    memcpy(c, buf, 32);
    or_fr_to_mont(out_mont, c);
}

void or_transcript_append_scalar(or_transcript *t, const char *label, const uint64_t s_mont[4]) {
    uint64_t c[4];
    or_fr_from_mont(c, s_mont);
    or_transcript_append_message(t, label, (const uint8_t *)c, 32);
}

void or_transcript_append_point(or_transcript *t, const char *label, const uint64_t aff[12]) {
    uint8_t buf[48];
    if (or_fq_is_zero(aff) && or_fq_eq(aff + 6, OR_FQ_ONE)) {
        memset(buf, 0, 48);
        buf[47] |= 1 << 6;  /* SWFlags::Infinity */
    } else {
        uint64_t x[6], y[6], ny[6], nyc[6];
        or_fq_from_mont(x, aff);
        or_fq_neg(ny, aff + 6);
        or_fq_from_mont(y, aff + 6);
        or_fq_from_mont(nyc, ny);
        memcpy(buf, x, 48);
        if (or_gt_n(y, nyc, 6)) buf[47] |= 1 << 7;  /* PositiveY */
    }
    or_transcript_append_message(t, label, buf, 48);
}

/* PublicInputs (pi.rs:16-22) serialised as its BTreeMap<usize, F>
 * (ark-serialize 0.3: u64 length, then (u64 key, 32-byte canonical value)
 * per entry in key order); zero values are never inserted (pi.rs:39-46). */
void or_transcript_append_pis(or_transcript *t, const char *label, uint64_t k,
                              const uint64_t *pos, const uint64_t *vals_canon) {
    uint64_t len = 0;
    for (uint64_t i = 0; i < k; i++) {
        uint64_t m[4];
        or_fr_to_mont(m, vals_canon + 4 * i);
        len += !or_fr_is_zero(m);
    }
    uint8_t *buf = (uint8_t *)malloc(8 + 40 * (len ? len : 1));
    memcpy(buf, &len, 8);
    size_t at = 8;
    for (uint64_t i = 0; i < k; i++) {
        uint64_t m[4], c[4];
        or_fr_to_mont(m, vals_canon + 4 * i);
        if (or_fr_is_zero(m)) continue;
        or_fr_from_mont(c, m);
        memcpy(buf + at, pos + i, 8);
        memcpy(buf + at + 8, c, 32);
        at += 40;
    }
    or_transcript_append_message(t, label, buf, at);
    free(buf);
}

void or_transcript_append_pi(or_transcript *t, const char *label,
                             const uint64_t pi_canon[4], uint64_t pos) {
    uint8_t buf[48];
    uint64_t len = 1;
    uint64_t m[4], c[4];
    /* append_pi: to_mont(item) then serialize (to_base): canonical round-trip */
    or_fr_to_mont(m, pi_canon);
    or_fr_from_mont(c, m);
    memcpy(buf, &len, 8);
    memcpy(buf + 8, &pos, 8);
    memcpy(buf + 16, c, 32);
    or_transcript_append_message(t, label, buf, 48);
}
