// transcript.cpp — see transcript.h for the reference mapping.
#include "transcript.h"
#include <vector>
#include <string.h>

namespace pnp {

namespace {
constexpr int kRate = 166;  // STROBE_R (strobe.h)
constexpr int kFlagI = 1, kFlagA = 2, kFlagC = 4, kFlagM = 16, kFlagK = 32;

constexpr uint64_t kRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

inline uint64_t rol(uint64_t v, int s) { return (v << s) | (v >> (64 - s)); }

// Keccak-f[1600] in lane form (rho offsets / pi lane order of the FIPS-202 spec)
void keccak_f(uint64_t a[25]) {
    static const int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int r = 0; r < 24; r++) {
        uint64_t c[5], b[25];
        for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++) {
            uint64_t d = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
            for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
        }
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                int s = rho[x + 5 * y];
                uint64_t v = a[x + 5 * y];
                b[y + 5 * ((2 * x + 3 * y) % 5)] = s ? rol(v, s) : v;
            }
        for (int y = 0; y < 5; y++)
            for (int x = 0; x < 5; x++)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= kRC[r];
    }
}
}  // namespace

Transcript::Transcript(const char *label) {
    memset(st_, 0, sizeof st_);
    const uint8_t init[6] = {1, kRate + 2, 1, 0, 1, 96};
    memcpy(st_, init, 6);
    memcpy(st_ + 6, "STROBEv1.0.2", 12);
    uint64_t lanes[25];
    memcpy(lanes, st_, 200);
    keccak_f(lanes);
    memcpy(st_, lanes, 200);
    const char *proto = "Merlin v1.0";
    meta_ad(reinterpret_cast<const uint8_t *>(proto), strlen(proto), false);
    append_message("dom-sep", reinterpret_cast<const uint8_t *>(label), strlen(label));
}

void Transcript::run_f() {
    st_[pos_] ^= (uint8_t)pos_begin_;
    st_[pos_ + 1] ^= 0x04;
    st_[kRate + 1] ^= 0x80;
    uint64_t lanes[25];
    memcpy(lanes, st_, 200);
    keccak_f(lanes);
    memcpy(st_, lanes, 200);
    pos_ = 0;
    pos_begin_ = 0;
}
void Transcript::absorb(const uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) {
        st_[pos_++] ^= d[i];
        if (pos_ == kRate) run_f();
    }
}
void Transcript::squeeze(uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) {
        d[i] = st_[pos_];
        st_[pos_++] = 0;
        if (pos_ == kRate) run_f();
    }
}
void Transcript::begin_op(int flags, bool more) {
    if (more) return;
    uint8_t hdr[2] = {(uint8_t)pos_begin_, (uint8_t)flags};
    pos_begin_ = pos_ + 1;
    cur_flags_ = flags;
    absorb(hdr, 2);
    if ((flags & (kFlagC | kFlagK)) && pos_ != 0) run_f();
}
void Transcript::meta_ad(const uint8_t *d, size_t n, bool more) {
    begin_op(kFlagM | kFlagA, more);
    absorb(d, n);
}

void Transcript::append_message(const char *label, const uint8_t *msg, size_t len) {
    const uint8_t l4[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    meta_ad(reinterpret_cast<const uint8_t *>(label), strlen(label), false);
    meta_ad(l4, 4, true);
    begin_op(kFlagA, false);
    absorb(msg, len);
}

void Transcript::challenge_bytes(const char *label, uint8_t *out, size_t len) {
    const uint8_t l4[4] = {(uint8_t)len, (uint8_t)(len >> 8), (uint8_t)(len >> 16), (uint8_t)(len >> 24)};
    meta_ad(reinterpret_cast<const uint8_t *>(label), strlen(label), false);
    meta_ad(l4, 4, true);
    begin_op(kFlagI | kFlagA | kFlagC, false);
    squeeze(out, len);
}

Fr Transcript::challenge_scalar(const char *label) {
    uint8_t b[32] = {0};
    challenge_bytes(label, b, 31);  // fr::MODULUS_BITS / 8
    uint64_t l[4];
    memcpy(l, b, 32);
    return to_mont(from_u64_limbs<FrP>(l));
}

void Transcript::append_scalar(const char *label, const Fr &mont) {
    uint64_t c[4];
    to_u64_limbs(from_mont(mont), c);
    append_message(label, reinterpret_cast<const uint8_t *>(c), 32);
}

void Transcript::append_point(const char *label, const uint64_t x[6], const uint64_t y[6]) {
    uint8_t b[48];
    Fq fx = from_u64_limbs<FqP>(x), fy = from_u64_limbs<FqP>(y);
    if (fx.is_zero() && fy == Fq::one()) {
        memset(b, 0, 48);
        b[47] |= 1 << 6;  // SWFlags::Infinity
    } else {
        uint64_t xc[6];
        to_u64_limbs(from_mont(fx), xc);
        memcpy(b, xc, 48);
        if (gt(from_mont(fy), from_mont(neg(fy)))) b[47] |= 1 << 7;  // PositiveY
    }
    append_message(label, b, 48);
}

void Transcript::append_pi(const char *label, const uint64_t pi_canon[4], uint64_t pos) {
    uint8_t b[48];
    uint64_t one = 1, c[4];
    to_u64_limbs(from_mont(to_mont(from_u64_limbs<FrP>(pi_canon))), c);
    memcpy(b, &one, 8);
    memcpy(b + 8, &pos, 8);
    memcpy(b + 16, c, 32);
    append_message(label, b, 48);
}

void Transcript::append_pis(const char *label, uint64_t k, const uint64_t *pos, const uint64_t *vals_canon) {
    std::vector<uint8_t> b(8 + 40 * k);
    memcpy(b.data(), &k, 8);
    for (uint64_t i = 0; i < k; i++) {
        uint64_t c[4];
        to_u64_limbs(from_mont(to_mont(from_u64_limbs<FrP>(vals_canon + 4 * i))), c);
        memcpy(b.data() + 8 + 40 * i, pos + i, 8);
        memcpy(b.data() + 16 + 40 * i, c, 32);
    }
    append_message(label, b.data(), b.size());
}

}  // namespace pnp
