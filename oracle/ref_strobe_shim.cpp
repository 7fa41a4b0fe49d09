// oracle/ref_strobe_shim.cpp — TEST INFRASTRUCTURE ONLY.
// Drives the reference's own Strobe128 (lib/PLONK/src/transcript/strobe.cpp,
// compiled in place by ref.mk) with the Merlin framing of
// lib/PLONK/src/transcript/transcript.cuh:21-64, so golden transcript
// fixtures come from the reference's STROBE/Keccak implementation.
#include "strobe.h"
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {
std::vector<uint8_t> u32le(size_t x) {
    return {uint8_t(x), uint8_t(x >> 8), uint8_t(x >> 16), uint8_t(x >> 24)};
}
}  // namespace

extern "C" {

void *refm_new(const char *label) {
    Strobe128 *s = new Strobe128(Strobe128::new_instance("Merlin v1.0"));
    std::vector<uint8_t> l = str_to_u8("dom-sep");
    std::vector<uint8_t> len = u32le(strlen(label));
    std::vector<uint8_t> msg(label, label + strlen(label));
    s->meta_ad(l, false);
    s->meta_ad(len, true);
    s->ad(msg, false);
    return s;
}

void refm_free(void *h) { delete static_cast<Strobe128 *>(h); }

void refm_append(void *h, const char *label, const uint8_t *msg, size_t n) {
    Strobe128 *s = static_cast<Strobe128 *>(h);
    std::vector<uint8_t> l = str_to_u8(label);
    std::vector<uint8_t> len = u32le(n);
    std::vector<uint8_t> m(msg, msg + n);
    s->meta_ad(l, false);
    s->meta_ad(len, true);
    s->ad(m, false);
}

void refm_challenge(void *h, const char *label, uint8_t *out, size_t n) {
    Strobe128 *s = static_cast<Strobe128 *>(h);
    std::vector<uint8_t> l = str_to_u8(label);
    std::vector<uint8_t> len = u32le(n);
    std::vector<uint8_t> d(n, 0);
    s->meta_ad(l, false);
    s->meta_ad(len, true);
    s->prf(d, false);
    memcpy(out, d.data(), n);
}

void refm_keccak(uint64_t st[25]) { keccak_p(st, 24); }

}  // extern "C"
