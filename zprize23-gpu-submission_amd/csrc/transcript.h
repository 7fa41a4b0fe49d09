// transcript.h — Merlin v1.0 transcript (STROBE-128 over Keccak-f[1600]) with
// the ark-serialize encodings of the reference prover.
//   lib/PLONK/src/transcript/transcript.cuh:21-73  append_message / challenge_*
//   lib/PLONK/src/transcript/strobe.{h,cpp}          STROBE-128, R = 166
//   lib/PLONK/src/serialize.cuh:32-84, flags.hpp     scalar / G1 / BTreeMap bytes
#pragma once
#include <stdint.h>
#include <string>
#include "field.cuh"

namespace pnp {

class Transcript {
   public:
    explicit Transcript(const char *label);
    void append_message(const char *label, const uint8_t *msg, size_t len);
    void append_scalar(const char *label, const Fr &mont);
    // affine Montgomery point; (0, one) is the point at infinity
    void append_point(const char *label, const uint64_t x[6], const uint64_t y[6]);
    void append_pi(const char *label, const uint64_t pi_canon[4], uint64_t pos);
    // PublicInputs (pi.rs:16-22) as its BTreeMap<usize, F>: u64 length, then
    // (u64 position, 32-byte canonical value) per entry; positions strictly
    // increasing, zero values already dropped (pi.rs:33-46)
    void append_pis(const char *label, uint64_t k, const uint64_t *pos, const uint64_t *vals_canon);
    void challenge_bytes(const char *label, uint8_t *out, size_t len);
    Fr challenge_scalar(const char *label);

   private:
    uint8_t st_[200];
    int pos_ = 0, pos_begin_ = 0, cur_flags_ = 0;
    void run_f();
    void absorb(const uint8_t *d, size_t n);
    void squeeze(uint8_t *d, size_t n);
    void begin_op(int flags, bool more);
    void meta_ad(const uint8_t *d, size_t n, bool more);
};

}  // namespace pnp
