// Host-side field arithmetic of csrc/field.cuh (the prover's challenge
// arithmetic and the commitments' affine conversion run on the host): prints
// seeded operands with their Montgomery product and inverse, one line each,
// for tests/test_host_field.py to check with Python integers.
//   host_field <count>   ->  "r|q a b a*b inv(a)" (hex limbs, Montgomery form),
//                            then "b a fr_inverse_bin(a)" (the device's batch-
//                            inverse base case, same source on the host)
#include "field.cuh"
#include <cstdio>
#include <cstdlib>

using namespace pnp;

static uint64_t sm = 0x9e3779b97f4a7c15ull;
static uint64_t next() {  // splitmix64
    uint64_t z = (sm += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
template <class P>
static Fp<P> draw(int k) {
    Fp<P> r = Fp<P>::zero();
    if (k == 0) return r;                                   // zero
    if (k == 1) return Fp<P>::one();                        // one (Montgomery)
    if (k == 2) return Fp<P>::zero() - Fp<P>::one();        // -1
    if (k == 3) { r.v[0] = 1; return r; }                   // the raw integer 1
    if (k == 4) return Fp<P>::modulus() - Fp<P>::one() - Fp<P>::one();  // below P, not reduced by '-'
    for (int i = 0; i < P::N; i++) r.v[i] = (uint32_t)next();
    if (k % 2) r.v[P::N - 1] &= 0x7fffffffu;  // up to ~2^255 / 2^383: reduce
    while (!gt(Fp<P>::modulus(), r)) reduce_once(r);
    return r;
}
template <class P>
static void hex(const Fp<P> &a) {
    printf(" ");
    for (int i = P::N - 1; i >= 0; i--) printf("%08x", a.v[i]);
}
template <class P>
static void run(const char *name, int count) {
    for (int k = 0; k < count; k++) {
        const Fp<P> a = draw<P>(k), b = draw<P>(k + 7);
        printf("%s", name);
        hex(a), hex(b), hex(a * b), hex(inverse(a));
        printf("\n");
    }
}
int main(int argc, char **argv) {
    const int count = argc > 1 ? atoi(argv[1]) : 200;
    run<FrP>("r", count);
    run<FqP>("q", count);
    for (int k = 0; k < count; k++) {
        const Fr a = draw<FrP>(k);
        printf("b");
        hex(a), hex(fr_inverse_bin(a));
        printf("\n");
    }
    return 0;
}
