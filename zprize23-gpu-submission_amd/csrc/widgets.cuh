// widgets.cuh — the custom-gate constraint polynomials of the reference
// prover (plonk-core/src/proof_system/widget: GateConstraint::constraints),
// host + device: the quotient evaluates selector(x) * constraints(values at x)
// per coset point (k_widgets_, protocol.hip), the linearisation scales the
// selector polynomial by constraints(evaluations at z) on the host
// (widget/mod.rs:83-104).
#pragma once
#include "field.cuh"

namespace pnp {

struct WidgetVals {
    Fr a, b, c, d;              // wire values
    Fr a_next, b_next, d_next;  // wire values of the next row (w x)
    Fr q_l, q_r, q_c;           // selector values
};

// Jubjub (ark-ed-on-bls12-381): a = -1, d = -10240/10241, Montgomery
PNP_HD Fr jj_coeff_a() {
    Fr r;
    const uint32_t v[8] = {0x3u, 0xfffffffdu, 0xfffb13fcu, 0xfb38ec08u,
                           0x1ce5880fu, 0x99ad8818u, 0x7cd877d8u, 0x5bc8f5f9u};
    for (int i = 0; i < 8; i++) r.v[i] = v[i];
    return r;
}
PNP_HD Fr jj_coeff_d() {
    Fr r;
    const uint32_t v[8] = {0xb974f6b0u, 0x2a522455u, 0x0d9acab3u, 0xfc6cc9efu,
                           0xc27628d1u, 0x7a08fb94u, 0xfe0e262eu, 0x57f8f6a8u};
    for (int i = 0; i < 8; i++) r.v[i] = v[i];
    return r;
}

PNP_HD Fr mul4(const Fr &x) { return dbl(dbl(x)); }

// delta(f) = f (f - 1)(f - 2)(f - 3)  (range.rs:66-74, logic.rs:84-93)
PNP_HD Fr gate_delta(const Fr &f) {
    const Fr one = Fr::one();
    const Fr f1 = f - one, f2 = f1 - one, f3 = f2 - one;
    return f * f1 * f2 * f3;
}

// Range::constraints (widget/range.rs:44-60)
PNP_HD Fr w_range(const Fr &sep, const WidgetVals &w) {
    const Fr kappa = sep * sep, kappa2 = kappa * kappa, kappa3 = kappa2 * kappa;
    Fr acc = gate_delta(w.c - mul4(w.d));
    acc += gate_delta(w.b - mul4(w.c)) * kappa;
    acc += gate_delta(w.a - mul4(w.b)) * kappa2;
    acc += gate_delta(w.d_next - mul4(w.a)) * kappa3;
    return acc * sep;
}

// delta_xor_and (widget/logic.rs:104-133), small constants by additions
PNP_HD Fr delta_xor_and(const Fr &a, const Fr &b, const Fr &w, const Fr &c, const Fr &q_c) {
    const Fr one = Fr::one();
    const Fr two = dbl(one), three = two + one, four = dbl(two), nine = dbl(four) + one;
    const Fr eighteen = dbl(nine), eighty_one = mul4(eighteen) + nine, eighty_three = eighty_one + two;
    const Fr apb = a + b;
    Fr F = w * (w * (four * w - eighteen * apb + eighty_one) + eighteen * (a * a + b * b) -
                eighty_one * apb + eighty_three);
    Fr E = three * (apb + c) - dbl(F);
    Fr B = q_c * (nine * c - three * apb);
    return B + E;
}

// Logic::constraints (widget/logic.rs:59-82)
PNP_HD Fr w_logic(const Fr &sep, const WidgetVals &w) {
    const Fr kappa = sep * sep, kappa2 = kappa * kappa, kappa3 = kappa2 * kappa, kappa4 = kappa3 * kappa;
    const Fr a = w.a_next - mul4(w.a), b = w.b_next - mul4(w.b), d = w.d_next - mul4(w.d);
    Fr acc = gate_delta(a);
    acc += gate_delta(b) * kappa;
    acc += gate_delta(d) * kappa2;
    acc += (w.c - a * b) * kappa3;
    acc += delta_xor_and(a, b, w.c, d, w.q_c) * kappa4;
    return acc * sep;
}

// FixedBaseScalarMul::constraints (widget/ecc/fixed_base_scalar_mul.rs:89-155)
PNP_HD Fr w_fbsm(const Fr &sep, const WidgetVals &w) {
    const Fr one = Fr::one();
    const Fr kappa = sep * sep, kappa2 = kappa * kappa, kappa3 = kappa2 * kappa;
    const Fr bit = w.d_next - dbl(w.d);                   // extract_bit
    const Fr bit_c = bit * (bit - one) * (bit + one);     // check_bit_consistency
    const Fr y_alpha = bit * bit * (w.q_r - one) + one;   // y_beta = q_r
    const Fr x_alpha = w.q_l * bit;                       // x_beta = q_l
    const Fr xy_c = (bit * w.q_c - w.c) * kappa;          // xy_alpha = c
    const Fr m = w.c * w.a * w.b * jj_coeff_d();          // xy_alpha acc_x acc_y D
    const Fr x_c = (w.a_next + w.a_next * m - (x_alpha * w.b + y_alpha * w.a)) * kappa2;
    const Fr y_c = (w.b_next - w.b_next * m - (y_alpha * w.b - jj_coeff_a() * x_alpha * w.a)) * kappa3;
    return (bit_c + x_c + y_c + xy_c) * sep;
}

// CurveAddition::constraints (widget/ecc/curve_addition.rs:61-96)
PNP_HD Fr w_cadd(const Fr &sep, const WidgetVals &w) {
    const Fr &x1 = w.a, &y1 = w.b, &x2 = w.c, &y2 = w.d, &x3 = w.a_next, &y3 = w.b_next,
             &x1y2 = w.d_next;
    const Fr kappa = sep * sep;
    const Fr xy_c = x1 * y2 - x1y2;
    const Fr y1x2 = y1 * x2, y1y2 = y1 * y2, x1x2 = x1 * x2;
    const Fr dm = jj_coeff_d() * x1y2 * y1x2;
    const Fr x3_c = (x1y2 + y1x2 - (x3 + x3 * dm)) * kappa;
    const Fr y3_c = (y1y2 - jj_coeff_a() * x1x2 - (y3 - y3 * dm)) * (kappa * kappa);
    return (xy_c + x3_c + y3_c) * sep;
}

}  // namespace pnp
