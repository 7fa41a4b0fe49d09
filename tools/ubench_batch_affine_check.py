"""Check the batch-affine microbenchmark's arithmetic (tools/ubench_batch_affine.hip):
for the pairs it dumped, the outputs are the affine sum's formulas mod q in
the radix-2^29 Montgomery form (R = 2^406):
    lambda = (y2 - y1) / (x2 - x1), x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1
    python tools/ubench_batch_affine_check.py pairs.json"""
import json
import sys

Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = pow(2, 406, Q)
RI = pow(R, -1, Q)


def val(limbs):
    return sum(int(v) << (29 * i) for i, v in enumerate(limbs))


def main():
    pairs = json.load(open(sys.argv[1]))
    ok = True
    for k, p in enumerate(pairs):
        x1, y1, x2, y2 = (val(p[c]) * RI % Q for c in ("x1", "y1", "x2", "y2"))
        lam = (y2 - y1) * pow(x2 - x1, -1, Q) % Q
        x3 = (lam * lam - x1 - x2) % Q
        y3 = (lam * (x1 - x3) - y1) % Q
        gx, gy = val(p["x3"]) * RI % Q, val(p["y3"]) * RI % Q
        good = gx == x3 and gy == y3
        ok &= good
        print(f"pair {k}: {'ok' if good else 'MISMATCH'}")
    print("all pairs match" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
