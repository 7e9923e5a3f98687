"""Fit of K10's GELU (cm_gemm.hip gelu_erf): h(u) = erfc(u) / 2 = 2^P(u), u = |x| / sqrt 2 in [0, 3.92],
P of degree 9 by least squares on Chebyshev nodes; GELU(x) = x (1 - h) for x >= 0, x h below.
Evaluates the fp32 form (fma Horner, exp2) against an fp64 GELU on a grid over [-7, 7] beside
torch's formula 0.5 x (1 + erff(x / sqrt 2)) with a correctly rounded erff, and prints the fp32
coefficients (CPU only: python tools/gelu_fit.py)."""
import math

import numpy as np

U = 3.92


def fit(deg):
    u = (np.cos(np.linspace(0, np.pi, 8000)) + 1) / 2 * U
    y = np.array([math.log2(0.5 * math.erfc(v)) for v in u])
    c, *_ = np.linalg.lstsq(np.vander(u, deg + 1, increasing=True), y, rcond=None)
    return [np.float32(a) for a in c]


def horner32(c, x):
    r = np.full_like(x, c[-1], dtype=np.float32)
    for a in c[-2::-1]:
        r = (r.astype(np.float64) * x.astype(np.float64) + np.float64(a)).astype(np.float32)   # fma
    return r


def main():
    x = np.linspace(-7, 7, 700001).astype(np.float32)
    g64 = np.array([0.5 * float(v) * (1 + math.erf(float(v) / math.sqrt(2))) for v in x])
    u32 = (x * np.float32(0.70710678118654752)).astype(np.float32)
    e_ref = np.array([math.erf(float(v)) for v in u32]).astype(np.float32)
    g_torch = (np.float32(0.5) * x * (np.float32(1) + e_ref).astype(np.float32)).astype(np.float32)
    m = (np.abs(x) < 5.5) & (np.abs(x) > 1e-3)

    def report(name, g):
        ea = np.abs(g.astype(np.float64) - g64)
        print(f"{name}: max abs {ea.max():.3e}, max rel (|x| < 5.5) {(ea / np.abs(g64))[m].max():.3e}")

    report("0.5 x (1 + erff)", g_torch)
    for deg in (7, 8, 9):
        c = fit(deg)
        u = np.abs(u32)
        h = np.exp2(horner32(c, np.minimum(u, np.float32(U))).astype(np.float64)).astype(np.float32)
        h = np.where(u >= np.float32(U), np.float32(0), h)
        g = np.where(x >= 0, x * (np.float32(1) - h).astype(np.float32), x * h).astype(np.float32)
        report(f"degree {deg}", g)
        if deg == 9:
            print("coefficients c0..c9:", [float(a) for a in c])


if __name__ == "__main__":
    main()
