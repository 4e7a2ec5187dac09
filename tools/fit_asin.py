"""Fit of asin_half_chord (csrc/sunsky_kernels.hip): asin(x) = x + x^3 P(x^2) on
x in [0, sqrt(0.5005)], degree 7 in t = x^2, iteratively reweighted least squares on
Chebyshev nodes towards equal-ripple relative error; prints the fp32 coefficients and
the max error of the fp32 Horner/FMA evaluation in ulp over 4M points."""
import numpy as np

TMAX, DEG = 0.5005, 7


def target(t):
    x = np.sqrt(t)
    out = np.empty_like(t)
    small = t < 1e-8
    out[~small] = (np.arcsin(x[~small]) - x[~small]) / (t[~small] * x[~small])
    out[small] = 1 / 6 + 3 / 40 * t[small]
    return out


def main():
    n = 400
    u = np.cos(np.pi * (np.arange(n) + 0.5) / n)
    t = (u + 1) / 2 * TMAX
    x = np.sqrt(t)
    w = np.maximum(x * t / np.maximum(np.arcsin(x), 1e-30), 1e-3)
    c = np.polynomial.polynomial.polyfit(t, target(t), DEG, w=w)
    for _ in range(30):
        e = np.abs((np.polynomial.polynomial.polyval(t, c) - target(t)) * w)
        c = np.polynomial.polynomial.polyfit(t, target(t), DEG, w=w * (1 + e / e.max()) ** 4)
    cs = c.astype(np.float32)
    xs = np.linspace(0, np.sqrt(TMAX), 4000001).astype(np.float32)
    ts = (xs * xs).astype(np.float32)
    p = np.full(ts.shape, cs[-1], dtype=np.float32)
    for a in cs[-2::-1]:
        p = (p.astype(np.float64) * ts + np.float64(a)).astype(np.float32)       # one rounding per fma
    r = ((xs * ts).astype(np.float32).astype(np.float64) * p + xs).astype(np.float32)
    ref = np.arcsin(xs.astype(np.float64))
    ulp = np.abs(r - ref) / np.spacing(ref.astype(np.float32)).astype(np.float64)
    print("coefficients (t^0 .. t^7):", [float(v) for v in cs])
    print("max error: %.3f ulp" % ulp.max())


if __name__ == "__main__":
    main()
