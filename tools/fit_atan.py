"""Fit of atan_unit (csrc/sunsky_kernels.hip, FAST kernels' atan2): atan(t) = t + t^3 P(t^2)
on t in [0, 1], iteratively reweighted least squares on Chebyshev nodes towards
equal-ripple relative error; prints the fp32 coefficients and the max error of the
fp32 Horner/FMA evaluation in ulp over 4M points, and of the assembled atan2
(t = min/max with a 1-ulp reciprocal, octant fix-ups) against fp64 atan2."""
import sys

import numpy as np

DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 8


def target(t):
    out = np.empty_like(t)
    small = t < 1e-8
    x = np.sqrt(t[~small])
    out[~small] = (np.arctan(x) - x) / (t[~small] * x)
    out[small] = -1 / 3 + t[small] / 5
    return out


def horner(cs, ts):
    p = np.full(ts.shape, cs[-1], dtype=np.float32)
    for a in cs[-2::-1]:
        p = (p.astype(np.float64) * ts + np.float64(a)).astype(np.float32)
    return p


def atan_unit(cs, xs):
    ts = (xs * xs).astype(np.float32)
    p = horner(cs, ts)
    return ((xs * ts).astype(np.float32).astype(np.float64) * p + xs).astype(np.float32)


def main():
    n = 600
    u = np.cos(np.pi * (np.arange(n) + 0.5) / n)
    t = (u + 1) / 2
    x = np.sqrt(t)
    w = np.maximum(x * t / np.maximum(np.arctan(x), 1e-30), 1e-3)
    c = np.polynomial.polynomial.polyfit(t, target(t), DEG, w=w)
    for _ in range(40):
        e = np.abs((np.polynomial.polynomial.polyval(t, c) - target(t)) * w)
        c = np.polynomial.polynomial.polyfit(t, target(t), DEG, w=w * (1 + e / e.max()) ** 4)
    cs = c.astype(np.float32)
    xs = np.linspace(0, 1, 4000001).astype(np.float32)
    r = atan_unit(cs, xs)
    ref = np.arctan(xs.astype(np.float64))
    ulp = np.abs(r - ref) / np.spacing(np.maximum(ref, 1e-30).astype(np.float32)).astype(np.float64)
    print("coefficients (t^0 .. t^%d):" % DEG, [float(v) for v in cs])
    print("atan on [0, 1] max error: %.3f ulp" % ulp.max())
    # assembled atan2 over random directions, reciprocal perturbed by +-1 ulp
    rng = np.random.default_rng(0)
    y = rng.standard_normal(2_000_000).astype(np.float32)
    xx = rng.standard_normal(2_000_000).astype(np.float32)
    ax, ay = np.abs(xx), np.abs(y)
    mx, mn = np.maximum(ax, ay), np.minimum(ax, ay)
    rc = (1.0 / mx.astype(np.float64)).astype(np.float32)
    rc = np.where(rng.random(rc.size) < 0.5, np.nextafter(rc, np.float32(0)), np.nextafter(rc, np.float32(9)))
    tt = (mn * rc).astype(np.float32)
    tt = np.minimum(tt, np.float32(1))
    a = atan_unit(cs, tt)
    a = np.where(ay > ax, (np.float32(np.pi / 2) - a).astype(np.float32), a)
    a = np.where(xx < 0, (np.float32(np.pi) - a).astype(np.float32), a)
    a = np.copysign(a, y)
    ref = np.arctan2(y.astype(np.float64), xx.astype(np.float64))
    ulp = np.abs(a - ref) / np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    print("atan2 max error: %.3f ulp, abs %.3e" % (ulp.max(), np.abs(a - ref).max()))


if __name__ == "__main__":
    main()
