"""Fit of sincos_fast (csrc/sunsky_kernels.hip, FAST sampling kernels): on r in
[-pi/4, pi/4], sin r = r + r^3 S(r^2) and cos r = 1 - r^2/2 + r^4 C(r^2), degree 3 in r^2,
iteratively reweighted least squares towards equal-ripple error (relative for sin,
absolute for cos); prints the fp32 coefficients and the error of the fp32 evaluation
with the two-constant Cody-Waite reduction by pi/2 over x in [-8 pi, 8 pi]."""
import numpy as np

R = np.pi / 4


def fit(target, deg, weight):
    n = 500
    t = (np.cos(np.pi * (np.arange(n) + 0.5) / n) + 1) / 2 * R * R
    w = weight(t)
    c = np.polynomial.polynomial.polyfit(t, target(t), deg, w=w)
    for _ in range(40):
        e = np.abs((np.polynomial.polynomial.polyval(t, c) - target(t)) * w)
        c = np.polynomial.polynomial.polyfit(t, target(t), deg, w=w * (1 + e / e.max()) ** 4)
    return c.astype(np.float32)


def f32fma(a, b, c):
    return (a.astype(np.float64) * b + c).astype(np.float32)


def horner(cs, t):
    p = np.full(t.shape, cs[-1], dtype=np.float32)
    for a in cs[-2::-1]:
        p = f32fma(p, t, np.float32(a))
    return p


def sincos(S, C, x):
    x = x.astype(np.float32)
    k = np.rint((x * np.float32(2 / np.pi)).astype(np.float32)).astype(np.float32)
    c1 = np.float32(np.pi / 2)
    c2 = np.float32(np.pi / 2 - np.float64(c1))
    r = f32fma(-k, c1, x)
    r = f32fma(-k, c2, r)
    r2 = (r * r).astype(np.float32)
    sn = f32fma((r * r2).astype(np.float32), horner(S, r2), r)
    cs = f32fma((r2 * r2).astype(np.float32), horner(C, r2), f32fma(np.float32(-0.5), r2, np.float32(1)))
    q = k.astype(np.int64)
    sv = np.where(q & 1, cs, sn)
    cv = np.where(q & 1, sn, cs)
    sv = np.where(q & 2, -sv, sv)
    cv = np.where((q + 1) & 2, -cv, cv)
    return sv, cv


def main():
    def ts(t):
        r = np.sqrt(t)
        out = np.full_like(t, -1 / 6)
        m = t > 1e-6
        out[m] = (np.sin(r[m]) - r[m]) / (t[m] * r[m])
        return out

    def tc(t):
        r = np.sqrt(t)
        out = np.full_like(t, 1 / 24)
        m = t > 1e-6
        out[m] = (np.cos(r[m]) - 1 + t[m] / 2) / (t[m] * t[m])
        return out

    S = fit(ts, 3, lambda t: np.sqrt(t) * t / np.maximum(np.sin(np.sqrt(t)), 1e-30))
    C = fit(tc, 3, lambda t: t * t)
    print("S:", [float(v) for v in S])
    print("C:", [float(v) for v in C])
    x = np.linspace(-8 * np.pi, 8 * np.pi, 8000001).astype(np.float32)
    s, c = sincos(S, C, x)
    xs = x.astype(np.float64)
    es, ec = np.abs(s - np.sin(xs)), np.abs(c - np.cos(xs))
    print("max abs error: sin %.3e  cos %.3e" % (es.max(), ec.max()))
    us = es / np.spacing(np.abs(np.sin(xs)).astype(np.float32).clip(1e-30))
    uc = ec / np.spacing(np.abs(np.cos(xs)).astype(np.float32).clip(1e-30))
    big = np.abs(np.sin(xs)) > 1e-3
    bigc = np.abs(np.cos(xs)) > 1e-3
    print("max ulp (|value| > 1e-3): sin %.2f  cos %.2f" % (us[big].max(), uc[bigc].max()))
    # libm-in-fp32 reference for scale: numpy float32 sin
    es32 = np.abs(np.sin(x).astype(np.float64) - np.sin(xs))
    print("numpy fp32 sin max abs error for scale: %.3e" % es32.max())


if __name__ == "__main__":
    main()
