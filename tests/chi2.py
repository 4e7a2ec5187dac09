"""Pearson chi^2 goodness-of-fit test of an emitter's sample_direction against
its pdf_direction -- a restatement of mitsuba's ChiSquareTest
(src/python/python/chi2.py:5-370, math.h:325-352 pooling) over torch/numpy,
driving the GPU product through sunsky_amd.  Test infrastructure.

Differences from the reference harness, none of which changes the statistic:
uniform variates come from torch's generator instead of TEA-seeded PCG32
(chi2.py:117-124), and histogram binning runs with torch.bincount instead of
dr.scatter_reduce.
"""
import math

import numpy as np
import torch
from scipy.special import gammaincc


class SphericalDomain:
    """[phi, -cos theta] parameterisation of the sphere (chi2.py:416-437)."""

    def __init__(self, sin_offset=0.0):
        # CroppedSphericalDomain of test_sunsky.py:228-234 when sin_offset > 0
        cos_bound = math.sqrt(1 - sin_offset * sin_offset) if sin_offset > 0 else 1.0
        self.min = np.array([-math.pi, -cos_bound], np.float32)
        self.max = np.array([math.pi, 1.0], np.float32)

    def aspect(self):
        return 2

    def map_forward(self, p):         # (n, 2) torch -> (3, n)
        cos_theta = -p[:, 1]
        sin_theta = torch.sqrt(torch.clamp(torch.addcmul(torch.ones_like(cos_theta), -cos_theta, cos_theta), min=0))
        return torch.stack([torch.cos(p[:, 0]) * sin_theta, torch.sin(p[:, 0]) * sin_theta, cos_theta])

    def map_backward(self, d):        # (3, n) -> (n, 2)
        return torch.stack([torch.atan2(d[1], d[0]), -d[2]], dim=1)


def pool_chi2(obs, exp, pool_threshold=5.0):
    """mitsuba::math::chi2 (math.h:325-352)."""
    chsq, pooled_obs, pooled_exp = 0.0, 0.0, 0.0
    dof = n_in = n_out = 0
    for o, e in zip(obs.tolist(), exp.tolist()):
        if e == 0 and o == 0:
            continue
        if e < pool_threshold:
            pooled_obs += o
            pooled_exp += e
            n_in += 1
            if pooled_exp > pool_threshold:
                diff = pooled_obs - pooled_exp
                chsq += diff * diff / pooled_exp
                pooled_obs = pooled_exp = 0.0
                n_out += 1
                dof += 1
        else:
            diff = o - e
            chsq += diff * diff / e
            dof += 1
    return chsq, dof - 1, n_in, n_out


class ChiSquareTest:
    def __init__(self, domain, sample_func, pdf_func, sample_count=1_000_000, res=101, ires=4, seed=0,
                 device="cuda", chunk=1 << 24, drop_outside=False):
        # drop_outside: samples outside a cropped domain are left out of the histogram
        # (the pdf integral leaves the same region out) instead of the reference
        # harness's clip into the border cells, which at >=2.5e8 samples piles the
        # cropped cap's mass into one row.
        assert ires >= 2
        self.domain, self.sample_func, self.pdf_func = domain, sample_func, pdf_func
        self.sample_count, self.ires, self.seed, self.device, self.chunk = sample_count, ires, seed, device, chunk
        self.drop_outside = drop_outside
        self.res = np.array([max(int(res / domain.aspect()), 1), res])
        self.messages, self.fail = "", False
        self.histogram = self.pdf = self.p_value = None

    def _log(self, m):
        self.messages += m + "\n"

    def tabulate_histogram(self):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed)
        rx, ry = int(self.res[0]), int(self.res[1])
        lo = torch.tensor(self.domain.min, device=self.device)
        ext = torch.tensor(self.domain.max - self.domain.min, device=self.device)
        eps = ext * 1e-4
        hist = torch.zeros(rx * ry, dtype=torch.float64, device=self.device)
        done = 0
        while done < self.sample_count:
            m = min(self.chunk, self.sample_count - done)
            u = torch.rand((2, m), generator=g, device=self.device, dtype=torch.float32)
            d = self.sample_func(u)
            xy = self.domain.map_backward(d)
            inside = ((xy >= lo - eps) & (xy <= lo + ext + eps)).all(dim=1)
            if self.drop_outside:
                xy = xy[((xy >= lo) & (xy <= lo + ext)).all(dim=1)]
            elif not bool(inside.all()):
                self._log("Encountered samples outside of the specified domain!")
                self.fail = True
            xy = (xy - lo) / ext
            res_f = torch.tensor([rx, ry], dtype=torch.float32, device=self.device)
            cell = torch.minimum(torch.clamp(xy * res_f, min=0), res_f - 1).to(torch.int64)
            hist += torch.bincount(cell[:, 0] + cell[:, 1] * rx, minlength=rx * ry).to(torch.float64)
            done += m
        self.histogram = hist.cpu().numpy()
        self.histogram_sum = self.histogram.sum() / self.sample_count
        if self.histogram_sum > 1.1:
            self._log(f"Sample weights add up to a value greater than 1.0: {self.histogram_sum}")
            self.fail = True

    def tabulate_pdf(self):
        rx, ry, ires = int(self.res[0]), int(self.res[1]), self.ires
        lo = self.domain.min.astype(np.float64)
        ext = (self.domain.max - self.domain.min).astype(np.float64)
        cell = ext / self.res
        spacing = cell / (ires - 1)
        # cell-major, then sample index (chi2.py:197-222), positions in fp32 like the reference
        cy, cx, sy, sx = np.meshgrid(np.arange(ry), np.arange(rx), np.arange(ires), np.arange(ires), indexing="ij")
        px = lo[0] + cx * cell[0] + (sx + 1e-4) * (1 - 2e-4) * spacing[0]
        py = lo[1] + cy * cell[1] + (sy + 1e-4) * (1 - 2e-4) * spacing[1]
        w = np.where((sx == 0) | (sx == ires - 1), 0.5, 1.0) * np.where((sy == 0) | (sy == ires - 1), 0.5, 1.0)
        w = w * spacing[0] * spacing[1] * self.sample_count
        p = torch.from_numpy(np.stack([px.ravel(), py.ravel()], 1).astype(np.float32)).to(self.device)
        pdf = self.pdf_func(self.domain.map_forward(p).contiguous()).double().cpu().numpy()
        self.pdf = (pdf * w.ravel()).reshape(ry * rx, ires * ires).sum(axis=1)
        if self.pdf.min() < 0:
            self._log("Failure: Encountered a cell with a negative PDF value")
            self.fail = True
        self.pdf_sum = self.pdf.sum() / self.sample_count
        if self.pdf_sum > 1.1:
            self._log(f"Failure: PDF integrates to a value greater than 1.0: {self.pdf_sum}")
            self.fail = True

    def run(self, significance_level=0.01, test_count=1):
        if self.histogram is None:
            self.tabulate_histogram()
        if self.pdf is None:
            self.tabulate_pdf()
        order = np.argsort(self.pdf, kind="stable")
        pdf, hist = self.pdf[order], self.histogram[order]
        chi2val, dof, n_in, n_out = pool_chi2(hist, pdf, 5)
        if dof < 1:
            self._log("Failure: The number of degrees of freedom is too low!")
            self.fail = True
        if np.any((pdf == 0) & (hist != 0)):
            self._log("Failure: Found samples in a cell with expected frequency 0.")
            self.fail = True
        self._log(f"Histogram sum = {self.histogram_sum:f}, PDF sum = {self.pdf_sum:f}")
        self._log(f"Chi^2 statistic = {chi2val:f} (d.o.f = {dof})")
        self.p_value = float(gammaincc(dof / 2, chi2val / 2))   # 1 - rlgamma(dof/2, chi2/2)
        significance_level = 1.0 - (1.0 - significance_level) ** (1.0 / test_count)
        if self.fail:
            return False
        if not np.isfinite(self.p_value) or self.p_value < significance_level:
            self._log(f"***** Rejected ***** the null hypothesis (p-value = {self.p_value:f})")
            return False
        self._log(f"Accepted the null hypothesis (p-value = {self.p_value:f}, significance level = "
                  f"{significance_level:f})")
        return True


def emitter_adapter(emitter):
    """EmitterAdapter (chi2.py:530-567) for a sunsky_amd.SunskyEmitter."""
    import sunsky_amd as ss

    def sample_func(u):
        ds, _ = emitter.sample_direction(ss.Interaction3f(), u)
        return ds.d

    def pdf_func(d):
        return emitter.pdf_direction(ss.Interaction3f(), ss.DirectionSample3f(d=d))

    return sample_func, pdf_func


def two_sample_chi2(h1, h2, min_count=10):
    """Chi^2 homogeneity test of two histograms with different totals (Press et al.,
    Numerical Recipes 14.3): are both samples drawn from the same distribution?
    Bins with fewer than `min_count` combined counts are pooled.  -> (chi2, dof, p)."""
    h1, h2 = np.asarray(h1, np.float64), np.asarray(h2, np.float64)
    n1, n2 = h1.sum(), h2.sum()
    order = np.argsort(h1 + h2, kind="stable")
    a, b = h1[order], h2[order]
    k1, k2 = math.sqrt(n2 / n1), math.sqrt(n1 / n2)
    chsq, dof, pa, pb = 0.0, 0, 0.0, 0.0
    for x, y in zip(a.tolist(), b.tolist()):
        if x + y == 0:
            continue
        if x + y < min_count:
            pa += x
            pb += y
            if pa + pb >= min_count:
                chsq += (k1 * pa - k2 * pb) ** 2 / (pa + pb)
                dof += 1
                pa = pb = 0.0
            continue
        chsq += (k1 * x - k2 * y) ** 2 / (x + y)
        dof += 1
    dof -= 1
    return chsq, dof, float(gammaincc(dof / 2, chsq / 2))
