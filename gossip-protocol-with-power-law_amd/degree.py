"""Degree-distribution check of an overlay.

The reference's demonstrate_powerlaw.py holds no such check (it imports networkx
and never uses it, demonstrate_powerlaw.py:2; SURVEY.md §0 finding 3), so this is
the build's own definition (parity unpinned): degree histogram, log-binned CCDF
and the discrete power-law MLE exponent with k_min chosen by minimum
Kolmogorov-Smirnov distance (Clauset, Shalizi & Newman 2009, eq. 3.7).
"""
import numpy as np


def histogram(deg):
    deg = np.asarray(deg, dtype=np.int64)
    return np.bincount(deg)


def ccdf(deg, bins=32):
    """Log-binned complementary CDF: (k, P[D >= k]) at geometric k."""
    deg = np.asarray(deg, dtype=np.int64)
    deg = deg[deg > 0]
    if deg.size == 0:
        return np.zeros(0), np.zeros(0)
    ks = np.unique(np.geomspace(1, deg.max(), bins).astype(np.int64))
    s = np.sort(deg)
    p = 1.0 - np.searchsorted(s, ks, side="left") / s.size
    return ks, p


def fit_gamma(deg, kmin_candidates=None, min_tail=50):
    """Discrete MLE gamma_hat = 1 + n / sum(ln(k / (kmin - 0.5))) over the tail
    k >= kmin; kmin minimises the KS distance between the empirical and fitted
    tail CCDFs.  Returns (gamma_hat, kmin, ks_distance, n_tail).

    Works on the degree histogram (suffix sums of counts and of count * ln k),
    so each kmin candidate costs O(#distinct degrees): the 2^26-vertex C5
    overlay is checked in well under a second."""
    deg = np.asarray(deg, dtype=np.int64)
    h = np.bincount(deg[deg > 0]) if deg.size else np.zeros(1, np.int64)
    ks_all = np.nonzero(h)[0]
    cnt = h[ks_all]
    N = int(cnt.sum())
    if N < min_tail:
        return float("nan"), 0, float("nan"), N
    suf = np.cumsum(cnt[::-1])[::-1]                          # #{deg >= ks_all[i]}
    lsum = np.cumsum((cnt * np.log(ks_all))[::-1])[::-1]      # sum of ln k over that tail
    if kmin_candidates is None:
        # distinct degrees up to the (N - min_tail)-th smallest degree
        thr = ks_all[np.searchsorted(np.cumsum(cnt), max(0, N - min_tail), side="right")]
        kmin_candidates = ks_all[ks_all <= thr]
        if kmin_candidates.size > 64:
            kmin_candidates = np.unique(np.geomspace(ks_all[0], kmin_candidates[-1], 64).astype(np.int64))
    best = (float("nan"), 0, float("inf"), 0)
    for kmin in kmin_candidates:
        i0 = int(np.searchsorted(ks_all, kmin))
        nt = int(suf[i0]) if i0 < ks_all.size else 0
        if nt < min_tail:
            continue
        g = 1.0 + nt / (lsum[i0] - nt * np.log(kmin - 0.5))
        # fitted continuous-approximation CCDF vs empirical, at the tail's degrees
        ks = ks_all[i0:]
        emp = suf[i0:] / nt
        fit = ((ks - 0.5) / (kmin - 0.5)) ** (1.0 - g)
        d = float(np.max(np.abs(emp - fit)))
        if d < best[2]:
            best = (float(g), int(kmin), d, nt)
    return best


def check_powerlaw(deg, gamma, tol=0.15):
    """Pass rule for generated overlays: |gamma_hat - gamma| <= tol."""
    g, kmin, d, nt = fit_gamma(deg)
    return {"gamma_hat": g, "kmin": kmin, "ks": d, "n_tail": nt,
            "mean_degree": float(np.mean(deg)) if len(deg) else 0.0,
            "max_degree": int(np.max(deg)) if len(deg) else 0,
            "ok": bool(abs(g - gamma) <= tol)}
