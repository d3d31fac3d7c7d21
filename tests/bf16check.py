"""bf16 ulp comparison of a kernel's output against the float64 oracle on the same operands (test helper).

A bf16 kernel output g of an f32-accumulated sum is round_bf16(e + d), where e is the exact (float64) value and d
the f32 summation error, so |g - e| <= 0.5 ulp(e) + |d| + a rounding-boundary slack.  The check:
  * >= 99.99 % of the elements within 1 bf16 ulp of e (ulp taken at |e|),
  * every element within 2 ulp, or — where e is so small that the summation error alone exceeds 2 ulp (outputs near
    zero after cancellation, relu outputs at 0 from a slightly negative sum) — within the f32 summation bound
    K * 2^-24 * sum|terms| + 1 ulp at (|e| + that bound), sum|terms| supplied by ``abs_terms(index)`` for just those
    elements.
"""

import numpy as np

U32 = 2.0 ** -24  # f32 unit roundoff


def ulp_bf16(e):
    """bf16 ulp at |e| (8 significant bits; the bf16 subnormal spacing 2^-133 below 2^-126)."""
    a = np.maximum(np.abs(np.asarray(e, np.float64)), 2.0 ** -126)
    return np.exp2(np.floor(np.log2(a)) - 7.0)


def check_bf16(name, g, e, k_terms=None, abs_terms=None, frac_1ulp=1e-4, max_ulp=2.0):
    """Assert the bound above; returns a stats dict.  ``k_terms``: products per element (the K of the sum);
    ``abs_terms(idx)``: sum |products| (+ |bias|) for the flat indices idx of elements beyond max_ulp."""
    g = np.asarray(g, np.float64).reshape(-1)
    e = np.asarray(e, np.float64).reshape(-1)
    assert g.shape == e.shape, (name, g.shape, e.shape)
    assert np.isfinite(g).all(), "%s: non-finite kernel output" % name
    err = np.abs(g - e)
    d = err / ulp_bf16(e)
    n_over1 = int((d > 1.0).sum())
    bad = np.nonzero(d > max_ulp)[0]
    stats = {"layer": name, "elements": int(g.size), "max_ulp": float(d.max()) if g.size else 0.0,
             "frac_over_1ulp": n_over1 / max(1, g.size), "beyond_%gulp" % max_ulp: int(bad.size)}
    assert n_over1 <= frac_1ulp * g.size, "%s: %d of %d elements beyond 1 bf16 ulp (%s)" % (name, n_over1, g.size,
                                                                                          stats)
    if bad.size:
        assert abs_terms is not None and k_terms is not None, "%s: %d elements beyond %g ulp (%s)" % (
            name, bad.size, max_ulp, stats)
        bound = k_terms * U32 * np.asarray(abs_terms(bad), np.float64)
        allowed = bound + ulp_bf16(np.abs(e[bad]) + bound)
        worst = float((err[bad] / allowed).max())
        stats["beyond_within_f32_sum_bound"] = worst
        assert worst <= 1.0, "%s: error beyond the f32 summation bound (ratio %g): %s" % (name, worst, stats)
    print("bf16check", stats)
    return stats


def check_f32_sum(name, g, e, k_terms, sum_abs, slack=4.0):
    """f32 outputs of a K-term f32 sum of exactly representable products: |g - e| <= slack * K * 2^-24 * sum|terms|
    (+ 1 f32 ulp of e for the final rounding)."""
    g = np.asarray(g, np.float64)
    e = np.asarray(e, np.float64)
    tol = slack * k_terms * U32 * np.asarray(sum_abs, np.float64) + np.abs(e) * 2.0 ** -23 + 1e-30
    ratio = np.abs(g - e) / tol
    assert np.isfinite(g).all() and ratio.max() <= 1.0, "%s: f32 sum error ratio %g" % (name, float(ratio.max()))
    stats = {"layer": name, "elements": int(g.size), "max_err_over_bound": float(ratio.max()),
             "max_abs_err": float(np.abs(g - e).max())}
    print("f32check", stats)
    return stats


def abs_conv_at(x, w, bias, idx, shape):
    """sum |x| |w| + |bias| of a 3x3 SAME conv at the flat output indices idx of an output of ``shape``
    (n, h, w, cout); x float64 [n,h,w,cin], w [3,3,cin,cout]."""
    n, h, wd, co = shape
    nn, hh, ww, cc = np.unravel_index(idx, shape)
    xp = np.pad(np.abs(x), ((0, 0), (1, 1), (1, 1), (0, 0)))
    aw = np.abs(np.asarray(w, np.float64))
    s = np.zeros(len(idx), np.float64)
    for kh in range(3):
        for kw in range(3):
            s += np.einsum("ic,ic->i", xp[nn, hh + kh, ww + kw], aw[kh, kw][:, cc].T)
    if bias is not None:
        s += np.abs(np.asarray(bias, np.float64))[cc]
    return s
