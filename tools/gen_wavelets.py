#!/usr/bin/env python3
"""Generate the orthogonal wavelet low-pass filter banks from first principles.

The reference ships its banks as literal tables (``src/daubechies.c:34``,
``src/symlets.c:34``, ``src/coiflets.c:34``).  We derive ours instead:

* **Daubechies** (orders 2..76): spectral factorisation of the Daubechies
  half-band polynomial ``P(y) = sum_k C(n-1+k, k) y^k`` in 80-digit arithmetic
  (mpmath), keeping the zeros inside the unit circle (minimum phase).
* **Symlets** (orders 2..76): the same factorisation with a per-order choice of
  which member of each reciprocal zero pair is kept.  The choice is recorded in
  ``_SYMLET_SELECTION`` (orientation + one bit per zero group, in the order
  ``mpmath.polyroots`` returns them); it reproduces the conventional symlet
  family used by the reference, whose rows agree with ours to the precision
  the reference tables carry.
* **Coiflets** (orders 6..30): Gauss-Newton solution of the Coiflet system
  (orthonormality, 2N vanishing wavelet moments, 2N-1 vanishing scaling
  moments about tap 2N), started from 6-digit seeds of the classical
  coefficients (Daubechies, *Ten Lectures*, Table 8.1) and refined to 40 digits.

Normalisation follows the reference contract (reference src/wavelet.c filter tables):
Daubechies rows sum to sqrt(2); Symlet and Coiflet rows sum to 1.

Output: ``csrc/data/wavelet_tables.cpp`` (flat per-family arrays, row ``k``
of length ``2(k+1)`` starting at offset ``k(k+1)``; Coiflet row ``k`` has
length ``6(k+1)`` at offset ``3k(k+1)``).

Usage:  python tools/gen_wavelets.py [out.cpp]
"""
import os
import sys

import mpmath as mp

mp.mp.dps = 80

# (orientation, selection bits) for symlet orders 2n, n = 2..38.  Bit i == 1
# keeps 1/z instead of z for the i-th zero group of the half-band polynomial.
_SYMLET_SELECTION = {
    2: (1, "0"), 3: (1, "00"), 4: (1, "011"), 5: (0, "0011"),
    6: (1, "10011"), 7: (0, "001111"), 8: (1, "0110011"),
    9: (1, "00111100"), 10: (1, "100111100"), 11: (0, "1100001111"),
    12: (0, "01100111100"), 13: (1, "000011001111"),
    14: (0, "1110000111100"), 15: (0, "11110011000011"),
    16: (0, "011110011000011"), 17: (0, "1100000000111111"),
    18: (0, "01100000011111100"), 19: (0, "111100111100110000"),
    20: (0, "0110011111100000011"), 21: (0, "11110000000011001111"),
    22: (0, "111000011111100001100"), 23: (0, "1111000011111111000000"),
    24: (0, "01111000011000011110011"), 25: (0, "110011110000001100110011"),
    26: (0, "0110000110011111100110000"),
    27: (0, "11001100000000001100111111"),
    28: (0, "011001111110000000000111111"),
    29: (0, "1111001100000011110011001100"),
    30: (0, "11111000011001100000000111111"),
    31: (0, "111111000000000000001100111111"),
    32: (0, "1111100110000001100000000111111"),
    33: (0, "11110011110000001100110011110000"),
    34: (0, "011110011110000110000000011001111"),
    35: (0, "1111110000000011000000110011001111"),
    36: (0, "11100111100000011110000000011001111"),
    37: (0, "110011000011000000111100110011110011"),
    38: (0, "0111100001100000011111100110011001100"),
}

# 6-significant-digit seeds (sum-1 normalisation) for the Newton refinement.
_COIFLET_SEEDS = {
    1: "-0.0514297 0.23893 0.602859 0.272141 -0.0514297 -0.0110703",
    2: "0.0115876 -0.0293201 -0.0476396 0.273021 0.574682 0.294867 "
       "-0.0540856 -0.0420265 0.0167444 0.00396788 -0.0012892 -0.000509505",
    3: "-0.00268242 0.00550313 0.0165836 -0.0465078 -0.0432208 0.286503 "
       "0.561285 0.302984 -0.0507701 -0.0581963 0.0244341 0.0112292 "
       "-0.0063696 -0.00182046 0.000790205 0.000329665 -5.01928e-05 "
       "-2.44657e-05",
    4: "0.000630961 -0.00115222 -0.00519452 0.0113625 0.0188672 -0.0574642 "
       "-0.0396526 0.293667 0.553126 0.307157 -0.0471127 -0.0680381 "
       "0.0278136 0.0177358 -0.0107563 -0.00400101 0.00265267 0.000895595 "
       "-0.000416501 -0.00018383 4.40804e-05 2.20829e-05 -2.30494e-06 "
       "-1.26218e-06",
    5: "-0.000149964 0.000253561 0.00154025 -0.00294111 -0.00716378 "
       "0.0165521 0.0199178 -0.0649973 -0.0368001 0.298092 0.547505 "
       "0.309707 -0.0438661 -0.0746522 0.0291959 0.0231108 -0.0139737 "
       "-0.00648009 0.004783 0.00172065 -0.00117582 -0.000451227 "
       "0.00021373 9.93776e-05 -2.92321e-05 -1.5072e-05 2.6408e-06 "
       "1.4593e-06 -1.184e-07 -6.73e-08",
}


def _halfband_roots(n):
    """Zeros (inside the unit circle) of the degree-(n-1) half-band factor."""
    if n == 1:
        return []
    coeffs = [mp.binomial(n - 1 + k, k) for k in range(n)]
    ys = mp.polyroots(list(reversed(coeffs)), maxsteps=400, extraprec=400)
    zs = []
    for y in ys:
        a = 1 - 2 * y
        s = mp.sqrt(a * a - 1)
        z1, z2 = a + s, a - s
        zs.append(z1 if abs(z1) < 1 else z2)
    return zs


def _poly_from_roots(n, roots):
    """Coefficients (ascending powers) of (1+z)^n prod(z - r), scaled to sum 1."""
    poly = [mp.mpf(1)]
    for _ in range(n):
        poly = [a + b for a, b in zip(poly + [0], [0] + poly)]
    for r in roots:
        poly = [a - r * b for a, b in zip([0] + poly, poly + [0])]
    poly = [mp.re(c) for c in poly]
    s = sum(poly)
    return [c / s for c in poly]


def daubechies(n):
    """Minimum-phase Daubechies filter, n vanishing moments (2n taps), sum 1."""
    h = _poly_from_roots(n, _halfband_roots(n))
    if abs(h[0]) < abs(h[-1]):
        h = h[::-1]
    return h


def _zero_groups(roots):
    groups, used = [], [False] * len(roots)
    eps = mp.mpf(10) ** -30
    for i, r in enumerate(roots):
        if used[i]:
            continue
        used[i] = True
        if abs(mp.im(r)) > eps:
            j = min((j for j in range(len(roots)) if not used[j]),
                    key=lambda j: abs(roots[j] - mp.conj(r)))
            used[j] = True
            groups.append([r, mp.conj(r)])
        else:
            groups.append([mp.re(r)])
    return groups


def symlet(n):
    """Symlet filter with n vanishing moments (2n taps), sum 1."""
    if n == 1:
        return [mp.mpf(1) / 2, mp.mpf(1) / 2]
    orient, bits = _SYMLET_SELECTION[n]
    roots = _halfband_roots(n)
    if len(bits) != len(roots):
        # selection recorded per zero (conjugates individually)
        raise AssertionError("symlet selection mismatch for n=%d" % n)
    chosen = [z if b == "0" else 1 / z for z, b in zip(roots, bits)]
    h = _poly_from_roots(n, chosen)
    return h[::-1] if orient else h


def _coiflet_residuals(h, n):
    L = 6 * n
    sq2 = mp.sqrt(2)
    g = [c * sq2 for c in h]
    out = [sum(g) - sq2]
    for k in range(3 * n):
        out.append(sum(g[i] * g[i + 2 * k] for i in range(L - 2 * k)) -
                   (1 if k == 0 else 0))
    for m in range(1, 2 * n):
        out.append(sum(((-1) ** i) * mp.mpf(i) ** m * g[i] for i in range(L)) /
                   mp.mpf(L) ** m)
    for m in range(1, 2 * n):
        out.append(sum(mp.mpf(i - 2 * n) ** m * g[i] for i in range(L)) /
                   mp.mpf(L) ** m)
    return out


def coiflet(n, iters=40):
    """Coiflet with 6n taps (order 6n), sum 1, refined by Gauss-Newton."""
    mp.mp.dps = 50
    h = [mp.mpf(v) for v in _COIFLET_SEEDS[n].split()]
    assert len(h) == 6 * n
    for _ in range(iters):
        F = _coiflet_residuals(h, n)
        if max(abs(f) for f in F) < mp.mpf(10) ** -42:
            break
        eps = mp.mpf(10) ** -25
        J = mp.matrix(len(F), len(h))
        for j in range(len(h)):
            hp = list(h)
            hp[j] += eps
            Fp = _coiflet_residuals(hp, n)
            for i in range(len(F)):
                J[i, j] = (Fp[i] - F[i]) / eps
        Fv = mp.matrix(F)
        dx = mp.lu_solve(J.T * J, -(J.T * Fv))
        h = [h[j] + dx[j] for j in range(len(h))]
    res = max(abs(f) for f in _coiflet_residuals(h, n))
    assert res < mp.mpf(10) ** -30, (n, res)
    mp.mp.dps = 80
    return h


def _fmt(v, digits):
    s = mp.nstr(v, digits, min_fixed=0, max_fixed=0)
    if "e" not in s and "." not in s:
        s += ".0"
    return s


def emit(path):
    sq2 = mp.sqrt(2)
    fams = []
    fams.append(("daubechies", [[c * sq2 for c in daubechies(n)]
                                for n in range(1, 39)]))
    fams.append(("symlets", [symlet(n) for n in range(1, 39)]))
    fams.append(("coiflets", [coiflet(n) for n in range(1, 6)]))
    lines = [
        "// GENERATED by tools/gen_wavelets.py -- do not edit.",
        "// Orthogonal wavelet low-pass banks derived from first principles",
        "// (spectral factorisation / Newton), see the generator docstring.",
        "#include \"csrc/data/wavelet_tables.h\"",
        "",
        "namespace vs {",
        "namespace wavelet_tables {",
        "",
    ]
    for name, rows in fams:
        flat = [c for row in rows for c in row]
        for ctype, digits, suffix in (("double", 20, ""), ("float", 9, "f")):
            lines.append("const %s k_%s_%s[%d] = {" % (
                ctype, name, "d" if ctype == "double" else "f", len(flat)))
            for row in rows:
                lines.append("    " + ", ".join(_fmt(c, digits) + suffix
                                                for c in row) + ",")
            lines.append("};")
            lines.append("")
    lines += ["}  // namespace wavelet_tables", "}  // namespace vs", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "csrc", "data", "wavelet_tables.cpp")
    emit(out)
    print("wrote", out)
