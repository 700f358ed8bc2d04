"""Rigorous first-order rounding bound of the f32 IDCT (pocketfft's DCT-III, ortho) at every slider
length: the input to the rank-1 pre-pass's eps_Y (csrc/tmfwm_rank1.hip).

The device and the reference compute Y = IDCT_fl(M) with pocketfft's op sequence in f32
(csrc/tmfwm_device.h dct::dct3 / rfft_forward / radf*; the op order is the parity contract).  This
script re-runs that op sequence on a value type that carries, next to the f32 value itself,
  c: the exact linear form of the value in the inputs (the algorithm's map with its f32 constants),
  e: a first-order bound of the accumulated rounding, |computed - c.x| <= u e.|x| (u = 2^-24):
     a rounded sum / difference / product by a constant adds |c| (|fl(s) - s| <= u |s|); an exact
     operation (negation, a product by a power of two) adds nothing.
Output per length N: the matrices C' (rows c) and E (rows e), and
  * the f32 values against the oracle's IDCT, bit for bit (pins the transcription);
  * max |C' - C| (C the exact orthonormal DCT-III matrix);
  * max E / |C| where |C| > 0, and whether |C| has zero entries (then no multiple of |C| can bound
    E: the pre-pass's `2 gamma_16 |C| |M| |C|^T` form is valid only where E <= 16 |C| entrywise).
usage: idct_bound.py [N ...]   (default 4 6 8 10 12 14 16)
       idct_bound.py --emit  -> thatsmyface_amd/csrc/tmfwm_idct_bounds.h (the pre-pass's tables)
"""
import math
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CONSTS = {}
for m in re.finditer(r"static constexpr float (\w+)(\[\d+\])? = \{?([^;}]*)\}?;",
                     open(os.path.join(ROOT, "thatsmyface_amd", "csrc", "tmfwm_consts.h")).read()):
    vals = [float.fromhex(t.strip()) for t in m.group(3).split(",") if t.strip()]
    CONSTS[m.group(1)] = vals if m.group(2) else vals[0]
F32 = np.float32
SQRT2, HSQT2 = float(F32(1.41421356237309504880)), float(F32(0.70710678118654752440))
TAUR, TAUI = float(F32(-0.5)), float(F32(0.8660254037844386467637231707529362))
TR11, TI11 = float(F32(0.3090169943749474241022934171828191)), float(F32(0.9510565162951535721164393333793821))
TR12, TI12 = float(F32(-0.8090169943749474241022934171828191)), float(F32(0.5877852522924731291687059546390728))


def _pow2(k):
    return k != 0 and math.frexp(abs(k))[0] == 0.5


class V:
    """an f32 value with its exact linear form c and first-order rounding bound e"""
    __slots__ = ("v", "c", "e")

    def __init__(self, v, c, e):
        self.v, self.c, self.e = F32(v), c, e

    def __add__(self, o):
        c = self.c + o.c
        return V(self.v + o.v, c, self.e + o.e + np.abs(c))

    def __sub__(self, o):
        c = self.c - o.c
        return V(self.v - o.v, c, self.e + o.e + np.abs(c))

    def __neg__(self):
        return V(-self.v, -self.c, self.e)

    def __rmul__(self, k):  # constant * value, the constant an f32 number
        k = float(F32(k))
        c = k * self.c
        return V(F32(k) * self.v, c, abs(k) * self.e + (0.0 if _pow2(k) else np.abs(c)))

    __mul__ = __rmul__


# ---- the device's op sequence (tmfwm_device.h), ido == 1 / 2 / ... as instantiated ----------
def radf2(cc, ido, l1, wa):
    ch = [None] * len(cc)
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]  # noqa: E731

    def CH(a, b, c, v):
        ch[a + ido * (b + 2 * c)] = v
    for k in range(l1):
        x, y = CC(0, k, 0), CC(0, k, 1)
        CH(0, 0, k, x + y)
        CH(ido - 1, 1, k, x - y)
    if ido % 2 == 0:
        for k in range(l1):
            CH(0, 1, k, -CC(ido - 1, k, 1))
            CH(ido - 1, 0, k, CC(ido - 1, k, 0))
    if ido > 2:
        for k in range(l1):
            for i in range(2, ido, 2):
                ic = ido - i
                w0, w1 = wa[i - 2], wa[i - 1]
                e, f = CC(i - 1, k, 1), CC(i, k, 1)
                tr2 = w0 * e + w1 * f
                ti2 = w0 * f - w1 * e
                a = CC(i - 1, k, 0)
                CH(i - 1, 0, k, a + tr2)
                CH(ic - 1, 1, k, a - tr2)
                c = CC(i, k, 0)
                CH(i, 0, k, ti2 + c)
                CH(ic, 1, k, ti2 - c)
    return ch


def radf4(cc, ido, l1, wa):
    ch = [None] * len(cc)
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]  # noqa: E731

    def CH(a, b, c, v):
        ch[a + ido * (b + 4 * c)] = v
    for k in range(l1):
        a, b = CC(0, k, 3), CC(0, k, 1)
        tr1 = a + b
        CH(0, 2, k, a - b)
        a, b = CC(0, k, 0), CC(0, k, 2)
        tr2 = a + b
        CH(ido - 1, 1, k, a - b)
        CH(0, 0, k, tr2 + tr1)
        CH(ido - 1, 3, k, tr2 - tr1)
    if ido % 2 == 0:
        for k in range(l1):
            ti1 = -HSQT2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3))
            tr1 = HSQT2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3))
            a = CC(ido - 1, k, 0)
            CH(ido - 1, 0, k, a + tr1)
            CH(ido - 1, 2, k, a - tr1)
            c = CC(ido - 1, k, 2)
            CH(0, 3, k, ti1 + c)
            CH(0, 1, k, ti1 - c)
    if ido > 2:
        for k in range(l1):
            for i in range(2, ido, 2):
                ic = ido - i
                w0, w1 = wa[i - 2], wa[i - 1]
                e, f = CC(i - 1, k, 1), CC(i, k, 1)
                cr2, ci2 = w0 * e + w1 * f, w0 * f - w1 * e
                w0, w1 = wa[(ido - 1) + i - 2], wa[(ido - 1) + i - 1]
                e, f = CC(i - 1, k, 2), CC(i, k, 2)
                cr3, ci3 = w0 * e + w1 * f, w0 * f - w1 * e
                w0, w1 = wa[2 * (ido - 1) + i - 2], wa[2 * (ido - 1) + i - 1]
                e, f = CC(i - 1, k, 3), CC(i, k, 3)
                cr4, ci4 = w0 * e + w1 * f, w0 * f - w1 * e
                tr1, tr4 = cr4 + cr2, cr4 - cr2
                ti1, ti4 = ci2 + ci4, ci2 - ci4
                a, c = CC(i - 1, k, 0), CC(i, k, 0)
                tr2, tr3 = a + cr3, a - cr3
                ti2, ti3 = c + ci3, c - ci3
                CH(i - 1, 0, k, tr2 + tr1)
                CH(ic - 1, 3, k, tr2 - tr1)
                CH(i, 0, k, ti1 + ti2)
                CH(ic, 3, k, ti1 - ti2)
                CH(i - 1, 2, k, tr3 + ti4)
                CH(ic - 1, 1, k, tr3 - ti4)
                CH(i, 2, k, tr4 + ti3)
                CH(ic, 1, k, tr4 - ti3)
    return ch


def radf3(cc, l1):
    ch = [None] * len(cc)
    for k in range(l1):
        cr2 = cc[k + l1] + cc[k + 2 * l1]
        ch[3 * k] = cc[k] + cr2
        ch[2 + 3 * k] = TAUI * (cc[k + 2 * l1] - cc[k + l1])
        ch[1 + 3 * k] = cc[k] + TAUR * cr2
    return ch


def radf5(cc, l1):
    ch = [None] * len(cc)
    for k in range(l1):
        cr2, ci5 = cc[k + 4 * l1] + cc[k + l1], cc[k + 4 * l1] - cc[k + l1]
        cr3, ci4 = cc[k + 3 * l1] + cc[k + 2 * l1], cc[k + 3 * l1] - cc[k + 2 * l1]
        ch[5 * k] = cc[k] + cr2 + cr3
        ch[5 * k + 1] = cc[k] + TR11 * cr2 + TR12 * cr3
        ch[5 * k + 2] = TI11 * ci5 + TI12 * ci4
        ch[5 * k + 3] = cc[k] + TR12 * cr2 + TR11 * cr3
        ch[5 * k + 4] = TI12 * ci5 - TI11 * ci4
    return ch


def radfg(cc, ip, l1, cs):
    """result left in cc (ch scratch), as the device's radfg"""
    cc = list(cc)
    ch = [None] * len(cc)
    ipph = (ip + 1) // 2
    for j in range(1, ipph):
        jc = ip - j
        for k in range(l1):
            t1, t2 = cc[k + l1 * j], cc[k + l1 * jc]
            cc[k + l1 * j] = t2 + t1
            cc[k + l1 * jc] = t2 - t1
    for l in range(1, ipph):
        lc = ip - l
        for ik in range(l1):
            ch[ik + l1 * l] = cc[ik] + cs[2 * l] * cc[ik + l1] + cs[4 * l] * cc[ik + 2 * l1]
            ch[ik + l1 * lc] = cs[2 * l + 1] * cc[ik + l1 * (ip - 1)] + cs[4 * l + 1] * cc[ik + l1 * (ip - 2)]
        iang = 2 * l
        for j in range(3, ipph):
            jc = ip - j
            iang += l
            if iang > ip:
                iang -= ip
            for ik in range(l1):
                ch[ik + l1 * l] = ch[ik + l1 * l] + cs[2 * iang] * cc[ik + l1 * j]
                ch[ik + l1 * lc] = ch[ik + l1 * lc] + cs[2 * iang + 1] * cc[ik + l1 * jc]
    for ik in range(l1):
        ch[ik] = cc[ik]
    for j in range(1, ipph):
        for ik in range(l1):
            ch[ik] = ch[ik] + cc[ik + l1 * j]
    for k in range(l1):
        cc[ip * k] = ch[k]
    for j in range(1, ipph):
        jc, j2 = ip - j, 2 * j - 1
        for k in range(l1):
            cc[j2 + ip * k] = ch[k + l1 * j]
            cc[j2 + 1 + ip * k] = ch[k + l1 * jc]
    return cc


def rfft_forward(c, n, fct):
    if n == 4:
        ch = radf4(c, 1, 1, None)
        return [fct * x for x in ch]
    if n == 6:
        c = radf2(radf3(c, 2), 3, 1, CONSTS["kRfftTw6"])
    elif n == 8:
        c = radf2(radf4(c, 1, 2, None), 4, 1, CONSTS["kRfftTw8"])
    elif n == 10:
        c = radf2(radf5(c, 2), 5, 1, CONSTS["kRfftTw10"])
    elif n == 12:
        c = radf4(radf3(c, 4), 3, 1, CONSTS["kRfftTw12"])
    elif n == 14:
        c = radfg(c, 7, 2, CONSTS["kRfftTws14"])
        ch = radf2(c, 7, 1, CONSTS["kRfftTw14"])
        return [fct * x for x in ch]
    else:
        c = radf4(radf4(c, 1, 4, None), 4, 1, CONSTS["kRfftTw16"])
    return [fct * x for x in c]


def dct3(c, n):
    ns2 = (n + 1) // 2
    tw = CONSTS[f"kDctTw{n}"]
    c = list(c)
    c[0] = SQRT2 * c[0]
    for k in range(1, ns2):
        kc = n - k
        t1, t2 = c[k] + c[kc], c[k] - c[kc]
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2
    c[ns2] = (2.0 * tw[ns2 - 1]) * c[ns2]
    c = rfft_forward(c, n, CONSTS[f"kNorm{n}"])
    for k in range(1, n - 1, 2):
        t = c[k]
        c[k] = t - c[k + 1]
        c[k + 1] = t + c[k + 1]
    return c


def exact_idct(n):
    """C[p][i]: the orthonormal DCT-III (scipy idct norm='ortho'), y = C x"""
    p, i = np.arange(n)[:, None], np.arange(n)[None, :]
    s = np.where(i == 0, math.sqrt(1.0 / n), math.sqrt(2.0 / n))
    return s * np.cos(math.pi * (2 * p + 1) * i / (2 * n))


def analyse(n, samples=None):
    x0 = np.zeros(n)
    out = dct3([V(0.0, np.eye(n)[i], np.zeros(n)) for i in range(n)], n)
    Cp = np.array([o.c for o in out])
    E = np.array([o.e for o in out])
    C = exact_idct(n)
    nz = np.abs(C) > 1e-12
    ratio = np.where(nz, E / np.where(nz, np.abs(C), 1.0), np.inf)
    res = {"n": n, "max_C_prime_minus_C": float(np.abs(Cp - C).max()),
           "zero_entries_of_C": int((~nz).sum()), "E_max": float(E.max()),
           "max_E_over_absC": float(ratio[nz].max()),
           "E_at_zero_entries_max": float(E[~nz].max()) if (~nz).any() else 0.0}
    if samples is not None:
        # the f32 values, 2-D (columns then rows), against the oracle's IDCT bit for bit
        from oracle import oracle as O
        got = np.empty_like(samples)
        for bi, blk in enumerate(samples):
            t = np.empty((n, n), np.float32)
            for col in range(n):
                t[:, col] = [o.v for o in dct3([V(blk[r, col], x0, x0) for r in range(n)], n)]
            for row in range(n):
                got[bi, row, :] = [o.v for o in dct3([V(t[row, cc], x0, x0) for cc in range(n)], n)]
        ref = O.dct2d_blocks(samples, inverse=True)
        res["f32_values_equal_oracle"] = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
    return res, Cp, E


def _up(v):
    """the smallest f32 >= v (v >= 0)"""
    f = F32(v)
    return float(f) if float(f) >= v else float(np.nextafter(f, F32(np.inf)))


def tables(n):
    """the pre-pass's tables: |C'| and E rounded up to f32, E with a 2^-16 allowance for the
    higher-order terms of the first-order analysis (at most ~12 roundings deep, each 2^-24)"""
    _, Cp, E = analyse(n)
    absc = [[_up(abs(x) * (1 + 2.0**-40) + 2.0**-60) for x in row] for row in Cp]
    err = [[_up(x * (1 + 2.0**-16)) for x in row] for row in E]
    return absc, err


def emit(path):
    out = ["// Generated by tools/exp/idct_bound.py --emit: do not edit.  The rank-1 pre-pass's IDCT",
           "// tables (DESIGN.md 5): absc[p][i] >= |C'[p][i]|, C' the exact linear map of the f32 IDCT",
           "// (pocketfft's DCT-III, ortho) with its f32 constants; err[p][i] >= E[p][i], the first-order",
           "// rounding bound |IDCT_fl(x)_p - (C' x)_p| <= 2^-24 sum_i E[p][i] |x_i| of that op sequence.",
           "#pragma once", "", "namespace tmf {", "", "template <int B>", "struct IdctBound;"]
    for n in (4, 6, 8, 10, 12, 14, 16):
        absc, err = tables(n)
        out.append(f"template <>\nstruct IdctBound<{n}> {{")
        for name, t in (("absc", absc), ("err", err)):
            out.append(f"    static constexpr float {name}[{n}][{n}] = {{")
            for row in t:
                out.append("        {" + ", ".join(float(x).hex() + "f" for x in row) + "},")
            out.append("    };")
        out.append("};")
    out += ["", "}  // namespace tmf", ""]
    open(path, "w").write("\n".join(out))


def main():
    if sys.argv[1:2] == ["--emit"]:
        emit(os.path.join(ROOT, "thatsmyface_amd", "csrc", "tmfwm_idct_bounds.h"))
        return
    ns = [int(a) for a in sys.argv[1:]] or [4, 6, 8, 10, 12, 14, 16]
    rng = np.random.default_rng(5)
    for n in ns:
        smp = (rng.standard_normal((6, n, n)) * rng.uniform(0.01, 30, (6, 1, 1))).astype(np.float32)
        res, _, _ = analyse(n, smp)
        print(res, flush=True)


if __name__ == "__main__":
    main()
