"""Probe: can pocketfft's real forward transform (scipy.fft.rfft, which is
also scipy.fft.fft of real input and so the forward half of
scipy.signal.hilbert, modem.py:309) be restated bit for bit?  A numpy
restatement of its FFTPACK-style passes (radf2/3/4/5) and its twiddle
generator, compared with scipy on this host.  Research for DESIGN.md §7
item 5 (FSK decisions inside digital silence); not product code.

    python tools/pocketfft_probe.py"""
import math

import numpy as np
import scipy.fft as F


def factorize(n):
    fact = []
    while n % 4 == 0:
        fact.append(4)
        n //= 4
    if n % 2 == 0:
        n //= 2
        fact.append(2)
        fact[0], fact[-1] = fact[-1], fact[0]
    d = 3
    while d * d <= n:
        while n % d == 0:
            fact.append(d)
            n //= d
        d += 2
    if n > 1:
        fact.append(n)
    return fact


class Twid:
    """pocketfft's sincos_2pibyn: exp(2 pi i k / n) from two tables."""

    def __init__(self, n):
        self.n = n
        # Thigh(0.25L*pi/n): x87 long double arithmetic, then rounded to double
        ang = float(np.longdouble("0.25") * np.longdouble("3.141592653589793238462643383279502884197") / np.longdouble(n))
        nval = (n + 2) // 2
        shift = 1
        while (1 << shift) * (1 << shift) < nval:
            shift += 1
        self.shift, self.mask = shift, (1 << shift) - 1
        self.v1 = [self.calc(i, n, ang) for i in range(self.mask + 1)]
        self.v1[0] = (1.0, 0.0)
        self.v2 = [self.calc(i * (self.mask + 1), n, ang) for i in range((nval + self.mask) // (self.mask + 1))]
        self.v2[0] = (1.0, 0.0)

    @staticmethod
    def calc(x, n, ang):
        x <<= 3
        if x < 4 * n:
            if x < 2 * n:
                if x < n:
                    return (math.cos(x * ang), math.sin(x * ang))
                return (math.sin((2 * n - x) * ang), math.cos((2 * n - x) * ang))
            x -= 2 * n
            if x < n:
                return (-math.sin(x * ang), math.cos(x * ang))
            return (-math.cos((2 * n - x) * ang), math.sin((2 * n - x) * ang))
        x = 8 * n - x
        if x < 2 * n:
            if x < n:
                return (math.cos(x * ang), -math.sin(x * ang))
            return (math.sin((2 * n - x) * ang), -math.cos((2 * n - x) * ang))
        x -= 2 * n
        if x < n:
            return (-math.sin(x * ang), -math.cos(x * ang))
        return (-math.cos((2 * n - x) * ang), -math.sin((2 * n - x) * ang))

    def __getitem__(self, idx):
        if 2 * idx <= self.n:
            x1, x2 = self.v1[idx & self.mask], self.v2[idx >> self.shift]
            return (x1[0] * x2[0] - x1[1] * x2[1], x1[0] * x2[1] + x1[1] * x2[0])
        idx = self.n - idx
        x1, x2 = self.v1[idx & self.mask], self.v2[idx >> self.shift]
        return (x1[0] * x2[0] - x1[1] * x2[1], -(x1[0] * x2[1] + x1[1] * x2[0]))


def rfft_twiddles(n, fact):
    tw = Twid(n)
    out, l1 = [], 1
    for k, ip in enumerate(fact):
        ido = n // (l1 * ip)
        t = np.zeros(max(0, (ip - 1) * (ido - 1)))
        if k < len(fact) - 1:
            for j in range(1, ip):
                for i in range(1, (ido - 1) // 2 + 1):
                    w = tw[j * l1 * i]
                    t[(j - 1) * (ido - 1) + 2 * i - 2] = w[0]
                    t[(j - 1) * (ido - 1) + 2 * i - 1] = w[1]
        out.append(t)
        l1 *= ip
    return out


def radf2(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 2 * c)] = v
    for k in range(l1):
        CHs(0, 0, k, CC(0, k, 0) + CC(0, k, 1))
        CHs(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 1))
    if ido % 2 == 0:
        for k in range(l1):
            CHs(0, 1, k, -CC(ido - 1, k, 1))
            CHs(ido - 1, 0, k, CC(ido - 1, k, 0))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1)
            ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1)
            CHs(i - 1, 0, k, CC(i - 1, k, 0) + tr2)
            CHs(ic - 1, 1, k, CC(i - 1, k, 0) - tr2)
            CHs(i, 0, k, ti2 + CC(i, k, 0))
            CHs(ic, 1, k, ti2 - CC(i, k, 0))


def radf3(ido, l1, cc, ch, wa):
    taur, taui = -0.5, 0.8660254037844386467637231707529362
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 3 * c)] = v
    WA = lambda x, i: wa[i + x * (ido - 1)]
    for k in range(l1):
        cr2 = CC(0, k, 1) + CC(0, k, 2)
        CHs(0, 0, k, CC(0, k, 0) + cr2)
        CHs(0, 2, k, taui * (CC(0, k, 2) - CC(0, k, 1)))
        CHs(ido - 1, 1, k, CC(0, k, 0) + taur * cr2)
    if ido == 1:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            cr2 = dr2 + dr3
            ci2 = di2 + di3
            CHs(i - 1, 0, k, CC(i - 1, k, 0) + cr2)
            CHs(i, 0, k, CC(i, k, 0) + ci2)
            tr2 = CC(i - 1, k, 0) + taur * cr2
            ti2 = CC(i, k, 0) + taur * ci2
            tr3 = taui * (di2 - di3)
            ti3 = taui * (dr3 - dr2)
            CHs(i - 1, 2, k, tr2 + tr3)
            CHs(ic - 1, 1, k, tr2 - tr3)
            CHs(i, 2, k, ti2 + ti3)
            CHs(ic, 1, k, ti3 - ti2)


def radf4(ido, l1, cc, ch, wa):
    hsqt2 = 0.707106781186547524400844362104849
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 4 * c)] = v
    WA = lambda x, i: wa[i + x * (ido - 1)]
    for k in range(l1):
        tr1 = CC(0, k, 3) + CC(0, k, 1)
        CHs(0, 2, k, CC(0, k, 3) - CC(0, k, 1))
        tr2 = CC(0, k, 0) + CC(0, k, 2)
        CHs(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 2))
        CHs(0, 0, k, tr2 + tr1)
        CHs(ido - 1, 3, k, tr2 - tr1)
    if ido % 2 == 0:
        for k in range(l1):
            ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3))
            tr1 = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3))
            CHs(ido - 1, 0, k, CC(ido - 1, k, 0) + tr1)
            CHs(ido - 1, 2, k, CC(ido - 1, k, 0) - tr1)
            CHs(0, 3, k, ti1 + CC(ido - 1, k, 2))
            CHs(0, 1, k, ti1 - CC(ido - 1, k, 2))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3)
            ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3)
            tr1, tr4 = cr4 + cr2, cr4 - cr2
            ti1, ti4 = ci2 + ci4, ci2 - ci4
            tr2, tr3 = CC(i - 1, k, 0) + cr3, CC(i - 1, k, 0) - cr3
            ti2, ti3 = CC(i, k, 0) + ci3, CC(i, k, 0) - ci3
            CHs(i - 1, 0, k, tr2 + tr1)
            CHs(ic - 1, 3, k, tr2 - tr1)
            CHs(i, 0, k, ti1 + ti2)
            CHs(ic, 3, k, ti1 - ti2)
            CHs(i - 1, 2, k, tr3 + ti4)
            CHs(ic - 1, 1, k, tr3 - ti4)
            CHs(i, 2, k, tr4 + ti3)
            CHs(ic, 1, k, tr4 - ti3)


def radf5(ido, l1, cc, ch, wa):
    tr11, ti11 = 0.3090169943749474241022934171828191, 0.9510565162951535721164393333793821
    tr12, ti12 = -0.8090169943749474241022934171828191, 0.5877852522924731291687059546390728
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 5 * c)] = v
    WA = lambda x, i: wa[i + x * (ido - 1)]
    for k in range(l1):
        cr2, ci5 = CC(0, k, 4) + CC(0, k, 1), CC(0, k, 4) - CC(0, k, 1)
        cr3, ci4 = CC(0, k, 3) + CC(0, k, 2), CC(0, k, 3) - CC(0, k, 2)
        CHs(0, 0, k, CC(0, k, 0) + cr2 + cr3)
        CHs(ido - 1, 1, k, CC(0, k, 0) + tr11 * cr2 + tr12 * cr3)
        CHs(0, 2, k, ti11 * ci5 + ti12 * ci4)
        CHs(ido - 1, 3, k, CC(0, k, 0) + tr12 * cr2 + tr11 * cr3)
        CHs(0, 4, k, ti12 * ci5 - ti11 * ci4)
    if ido == 1:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1)
            di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1)
            dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2)
            di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2)
            dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3)
            di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3)
            dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4)
            di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4)
            cr2, ci5 = dr5 + dr2, dr5 - dr2
            ci2, cr5 = di2 + di5, di2 - di5
            cr3, ci4 = dr4 + dr3, dr4 - dr3
            ci3, cr4 = di3 + di4, di3 - di4
            CHs(i - 1, 0, k, CC(i - 1, k, 0) + cr2 + cr3)
            CHs(i, 0, k, CC(i, k, 0) + ci2 + ci3)
            tr2 = CC(i - 1, k, 0) + tr11 * cr2 + tr12 * cr3
            ti2 = CC(i, k, 0) + tr11 * ci2 + tr12 * ci3
            tr3 = CC(i - 1, k, 0) + tr12 * cr2 + tr11 * cr3
            ti3 = CC(i, k, 0) + tr12 * ci2 + tr11 * ci3
            tr5, tr4 = cr5 * ti11 + cr4 * ti12, cr5 * ti12 - cr4 * ti11
            ti5, ti4 = ci5 * ti11 + ci4 * ti12, ci5 * ti12 - ci4 * ti11
            CHs(i - 1, 2, k, tr2 + tr5)
            CHs(ic - 1, 1, k, tr2 - tr5)
            CHs(i, 2, k, ti2 + ti5)
            CHs(ic, 1, k, ti5 - ti2)
            CHs(i - 1, 4, k, tr3 + tr4)
            CHs(ic - 1, 3, k, tr3 - tr4)
            CHs(i, 4, k, ti3 + ti4)
            CHs(ic, 3, k, ti4 - ti3)


PASSES = {2: radf2, 3: radf3, 4: radf4, 5: radf5}


def rfft(x):
    n = x.size
    fact = factorize(n)
    tws = rfft_twiddles(n, fact)
    c = [float(v) for v in x]
    ch = [0.0] * n
    p1, p2 = c, ch
    l1 = n
    for k1 in range(len(fact)):
        k = len(fact) - k1 - 1
        ip = fact[k]
        ido = n // l1
        l1 //= ip
        PASSES[ip](ido, l1, p1, p2, tws[k])
        p1, p2 = p2, p1
    r = p1
    out = np.zeros(n // 2 + 1, complex)
    out[0] = r[0]
    for i in range(1, (n - 1) // 2 + 1):
        out[i] = complex(r[2 * i - 1], r[2 * i])
    if n % 2 == 0:
        out[n // 2] = r[n - 1]
    return out


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for n in (2, 3, 4, 5, 8, 6, 10, 12, 15, 16, 20, 25, 30, 60, 100, 120, 300, 320, 960, 4000):
        x = rng.normal(size=n)
        a, b = rfft(x), F.rfft(x)
        ok = np.array_equal(a.view(np.float64), b.view(np.float64))
        print(n, factorize(n), "bit-exact" if ok else f"differs: max {np.abs(a - b).max():.3e}, "
              f"{int(np.sum(a.view(np.float64) != b.view(np.float64)))} words")


# ---- complex transforms (cfftp): the inverse half of hilbert ---------------
def cfactorize(n, with8):
    fact = []
    if with8:
        while n % 8 == 0:
            fact.append(8)
            n //= 8
    while n % 4 == 0:
        fact.append(4)
        n //= 4
    if n % 2 == 0:
        n //= 2
        fact.append(2)
        fact[0], fact[-1] = fact[-1], fact[0]
    d = 3
    while d * d <= n:
        while n % d == 0:
            fact.append(d)
            n //= d
        d += 2
    if n > 1:
        fact.append(n)
    return fact


def c_twiddles(n, fact):
    tw = Twid(n)
    out, l1 = [], 1
    for ip in fact:
        ido = n // (l1 * ip)
        t = [None] * ((ip - 1) * (ido - 1))
        for j in range(1, ip):
            for i in range(1, ido):
                t[(j - 1) * (ido - 1) + i - 1] = tw[j * l1 * i]
        out.append(t)
        l1 *= ip
    return out


def cadd(a, b): return (a[0] + b[0], a[1] + b[1])
def csub(a, b): return (a[0] - b[0], a[1] - b[1])


def smul(fwd, v, w):
    if fwd:
        return (v[0] * w[0] + v[1] * w[1], v[1] * w[0] - v[0] * w[1])
    return (v[0] * w[0] - v[1] * w[1], v[0] * w[1] + v[1] * w[0])


def rotx90(fwd, a):
    return (a[1], -a[0]) if fwd else (-a[1], a[0])


def pass2(fwd, ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + 2 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i - 1 + x * (ido - 1)]
    for k in range(l1):
        CHs(0, k, 0, cadd(CC(0, 0, k), CC(0, 1, k)))
        CHs(0, k, 1, csub(CC(0, 0, k), CC(0, 1, k)))
        for i in range(1, ido):
            CHs(i, k, 0, cadd(CC(i, 0, k), CC(i, 1, k)))
            CHs(i, k, 1, smul(fwd, csub(CC(i, 0, k), CC(i, 1, k)), WA(0, i)))


def pass4(fwd, ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + 4 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i - 1 + x * (ido - 1)]
    for k in range(l1):
        for i in range(ido):
            t2, t1 = cadd(CC(i, 0, k), CC(i, 2, k)), csub(CC(i, 0, k), CC(i, 2, k))
            t3, t4 = cadd(CC(i, 1, k), CC(i, 3, k)), csub(CC(i, 1, k), CC(i, 3, k))
            t4 = rotx90(fwd, t4)
            if i == 0:
                CHs(0, k, 0, cadd(t2, t3))
                CHs(0, k, 2, csub(t2, t3))
                CHs(0, k, 1, cadd(t1, t4))
                CHs(0, k, 3, csub(t1, t4))
            else:
                CHs(i, k, 0, cadd(t2, t3))
                CHs(i, k, 1, smul(fwd, cadd(t1, t4), WA(0, i)))
                CHs(i, k, 2, smul(fwd, csub(t2, t3), WA(1, i)))
                CHs(i, k, 3, smul(fwd, csub(t1, t4), WA(2, i)))


def pass3(fwd, ido, l1, cc, ch, wa):
    tw1r = -0.5
    tw1i = (-1 if fwd else 1) * 0.8660254037844386467637231707529362
    CC = lambda a, b, c: cc[a + ido * (b + 3 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i - 1 + x * (ido - 1)]
    for k in range(l1):
        for i in range(ido):
            t0 = CC(i, 0, k)
            t1, t2 = cadd(CC(i, 1, k), CC(i, 2, k)), csub(CC(i, 1, k), CC(i, 2, k))
            CHs(i, k, 0, cadd(t0, t1))
            ca = (t0[0] + t1[0] * tw1r, t0[1] + t1[1] * tw1r)
            cb = (-(t2[1] * tw1i), t2[0] * tw1i)
            if i == 0:
                CHs(0, k, 1, cadd(ca, cb))
                CHs(0, k, 2, csub(ca, cb))
            else:
                CHs(i, k, 1, smul(fwd, cadd(ca, cb), WA(0, i)))
                CHs(i, k, 2, smul(fwd, csub(ca, cb), WA(1, i)))


def pass5(fwd, ido, l1, cc, ch, wa):
    s = -1 if fwd else 1
    tw1r, tw1i = 0.3090169943749474241022934171828191, s * 0.9510565162951535721164393333793821
    tw2r, tw2i = -0.8090169943749474241022934171828191, s * 0.5877852522924731291687059546390728
    CC = lambda a, b, c: cc[a + ido * (b + 5 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i - 1 + x * (ido - 1)]
    for k in range(l1):
        for i in range(ido):
            t0 = CC(i, 0, k)
            t1, t4 = cadd(CC(i, 1, k), CC(i, 4, k)), csub(CC(i, 1, k), CC(i, 4, k))
            t2, t3 = cadd(CC(i, 2, k), CC(i, 3, k)), csub(CC(i, 2, k), CC(i, 3, k))
            CHs(i, k, 0, (t0[0] + t1[0] + t2[0], t0[1] + t1[1] + t2[1]))
            for (u1, u2, twar, twbr, twai, twbi) in ((1, 4, tw1r, tw2r, tw1i, tw2i), (2, 3, tw2r, tw1r, tw2i, -tw1i)):
                ca = (t0[0] + twar * t1[0] + twbr * t2[0], t0[1] + twar * t1[1] + twbr * t2[1])
                cb = (-(twai * t4[1] + twbi * t3[1]), twai * t4[0] + twbi * t3[0])
                if i == 0:
                    CHs(0, k, u1, cadd(ca, cb))
                    CHs(0, k, u2, csub(ca, cb))
                else:
                    CHs(i, k, u1, smul(fwd, cadd(ca, cb), WA(u1 - 1, i)))
                    CHs(i, k, u2, smul(fwd, csub(ca, cb), WA(u2 - 1, i)))


CPASSES = {2: pass2, 3: pass3, 4: pass4, 5: pass5}


def cfft(x, fwd, fct, with8=False):
    n = x.size
    fact = cfactorize(n, with8)
    tws = c_twiddles(n, fact)
    c = [(float(v.real), float(v.imag)) for v in x]
    ch = [None] * n
    p1, p2 = c, ch
    l1 = 1
    for k, ip in enumerate(fact):
        l2 = ip * l1
        ido = n // l2
        CPASSES[ip](fwd, ido, l1, p1, p2, tws[k])
        p1, p2 = p2, p1
        l1 = l2
    out = np.array([complex(v[0] * fct, v[1] * fct) if fct != 1.0 else complex(*v) for v in p1])
    return out


def ifft_check(sizes):
    rng = np.random.default_rng(3)
    for n in sizes:
        x = rng.normal(size=n) + 1j * rng.normal(size=n)
        fct = float(np.longdouble(1) / np.longdouble(n))
        want = F.ifft(x)
        for w8 in (False, True):
            if w8 and n % 8:
                continue
            got = cfft(x, False, fct, w8)
            ok = np.array_equal(got.view(np.float64), want.view(np.float64))
            print("ifft", n, cfactorize(n, w8), "bit-exact" if ok else
                  f"differs {int(np.sum(got.view(np.float64) != want.view(np.float64)))} words")


HSQT2 = 0.707106781186547524400844362104849


def rotx45(fwd, a):
    if fwd:
        return (HSQT2 * (a[0] + a[1]), HSQT2 * (a[1] - a[0]))
    return (HSQT2 * (a[0] - a[1]), HSQT2 * (a[1] + a[0]))


def rotx135(fwd, a):
    if fwd:
        return (HSQT2 * (a[1] - a[0]), HSQT2 * (-a[0] - a[1]))
    return (HSQT2 * (-a[0] - a[1]), HSQT2 * (a[0] - a[1]))


def pass8(fwd, ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + 8 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i - 1 + x * (ido - 1)]
    for k in range(l1):
        for i in range(ido):
            a1, a5 = cadd(CC(i, 1, k), CC(i, 5, k)), csub(CC(i, 1, k), CC(i, 5, k))
            a3, a7 = cadd(CC(i, 3, k), CC(i, 7, k)), csub(CC(i, 3, k), CC(i, 7, k))
            a1, a3 = cadd(a1, a3), csub(a1, a3)
            a3 = rotx90(fwd, a3)
            a7 = rotx90(fwd, a7)
            a5, a7 = cadd(a5, a7), csub(a5, a7)
            a5 = rotx45(fwd, a5)
            a7 = rotx135(fwd, a7)
            a0, a4 = cadd(CC(i, 0, k), CC(i, 4, k)), csub(CC(i, 0, k), CC(i, 4, k))
            a2, a6 = cadd(CC(i, 2, k), CC(i, 6, k)), csub(CC(i, 2, k), CC(i, 6, k))
            if i == 0:
                s02, d02 = cadd(a0, a2), csub(a0, a2)
                CHs(0, k, 0, cadd(s02, a1))
                CHs(0, k, 4, csub(s02, a1))
                CHs(0, k, 2, cadd(d02, a3))
                CHs(0, k, 6, csub(d02, a3))
                a6 = rotx90(fwd, a6)
                s46, d46 = cadd(a4, a6), csub(a4, a6)
                CHs(0, k, 1, cadd(s46, a5))
                CHs(0, k, 5, csub(s46, a5))
                CHs(0, k, 3, cadd(d46, a7))
                CHs(0, k, 7, csub(d46, a7))
            else:
                a0, a2 = cadd(a0, a2), csub(a0, a2)
                CHs(i, k, 0, cadd(a0, a1))
                CHs(i, k, 4, smul(fwd, csub(a0, a1), WA(3, i)))
                CHs(i, k, 2, smul(fwd, cadd(a2, a3), WA(1, i)))
                CHs(i, k, 6, smul(fwd, csub(a2, a3), WA(5, i)))
                a6 = rotx90(fwd, a6)
                a4, a6 = cadd(a4, a6), csub(a4, a6)
                CHs(i, k, 1, smul(fwd, cadd(a4, a5), WA(0, i)))
                CHs(i, k, 5, smul(fwd, csub(a4, a5), WA(4, i)))
                CHs(i, k, 3, smul(fwd, cadd(a6, a7), WA(2, i)))
                CHs(i, k, 7, smul(fwd, csub(a6, a7), WA(6, i)))


CPASSES[8] = pass8
