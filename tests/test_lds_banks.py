"""Host model of the LDS bank conflicts of the FFT exchanges (fft_core.hpp
pass_exchange / pass_exchange_ri): the per-pass paddings ri_pad<2048, p> and
cx_pad<4096, 1> are one-to-one, fit the transform's buffer, and leave no
conflict in any exchange write or read, where Geo::pad (e + (e >> 4)) cost one
extra LDS cycle per 32-lane group of every exchange read (the N = 2048 kernel's
SQ_LDS_BANK_CONFLICT, profiles/r06_pmc_stft256_2048_pow.txt).

Banking follows /opt/skills/guides/MI355X_MICROARCH.md (LDS table):
ds_write_b32 / ds_read_b32 in two 32-lane groups, bank (a/4) mod 32;
ds_write_b64 in four 16-lane groups, bank (a/4) mod 32; ds_read_b64 in two
32-lane groups, bank (a/4) mod 64.  Extra cycles = per group, the largest
number of distinct dword addresses on one bank, minus one."""


def _radix(n, p):
    lg = n.bit_length() - 1
    return n if n < 16 else (16 if lg - 4 * p >= 4 else 1 << (lg - 4 * p))


def _geo(n):
    pp = 16 if n >= 16 else n
    lg = n.bit_length() - 1
    return pp, n // pp, ((lg + 3) // 4 if n >= 16 else 1)


def _ns(n, p):
    s = 1
    for q in range(p):
        s *= _radix(n, q)
    return s


def _bfly(n, p, t, i, paired):
    pp, tt, npass = _geo(n)
    nb = n // _radix(n, npass - 1)
    if paired and tt > 1 and p == npass - 1:
        b0 = t + tt * (i >> 1)
        if (i & 1) == 0:
            return b0
        return nb // 2 if b0 == 0 else nb - b0
    return t + tt * i


def _extra(addr, width, groups, nbanks):
    ex = 0
    for g in groups:
        banks = {}
        for lane in g:
            if lane in addr:
                for d in range(width):
                    banks.setdefault((addr[lane] + d) % nbanks, set()).add(addr[lane] + d)
        if banks:
            ex += max(len(v) for v in banks.values()) - 1
    return ex


G32 = [list(range(0, 32)), list(range(32, 64))]
G16 = [list(range(k, k + 16)) for k in range(0, 64, 16)]


def _exchange(n, paired, p, pad, complex_):
    """extra LDS cycles of exchange p over every wave of one transform"""
    pp, tt, _ = _geo(n)
    r1, ns, r2 = _radix(n, p), _ns(n, p), _radix(n, p + 1)
    w_dw, scale = (2, 2) if complex_ else (1, 1)
    ex = 0
    for wave in range(max(1, tt // 64)):
        for i in range(pp // r1):
            for r in range(r1):
                a = {}
                for lane in range(64):
                    t = (64 * wave + lane) % tt
                    b = _bfly(n, p, t, i, paired)
                    a[lane] = scale * pad((b // ns) * ns * r1 + b % ns + r * ns)
                ex += _extra(a, w_dw, G16 if complex_ else G32, 32)
        for i in range(pp // r2):
            for r in range(r2):
                a = {}
                for lane in range(64):
                    t = (64 * wave + lane) % tt
                    a[lane] = scale * pad(_bfly(n, p + 1, t, i, paired) + r * (n // r2))
                ex += _extra(a, w_dw, G32, 64 if complex_ else 32)
    return ex


def geo_pad(e):
    return e + (e >> 4)


RI2048 = {0: lambda e: e + (e >> 5), 1: lambda e: e + 16 * (e >> 8)}   # fft_core.hpp ri_pad<2048, p>
CX4096 = {1: lambda e: e + (e >> 9)}                                    # fft_core.hpp cx_pad<4096, 1>


def test_pads_one_to_one_and_inside_the_buffer():
    for pad, n, cap in [(RI2048[0], 2048, 2048 + 128), (RI2048[1], 2048, 2048 + 128),
                        (CX4096[1], 4096, 4096 + 256)]:
        idx = [pad(e) for e in range(n)]
        assert all(b > a for a, b in zip(idx, idx[1:]))
        assert idx[-1] < cap


def test_2048_exchanges_conflict_free():
    for p in (0, 1):
        assert _exchange(2048, True, p, geo_pad, False) > 0   # what the old padding cost
        assert _exchange(2048, True, p, RI2048[p], False) == 0


def test_4096_second_exchange_conflict_free():
    assert _exchange(4096, False, 1, geo_pad, True) > 0
    assert _exchange(4096, False, 1, CX4096[1], True) == 0
