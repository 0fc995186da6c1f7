"""Exhaustive CPU checks behind the device's Halton fast paths
(cuda-raytrace_amd/csrc/pm_device.h permuted_halton4), which must equal the
reference's loop (photontracing.cu:19-31: digit p[n % base], then the quirk
`n *= invBase` on a uint — a float multiply truncated) bit for bit:

* bases 3, 5, 7: below 12,582,912 the quirk's truncated product equals
  n / base, so the device takes the digit as m - base * next instead of a
  modulo (halton_chains<true>); at and above it the device uses the modulo.
  Checked for every m < 2^24, with the first mismatches where the device
  switches paths;
* base 2: for n < 2^24 the quirk is an exact halving and the loop's float
  sum equals bitreverse(n) / 2^32 (table (0,1)) or (1 - 2^-L) - that
  (table (1,0)), L = bit length of n. Checked for every n < 2^24.
"""
import numpy as np

N24 = 1 << 24


def test_quirk_equals_division_below_12582912():
    m = np.arange(N24, dtype=np.uint32)
    mf = m.astype(np.float32)
    first = {}
    for b in (3, 5, 7):
        q = (mf * (np.float32(1.0) / np.float32(b))).astype(np.uint32)
        bad = np.nonzero(q != m // np.uint32(b))[0]
        first[b] = int(bad[0]) if bad.size else None
        assert bad.size == 0 or bad[0] >= 12_582_912, (b, bad[:4])
    assert first[7] == 12_582_912 and first[3] == 12_582_914, first


def _bitreverse32(v):
    v = v.astype(np.uint32)
    v = ((v >> 1) & 0x55555555) | ((v & 0x55555555) << 1)
    v = ((v >> 2) & 0x33333333) | ((v & 0x33333333) << 2)
    v = ((v >> 4) & 0x0F0F0F0F) | ((v & 0x0F0F0F0F) << 4)
    v = ((v >> 8) & 0x00FF00FF) | ((v & 0x00FF00FF) << 8)
    return ((v >> 16) | (v << 16)).astype(np.uint32)


def test_base2_closed_form_equals_loop():
    n = np.arange(N24, dtype=np.uint32)
    rev = _bitreverse32(n).astype(np.float32) * np.float32(2.0 ** -32)
    L = np.zeros(N24, np.int32)
    nz = n > 0
    L[nz] = np.floor(np.log2(n[nz].astype(np.float64))).astype(np.int32) + 1
    for table in ((0, 1), (1, 0)):
        p = np.asarray(table, np.uint32)
        val = np.zeros(N24, np.float32)
        inv = np.float32(1.0) / np.float32(2.0)
        invBi = np.full(N24, inv, np.float32)
        m = n.copy()
        for _ in range(25):                      # every loop of photontracing.cu:21-29
            live = m > 0
            d = p[m % 2].astype(np.float32)
            val = np.where(live, val + d * invBi, val).astype(np.float32)
            m = np.where(live, (m.astype(np.float32) * inv).astype(np.uint32), m)
            invBi = np.where(live, invBi * inv, invBi).astype(np.float32)
        assert not (m > 0).any()
        closed = rev if table[0] == 0 else (np.float32(1.0) - np.ldexp(np.float32(1.0), -L).astype(np.float32)) - rev
        assert np.array_equal(val.view(np.uint32), closed.astype(np.float32).view(np.uint32)), table
