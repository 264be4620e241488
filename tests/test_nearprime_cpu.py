"""The near-prime partition's arithmetic (khmer_amd/csrc/kh_nearprime.cuh,
np_geometry in kh_engine.hip), restated in Python and checked against the
reference's per-table reduction h % p_i (include/oxli/storage.hh:577) on the
tables khmer itself sizes (get_n_primes_near_x, include/oxli/hashtable.hh:
99-123).

Level 1 keeps, per k-mer, only (q, r) = divmod(h, P) for the largest table
size P and buckets it by r; level 2 recovers every table's bin as
(r + q (P - p_i)) mod p_i with one subtraction and routes it to destination
i * Rloc + (its region - R' b) (+ table i's regions when it wrapped).  This
test walks edge hashes (0, 4^k - 1, multiples of P and of every p_i +- 1,
bucket boundaries, wrap-around) and random ones through that arithmetic for
the C2 / C4 geometries and checks the bins, the destination range, the
record bit layout and the bucket magic.  Tables past 256 level-1 buckets (C4)
take three levels: k_scatter_n1b splits each coarse bucket into F fine ones
and rewrites the record as j << 32 | q << ob_f | offset; the same bins come
out of level 2 over the fine geometry."""
import random

import pytest

S0 = 14
R = 1 << S0


def is_prime(n):
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def primes_near(n, x):
    """get_n_primes_near_x: the n largest primes <= x (hashtable.hh:99-123)."""
    out, v = [], int(x)
    while len(out) < n:
        if is_prime(v):
            out.append(v)
        v -= 1
    return out


def ceil_log2(x):
    s = 0
    while (1 << s) < x:
        s += 1
    return s


def np_geometry(sizes, k, span_bits=24, lim=256):
    """np_geometry (kh_engine.hip) restated; None when the path is not taken.
    More than `lim` level-1 buckets: three levels (G["F"] fine buckets of
    G["rpf"] regions a coarse bucket of G["rp"] = F x rpf regions)."""
    n = len(sizes)
    if not 2 <= n <= 4 or k > 26:
        return None
    tbase, base = [], 0
    span = 1 << span_bits
    for p in sizes:
        tbase.append(base)
        base += (p + span - 1) // span * span
    pm = max(sizes)
    d = [pm - p for p in sizes]
    qmax = ((1 << 2 * k) - 1) // pm
    if qmax >= 1 << 31:
        return None
    maxoff = qmax * max(d)
    if maxoff + 2 * max(d) >= pm:
        return None
    rloc = 1024 // n
    E = (maxoff + R - 1) >> S0
    if E + 1 >= rloc // 2:
        return None
    rpf = rloc - E - 1
    Rm = (pm + R - 1) >> S0
    F, rp1, fine = 1, rpf, None
    if (Rm + rpf - 1) // rpf > lim:   # three levels
        qb = ceil_log2(qmax + 1)
        if qb + S0 + 1 > 32:
            return None
        rp1 = min(rpf, ((1 << (32 - qb)) - 1) // R)
        F = (Rm + rp1 * lim - 1) // (rp1 * lim)
        obf = ceil_log2(rp1 * R + 1)
        if F > 16 or obf + qb > 32:
            return None
        fine = dict(F=F, rp=rp1, ob=obf, magic=((1 << 32) + rp1 - 1) // rp1, rloc=rp1 + E + 1)
    rp = rp1 * F
    nb = (Rm + rp - 1) // rp
    if nb > lim:
        return None
    ob = ceil_log2(rp * R + 1)
    pb = ob + ceil_log2(qmax + 1)
    if pb > 42 or 64 - pb < 26:
        return None
    magic = ((1 << 32) + rp - 1) // rp
    return dict(n=n, pm=pm, d=d, p=list(sizes), qmax=qmax, rloc=rloc, rp=rp, nb=nb, ob=ob, pb=pb, magic=magic,
                rt=[(p + R - 1) >> S0 for p in sizes], rbase=[t >> S0 for t in tbase], Rm=Rm, E=E, fine=fine)


def fine_geometry(G):
    """np_fine_geo: level 2's view of a three-level partition."""
    f = G["fine"]
    H = dict(G)
    H.update(rp=f["rp"], magic=f["magic"], nb=G["nb"] * f["F"], ob=f["ob"], pb=32, rloc=f["rloc"], fine=None)
    return H


def level1b(G, b, pay, j):
    """k_scatter_n1b: coarse bucket b's record -> (fine bucket, fine record)."""
    f = G["fine"]
    q, off = pay >> G["ob"], pay & ((1 << G["ob"]) - 1)
    fb = ((off >> S0) * f["magic"]) >> 32
    assert fb < f["F"] and fb == (off >> S0) // f["rp"]
    offf = off - fb * (f["rp"] << S0)
    assert 0 <= offf < f["rp"] << S0
    rec = (j << 32) | (q << f["ob"]) | offf
    assert (q << f["ob"]) | offf < 1 << 32 and rec != (1 << 64) - 1
    return b * f["F"] + fb, rec & 0xFFFFFFFF


def level1(G, h):
    """k_scatter_n1's hash_rank: (bucket, payload) of hash h."""
    q, r = divmod(h, G["pm"])
    b = ((r >> S0) * G["magic"]) >> 32
    off = r - b * (G["rp"] << S0)
    assert 0 <= off < G["rp"] << S0 and off != (1 << G["ob"]) - 1
    pay = (q << G["ob"]) | off
    assert pay < 1 << G["pb"]
    return b, pay


def level2(G, b, pay):
    """k_scatter_n2's expansion: (destination, global region, offset) per table."""
    q, off = pay >> G["ob"], pay & ((1 << G["ob"]) - 1)
    r = b * (G["rp"] << S0) + off
    out = []
    for i in range(G["n"]):
        v = r + q * G["d"][i]
        assert v < 2 * G["p"][i]
        bin_ = v - G["p"][i] if v >= G["p"][i] else v
        rho = bin_ >> S0
        loc = rho - G["rp"] * b
        if loc < 0:
            loc += G["rt"][i]
        assert 0 <= loc < G["rloc"], (i, loc)
        # the destination maps back to the same region (greg in k_scatter_n2)
        rr = G["rp"] * b + loc
        if rr >= G["rt"][i]:
            rr -= G["rt"][i]
        assert rr == rho
        out.append((i * G["rloc"] + loc, G["rbase"][i] + rho, bin_ & (R - 1), bin_))
    return out


def edge_hashes(G, k, rnd, nrand):
    hmax = (1 << 2 * k) - 1
    hs = {0, 1, hmax, hmax - 1}
    for p in G["p"]:
        for m in (1, 2, 3, G["qmax"] - 1, G["qmax"]):
            for e in (-1, 0, 1):
                hs.add(m * p + e)
    # the start / end of every bucket's range of r, at the largest quotients
    for b in range(G["nb"]):
        for r in (b * (G["rp"] << S0), (b + 1) * (G["rp"] << S0) - 1):
            for q in (0, G["qmax"] // 2, G["qmax"]):
                hs.add(q * G["pm"] + min(r, G["pm"] - 1))
    # wrap-around: r near P at the largest quotient
    for t in range(1, 300):
        hs.add(G["qmax"] * G["pm"] + G["pm"] - t)
    hs.update(rnd.randrange(0, hmax + 1) for _ in range(nrand))
    return sorted(h for h in hs if 0 <= h <= hmax)


@pytest.mark.parametrize("x,k,expect_nb", [(1e9, 21, 255), (1e9, 19, None), (8e9, 21, None), (5e8, 21, None),
                                           (2e9, 21, None)])
def test_bins_equal_per_table_modulo(x, k, expect_nb):
    sizes = primes_near(4, x)
    G = np_geometry(sizes, k)
    if G is None:
        pytest.skip("near-prime path not taken for %g, k=%d" % (x, k))
    if expect_nb is not None:
        assert G["nb"] == expect_nb
    # C2's geometry as DESIGN.md states it
    if (x, k) == (1e9, 21):
        assert (G["qmax"], G["rp"], G["ob"], G["pb"]) == (4398, 240, 22, 35)
    rnd = random.Random(int(x) ^ k)
    hs = edge_hashes(G, k, rnd, 3000)
    H = fine_geometry(G) if G["fine"] else G
    for h in hs:
        b, pay = level1(G, h)
        assert b < G["nb"]
        if G["fine"]:   # three levels (tables past 256 buckets: C4's 8e9, 2e9)
            b, pay = level1b(G, b, pay, j=7)
        for i, (dst, greg, off, bin_) in enumerate(level2(H, b, pay)):
            assert bin_ == h % G["p"][i]
            assert dst < H["n"] * H["rloc"] <= 1024


def test_bucket_magic_exact():
    for x in (1e9, 8e9, 2e9):
        G = np_geometry(primes_near(4, x), 21)
        if G is None:
            continue
        for rho in range(G["Rm"]):
            assert (rho * G["magic"]) >> 32 == rho // G["rp"]


def test_geometry_refusals():
    # primes far apart (q d_i spans more than a bucket): not taken
    assert np_geometry([1000000007, 900000011, 800000011, 700000001], 21) is None
    # one table or k too large for a double-exact hash: not taken
    assert np_geometry(primes_near(1, 1e9), 21) is None
    assert np_geometry(primes_near(4, 1e9), 31) is None
    # C3 / C5 (k = 31) and small tables (C1: 4 x 1e7, q_max d_max > the table) keep the per-table level 1
    assert np_geometry(primes_near(4, 1e7), 21) is None


def test_record_layout_and_span():
    """Record = (j - block base) << PB | payload: the ~0 sentinel is never a
    record, and the block span 2^(64 - PB) - 1 covers far more than a tile."""
    G = np_geometry(primes_near(4, 1e9), 21)
    jbits = 64 - G["pb"]
    assert jbits == 29 and (1 << jbits) - 1 >= 4096 * 32
    worst = (((1 << jbits) - 1) << G["pb"]) | (G["qmax"] << G["ob"]) | (G["rp"] * R - 1)
    assert worst != (1 << 64) - 1


@pytest.mark.parametrize("x,k,lim,expect", [(8e9, 21, 256, (8, 242, 253)), (1e8, 19, 8, (13, 8, 63)),
                                            (1e9, 21, 128, (16, 124, 31))])
def test_three_level_bins_equal_per_table_modulo(x, k, lim, expect):
    """C4 (and the GPU tests' KH_NP_L1MAX geometries): level 1 into coarse
    buckets, level 1b into fine ones (q and the offset in 32 bits beside the
    pass index), level 2 from the fine record -- every table's bin is still
    h % p_i and every destination is inside the fine bucket's range."""
    G = np_geometry(primes_near(4, x), k, lim=lim)
    assert G is not None and G["fine"] is not None
    assert (G["fine"]["F"], G["nb"], G["fine"]["rp"]) == expect
    H = fine_geometry(G)
    assert H["n"] * H["rloc"] <= 1024
    rnd = random.Random(int(x) ^ k ^ lim)
    hs = edge_hashes(G, k, rnd, 2000) + edge_hashes(H, k, rnd, 0)
    for h in hs:
        b, pay = level1(G, h)
        assert b < G["nb"]
        fb, fpay = level1b(G, b, pay, j=12345)
        for i, (dst, greg, off, bin_) in enumerate(level2(H, fb, fpay)):
            assert bin_ == h % G["p"][i]
            assert dst < H["n"] * H["rloc"]


def test_three_level_magic_exact():
    G = np_geometry(primes_near(4, 8e9), 21)
    f = G["fine"]
    for rho in range(G["Rm"]):
        assert (rho * G["magic"]) >> 32 == rho // G["rp"]
    for rho in range(G["rp"]):
        assert (rho * f["magic"]) >> 32 == rho // f["rp"]
