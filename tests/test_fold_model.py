"""CPU model of the row-order fold's exact block step (wx::xf_sums / XfTies /
xf_block in warpdb_amd/csrc/kernels/wx_util.hip), restated in Python floats
(IEEE doubles, round half to even -- the arithmetic of the reference's
`g.sum += val`, src/warpdb.cpp:373-385).

Whenever the model takes the fast path (one exact integer sum per block), its
result must equal the dependent chain s = ((s + v0) + v1) + ... bit for bit;
blocks it rejects fall back to that chain.  The GPU tests check the kernels
themselves (tests/test_gpu_group_row_order.py); this pins the algebra: the
binade lemma (inside one binade every step is s + round_u(v)) and the tie scan
(a tie's rounding depends only on S's parity and leaves S even)."""
from __future__ import annotations

import math

import numpy as np

M = 1.5 * 2.0 ** 52


def _popc(x: int) -> int:
    return bin(x).count("1")


class Ties:
    """XfTies::row over rows of 64 values, in row order."""

    def __init__(self):
        self.seen = self.cpar = self.has = self.cf = 0
        self.adj = 0

    def row(self, tie, bpar):
        pm = sum(1 << i for i, p in enumerate(bpar) if p)
        tm = sum(1 << i for i, t in enumerate(tie) if t)
        if tm == 0:
            self.cpar ^= _popc(pm) & 1
            return
        plus, cfl = [False] * 64, [0] * 64
        for lane in range(64):
            if not tie[lane]:
                continue
            below, bp = (1 << lane) - 1, int(bpar[lane])
            tb = tm & below
            if tb:
                lt = tb.bit_length() - 1
                plus[lane] = ((_popc(pm & below & ~((2 << lt) - 1)) & 1) ^ bp) != 0
            elif self.seen:
                plus[lane] = ((self.cpar ^ (_popc(pm & below) & 1)) ^ bp) != 0
            else:
                cfl[lane] = (self.cpar ^ (_popc(pm & below) & 1)) ^ bp
        self.adj += sum(plus)
        if not self.seen:
            self.has, self.cf = 1, cfl[(tm & -tm).bit_length() - 1]
        lt = tm.bit_length() - 1
        self.cpar = _popc(pm & ~((2 << lt) - 1) & ((1 << 64) - 1)) & 1
        self.seen = 1


def block_fast(s: float, x: np.ndarray):
    """The fast path of one block of 64 * J values (row j = x[64 j : 64 j + 64]);
    None when it does not apply."""
    if not (2.0 ** -900 <= abs(s) < 2.0 ** 1000):
        return None
    k = math.frexp(s)[1] - 1
    p2 = math.ldexp(1.0, 52 - k)
    t = a = 0
    T = Ties()
    for j in range(0, len(x), 64):
        tie, bpar = [], []
        for v in x[j:j + 64]:
            q = float(v) * p2
            if not abs(q) < 2.0 ** 44:
                return None
            r = (q + M) - M
            ti = abs(q - r) == 0.5
            b = r - 1.0 if ti and r > q else r
            t += int(b)
            a += abs(int(b)) + (1 if ti else 0)
            tie.append(ti)
            bpar.append(int(b) & 1)
        T.row(tie, bpar)
    S = int(math.ldexp(s, 52 - k))
    lo, hi = 1 << 52, 1 << 53
    if not (S - a > lo and S + a < hi if s > 0 else S + a < -lo and S - a > -hi):
        return None
    R = t + T.adj + ((S & 1) ^ T.cf if T.has else 0)
    return math.ldexp(float(S + R), k - 52)


def chain(s: float, x) -> float:
    for v in x:
        s = s + float(v)
    return s


def _check(s0, x):
    fast = block_fast(s0, x)
    want = chain(s0, x)
    if fast is not None:
        assert np.float64(fast).view(np.uint64) == np.float64(want).view(np.uint64), (s0, fast, want)
    return fast is not None


def test_fast_path_equals_chain_with_ties():
    rng = np.random.default_rng(7)
    taken = 0
    for _ in range(300):
        # half the values ties against u = 2^-19 under a 1.5 * 2^33 start
        x = (rng.integers(-8, 9, 512).astype(np.float32) * np.float32(2.0 ** -20)).astype(np.float32)
        taken += _check(1.5 * 2.0 ** 33 + rng.integers(0, 1 << 20) * 2.0 ** -19, x)
    assert taken == 300


def test_fast_path_equals_chain_mixed():
    rng = np.random.default_rng(11)
    taken = 0
    for _ in range(300):
        scale = rng.choice(np.array([1e4, 1.0, 1e-3, 40.0], np.float32), 512)
        x = (rng.uniform(-1.0, 1.0, 512).astype(np.float32) * scale).astype(np.float32)
        s0 = float(rng.uniform(1e5, 1e9)) * float(rng.choice([1.0, -1.0]))
        taken += _check(s0, x)
    assert taken > 200  # most blocks stay in their binade


def test_fast_path_rejects_crossings():
    # a block that carries the sum across a power of two must not take the fast path
    x = np.full(512, 1.0, np.float32)
    assert block_fast(2.0 ** 20 - 100.0, x) is None
    assert block_fast(0.0, x) is None
    assert _check(2.0 ** 20 + 1000.0, x)
