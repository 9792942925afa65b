"""Host-side proofs of the bit-sliced B3/S23 circuits in gol_kernels.hip.

The kernels evaluate the rule with v_bitop3_b32 gates whose 8-bit truth
tables are literals in the source.  These tests read those literals and check,
over every input combination, that the circuits compute the rule of
main.cpp:87-89 (`next = sum==3 || (alive && sum==2)` with sum = the 8
neighbours; here S = sum + alive, so next = S==3 || (alive && S==4)).
No GPU needed.
"""
import os
import re

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi_amd", "csrc",
                   "gol_kernels.hip")


def _bitop3(tt, a, b, c):
    """v_bitop3_b32 on single bits: result = tt[(a<<2)|(b<<1)|c]."""
    return (tt >> ((a << 2) | (b << 1) | c)) & 1


def _body(fn):
    s = open(SRC).read()
    i = s.index(fn)
    return s[i:s.index("\n}\n", i)]


def _tables(body):
    return [int(t, 16) for t in re.findall(r"bitop3_b32\([^;]*?,\s*(0x[0-9A-Fa-f]+)\)", body)]


def test_life_bits_circuit():
    """life_bits: vertical adders (xor3/maj) + the 4-gate rule, all 2^7 inputs, mask = 1."""
    u_t, s_t, m_t, f_t = _tables(_body("uint32_t life_bits("))
    xor3 = lambda a, b, c: a ^ b ^ c
    maj = lambda a, b, c: (a & b) | (a & c) | (b & c)
    for r in range(128):
        a0, a1, b0, b1, c0, c1, al = [(r >> i) & 1 for i in range(7)]
        o, co, p, q = xor3(a0, b0, c0), maj(a0, b0, c0), xor3(a1, b1, c1), maj(a1, b1, c1)
        u = _bitop3(u_t, co, p, 1)
        s = _bitop3(s_t, q, co, p)
        m = _bitop3(m_t, u, o, s)
        nxt = _bitop3(f_t, m, u, al)
        S = a0 + b0 + c0 + 2 * (a1 + b1 + c1)
        assert nxt == int(S == 3 or (al and S == 4)), r
        # mask = 0 forces a dead cell dead
        if not al:
            u0 = _bitop3(u_t, co, p, 0)
            assert _bitop3(f_t, _bitop3(m_t, u0, o, s), u0, al) == 0


def test_life_bits_full_circuit():
    """life_bits_full (interior words, no column mask): u = co ^ p as a plain
    XOR, then the same three rule gates, all 2^7 inputs."""
    s_t, m_t, f_t = _tables(_body("uint32_t life_bits_full("))
    assert "const uint32_t u = co ^ p;" in _body("uint32_t life_bits_full(")
    xor3 = lambda a, b, c: a ^ b ^ c
    maj = lambda a, b, c: (a & b) | (a & c) | (b & c)
    for r in range(128):
        a0, a1, b0, b1, c0, c1, al = [(r >> i) & 1 for i in range(7)]
        o, co, p, q = xor3(a0, b0, c0), maj(a0, b0, c0), xor3(a1, b1, c1), maj(a1, b1, c1)
        u = co ^ p
        nxt = _bitop3(f_t, _bitop3(m_t, u, o, _bitop3(s_t, q, co, p)), u, al)
        S = a0 + b0 + c0 + 2 * (a1 + b1 + c1)
        assert nxt == int(S == 3 or (al and S == 4)), r


@pytest.mark.parametrize("alive_row", ["first", "second"])
def test_life_pair_circuit(alive_row):
    """life_pair (the k=8 row-pair pipeline): every horizontal-sum triple of the
    three rows and every consistent alive bit; alive's row is one of the pair
    (the don't-cares the 4-gate circuit relies on)."""
    g1_t, g2_t, g3_t, f_t = _tables(_body("uint32_t life_pair("))
    rows = [(L, C, R) for L in (0, 1) for C in (0, 1) for R in (0, 1)]   # H = L + C + R of one row
    for A in rows:           # the single row (H(r-2) for output r-1, H(r+1) for output r)
        for X in rows:       # the pair rows
            for Y in rows:
                hA, hX, hY = sum(A), sum(X), sum(Y)
                alive = X[1] if alive_row == "first" else Y[1]
                x0, x1 = hX & 1, hX >> 1                  # pair code exactly as pair_event forms it
                y0, y1 = hY & 1, hY >> 1
                p0, k = x0 ^ y0, x0 & y0
                e0 = x1 ^ y1 ^ k
                e1 = (x1 & y1) | (x1 & k) | (y1 & k)
                a0, a1 = hA & 1, hA >> 1
                g1 = _bitop3(g1_t, p0, a0, alive)
                g2 = _bitop3(g2_t, e0, e1, a1)
                g3 = _bitop3(g3_t, e0, a1, alive)
                nxt = _bitop3(f_t, g3, g1, g2)
                S = hA + hX + hY
                assert p0 + 2 * e0 + 4 * e1 == hX + hY
                assert nxt == int(S == 3 or (alive and S == 4)), (A, X, Y)
