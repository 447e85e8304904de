#!/usr/bin/env python3
"""Generate delta-node_amd/csrc/mt19937_jump.inc: jump-ahead polynomials of
CPython's MT19937 for the device coefficient draw (dn_mt19937_draw_coeffs_device).

MT19937's one-word transition f (window (x_T..x_T+623) -> (x_T+1..x_T+624),
x_{T+624} = x_{T+397} ^ twist(x_T, x_{T+1})) is F2-linear on its 19937
effective state bits.  Its characteristic polynomial P (degree 19937) is found
here by Berlekamp-Massey on 2*19937 bits of one coordinate sequence; jumping J
words is then g(f) with g = x^J mod P, evaluated by Horner (Haramoto,
Matsumoto, Nishimura, Panneton, L'Ecuyer, "Efficient jump ahead for F2-linear
random number generators", INFORMS J. Computing 20(3), 2008).

Emitted: P is not needed at run time, only g for the substream windows of
the device draw (L = 17 * 2^14 words = 2^14 whole 521-bit draws per substream).
Window s >= 1 starts L - 624 + (s - 1) L words after the caller's position;
with s - 1 = 4096 c + 64 a + b (radix-64 digits, c, a, b < 64) it is
  W(1 + 64 a)               = A_a (W_idx),  A_a = x^(L - 624 + 64 a L), a = 0..63
  W(1 + 4096 c + 64 a)      = C_c (W(1 + 64 a)),  C_c = x^(4096 c L), c = 1..63
  W(1 + 4096 c + 64 a + b)  = B_b (W(1 + 4096 c + 64 a)),  B_b = x^(b L), b = 1..63
so every window is at most three jumps from the caller's window, and all the
windows of one level are independent (one GPU launch per level).
The script checks the two smallest polynomials against plain stepping, and
every product against an independent square-and-multiply.
Run once; the output is committed (~1.3 MB of hex).
"""
import os
import random
import sys

N, M = 624, 397
UP, LO, MA = 0x80000000, 0x7FFFFFFF, 0x9908B0DF
L_WORDS = 17 * (1 << 14)
RADIX = 64
DEG = 19937


def step(win):
    y = (win[0] & UP) | (win[1] & LO)
    return win[1:] + [win[M] ^ (y >> 1) ^ (MA if y & 1 else 0)]


def berlekamp_massey(bits):
    sint = 0
    for i, b in enumerate(bits):
        sint |= b << i
    C, B, L, m = 1, 1, 0, 1
    for i in range(len(bits)):
        if i >= L:
            seg = (sint >> (i - L)) & ((1 << (L + 1)) - 1)
            rev = int(bin(seg)[2:].zfill(L + 1)[::-1], 2)
            d = bin(C & rev).count("1") & 1
        else:
            d = bits[i]
            for j in range(1, L + 1):
                d ^= ((C >> j) & 1) & bits[i - j]
        if d == 0:
            m += 1
        elif 2 * L <= i:
            C, B, L, m = C ^ (B << m), C, i + 1 - L, 1
        else:
            C ^= B << m
            m += 1
    return C, L


SPREAD = [int("".join("0" + c for c in bin(b)[2:].zfill(8)), 2) for b in range(256)]


def sq(a):
    r, sh = 0, 0
    while a:
        r |= SPREAD[a & 0xFF] << sh
        a >>= 8
        sh += 16
    return r


def mod(a, P):
    d = P.bit_length() - 1
    while a.bit_length() - 1 >= d:
        a ^= P << (a.bit_length() - 1 - d)
    return a


def clmul(a, b):
    """carry-less product, 8-bit windows of b"""
    tab = [0] * 256
    for m in range(1, 256):
        low = m & -m
        tab[m] = tab[m ^ low] ^ (a << (low.bit_length() - 1))
    r, sh = 0, 0
    while b:
        r ^= tab[b & 0xFF] << sh
        b >>= 8
        sh += 8
    return r


class Reducer:
    """a mod P, eight bits at a time: R[t] clears the top byte t."""

    def __init__(self, P):
        self.P = P
        self.d = P.bit_length() - 1
        self.R = [0] * 256
        for t in range(256):
            v, q = t << self.d, 0
            for i in range(7, -1, -1):
                if (v >> (self.d + i)) & 1:
                    v ^= P << i
                    q |= 1 << i
            self.R[t] = clmul(P, q)

    def __call__(self, a):
        d = self.d
        while a.bit_length() > d + 8:
            top = a.bit_length() - 8
            t = a >> top
            a ^= self.R[t] << (top - d)
        return mod(a, self.P)


def xpow(J, P):
    r = 1
    for b in bin(J)[2:]:
        r = mod(sq(r), P)
        if b == "1":
            r = mod(r << 1, P)
    return r


def jump(win, g):
    r = [0] * N
    for i in range(g.bit_length() - 1, -1, -1):
        r = step(r)
        if (g >> i) & 1:
            r = [a ^ b for a, b in zip(r, win)]
    return r


def char_poly():
    rs = random.Random(20251016)
    win = list(rs.getstate()[1][:N])
    bits = []
    for _ in range(2 * DEG + 2):
        win = step(win)
        bits.append(win[0] & 1)
    C, L = berlekamp_massey(bits)
    assert L == DEG, L
    P = int(bin(C)[2:].zfill(L + 1)[::-1], 2)
    assert P.bit_length() - 1 == DEG
    return P


def jump_polys(P, l_words):
    """[(name, J, x^J mod P)] of the A, C, B rows for substreams of l_words, checked."""
    red = Reducer(P)
    mm = lambda x, y: red(clmul(x, y))  # noqa: E731
    xL = xpow(l_words, P)
    x64L = xpow(64 * l_words, P)
    x4096L = xpow(4096 * l_words, P)
    polys = []
    g = xpow(l_words - N, P)
    for a in range(RADIX):  # A_a = x^(L - 624 + 64 a L)
        polys.append((f"A{a}", l_words - N + 64 * a * l_words, g))
        g = mm(g, x64L)
    g = x4096L
    for c in range(1, RADIX):  # C_c = x^(4096 c L)
        polys.append((f"C{c}", 4096 * c * l_words, g))
        g = mm(g, x4096L)
    g = xL
    for b in range(1, RADIX):  # B_b = x^(b L)
        polys.append((f"B{b}", b * l_words, g))
        g = mm(g, xL)
    for name, J, gp in polys[::17]:  # products vs direct square-and-multiply
        assert gp == xpow(J, P), name
    # check the two smallest jumps (A_0, B_1) against plain stepping
    w0 = list(random.Random(5).getstate()[1][:N])
    for name, J, gp in (polys[0], polys[2 * RADIX - 1]):
        a = jump(w0, gp)
        b = w0
        for _ in range(J):
            b = step(b)
        assert a[1:] == b[1:] and (a[0] ^ b[0]) >> 31 == 0, name
    return polys


def write_polys(f, macro, polys):
    nw = (DEG + 1 + 63) // 64
    f.write(f"#define {macro} {{ \\\n")
    for name, J, gp in polys:
        f.write(f"  /* {name}: J = {J} */ {{ \\")
        ws = [(gp >> (64 * i)) & ((1 << 64) - 1) for i in range(nw)]
        for i, wv in enumerate(ws):
            if i % 6 == 0:
                f.write("\n   ")
            f.write(f" 0x{wv:016x}ull,")
            if i % 6 == 5 or i == nw - 1:
                f.write(" \\")
        f.write("\n  }, \\\n")
    f.write("}\n")


def main(out_path):
    P = char_poly()
    polys = jump_polys(P, L_WORDS)
    nw = (DEG + 1 + 63) // 64
    with open(out_path, "w") as f:
        f.write("// Generated by tools/gen_mt_jump.py — do not edit.\n")
        f.write("// MT19937 jump-ahead polynomials g(x) = x^J mod P(x), P = the characteristic\n")
        f.write("// polynomial of MT19937's one-word transition (degree 19937); bit i of word\n")
        f.write("// i/64 is the coefficient of x^i.\n")
        f.write(f"constexpr uint64_t kMtJumpL = {L_WORDS}ull;  // words per device substream\n")
        f.write(f"constexpr int kMtJumpRadix = {RADIX};\n")
        f.write(f"constexpr int kMtPolyWords = {nw};\n")
        f.write("// rows: A_a = x^(L - 624 + 64 a L) (a = 0..63) at row a; C_c = x^(4096 c L) (c = 1..63) at\n")
        f.write("// row 63 + c; B_b = x^(b L) (b = 1..63) at row 126 + b.\n")
        f.write("constexpr int kMtRowA = 0, kMtRowC = 63, kMtRowB = 126;\n")
        f.write(f"constexpr int kMtJumpRows = {len(polys)};\n")
        f.write("// initializer of a [kMtJumpRows][kMtPolyWords] uint64_t array (host and device copies)\n")
        write_polys(f, "DN_MT_JUMP_POLYS", polys)
    print("wrote", out_path)


def main_short(out_path):
    """The same rows for shorter substreams (17 * 2^10 and 17 * 2^12 words:
    2^10 / 2^12 whole draws), which the device draw uses for smaller vectors
    so that a substream's sequential generation does not dominate."""
    P = char_poly()
    with open(out_path, "w") as f:
        f.write("// Generated by tools/gen_mt_jump.py --short — do not edit.\n")
        f.write("// As mt19937_jump.inc (same rows A, C, B and layout) for substreams of\n")
        f.write("// L = 17 * 2^10 and 17 * 2^12 words.\n")
        for k in (10, 12):
            lw = 17 * (1 << k)
            f.write(f"constexpr uint64_t kMtJumpL{k} = {lw}ull;\n")
            write_polys(f, f"DN_MT_JUMP_POLYS_L{k}", jump_polys(P, lw))
    print("wrote", out_path)


def direct_polys(P, l_words, rows=RADIX):
    """D_s = x^(L - 624 + (s - 1) L), s = 1..rows: window s straight from W_idx
    (one jump level for draws of at most rows + 1 substreams), checked."""
    red = Reducer(P)
    xL = xpow(l_words, P)
    g = xpow(l_words - N, P)
    polys = []
    for s in range(1, rows + 1):
        polys.append((f"D{s}", l_words - N + (s - 1) * l_words, g))
        g = red(clmul(g, xL))
    for name, J, gp in polys[::17] + polys[-1:]:
        assert gp == xpow(J, P), name
    w0 = list(random.Random(7).getstate()[1][:N])
    for name, J, gp in polys[:2]:  # the two smallest against plain stepping
        a = jump(w0, gp)
        b = w0
        for _ in range(J):
            b = step(b)
        assert a[1:] == b[1:] and (a[0] ^ b[0]) >> 31 == 0, name
    return polys


def main_direct(out_path):
    """Direct rows D_1..D_64 for the four substream lengths of the device draw
    (17 * 2^k words, k = 10, 12, 14 and 8, in the device's table order): a
    draw of S <= 65 substreams reaches every window in ONE jump level."""
    P = char_poly()
    with open(out_path, "w") as f:
        f.write("// Generated by tools/gen_mt_jump.py --direct — do not edit.\n")
        f.write("// Direct jump rows D_s = x^(L - 624 + (s - 1) L) mod P, s = 1..64 (row s - 1):\n")
        f.write("// W(s) = D_s(W_idx), for substreams of L = 17 * 2^k words, k = 10, 12, 14, 8.\n")
        f.write("constexpr int kMtDirectRows = 64;\n")
        f.write("constexpr uint64_t kMtJumpL8 = 4352ull;\n")
        for k in (10, 12, 14, 8):
            write_polys(f, f"DN_MT_JUMP_DIRECT_L{k}", direct_polys(P, 17 * (1 << k)))
    print("wrote", out_path)


def main_charpoly(out_path):
    """P itself (degree 19937, 312 words): the device draw's host side
    multiplies tabulated rows mod P at run time (runtime direct rows,
    mt19937_device.hip)."""
    P = char_poly()
    nw = (DEG + 1 + 63) // 64
    assert P.bit_length() - 1 == DEG
    # x^L mod P from P agrees with the tabulated B_1 for L = 17 * 2^14
    assert xpow(L_WORDS, P) == jump_polys(P, L_WORDS)[2 * RADIX - 1][2]
    with open(out_path, "w") as f:
        f.write("// Generated by tools/gen_mt_jump.py --charpoly — do not edit.\n")
        f.write("// P, the characteristic polynomial of MT19937's one-word transition\n")
        f.write("// (degree 19937; bit i of word i/64 is the coefficient of x^i).\n")
        write_polys(f, "DN_MT_CHAR_POLY", [("P", 0, P)])
    print("wrote", out_path)


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "delta-node_amd", "csrc")
    if len(sys.argv) > 1 and sys.argv[1] == "--charpoly":
        main_charpoly(sys.argv[2] if len(sys.argv) > 2 else os.path.join(csrc, "mt19937_charpoly.inc"))
    elif len(sys.argv) > 1 and sys.argv[1] == "--direct":
        main_direct(sys.argv[2] if len(sys.argv) > 2 else os.path.join(csrc, "mt19937_jump_direct.inc"))
    elif len(sys.argv) > 1 and sys.argv[1] == "--short":
        main_short(sys.argv[2] if len(sys.argv) > 2 else os.path.join(csrc, "mt19937_jump_short.inc"))
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(csrc, "mt19937_jump.inc"))
