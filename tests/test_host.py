"""Host-side logic and the C-ABI boundary, on CPU (no kernel launches).

* the library loads and exports every symbol include/dn_shamir.h declares;
* the native MT19937 coefficient stream equals the reference's draws;
* the Lagrange descriptors equal the reference's weights (as field values);
* the tiled layout round-trips; the byte codec matches the reference's shares;
* the reference's argument errors fire before any device work, and a device
  call without a HIP device raises (no CPU fallback).
"""
import glob
import os
import random
import re

import numpy as np
import pytest
import torch

from delta_node import serialize
from delta_node.crypto import shamir
from delta_node.crypto.shamir import _native, field, op
from delta_node.crypto.shamir import shamir as shamir_mod
from golden.fixtures import P, load_json, load_npz, manifest
from oracle.py_shamir import RefSecretShare

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))


def header_symbols():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w ]+?\*?\s*\b(dn_\w+)\s*\(", text, re.M)))


def test_library_exports_header_symbols():
    from delta_node.crypto import aes
    from delta_node.crypto.shamir import codec
    from delta_node.utils import _mask_native, mimc7

    syms = header_symbols()
    assert len(syms) >= 21
    L = _native.lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_native.EXPORTS + _mask_native.EXPORTS + codec.EXPORTS + mimc7.EXPORTS + aes.EXPORTS) == syms


def _mt_step_window(w: np.ndarray, n: int) -> np.ndarray:
    """The 624-word MT window advanced n words (word 624 + i = mix(i, i + 1, i + 397))."""
    s = [int(x) for x in w]
    for i in range(n):
        y = (s[i] & 0x80000000) | (s[i + 1] & 0x7FFFFFFF)
        s.append(s[i + 397] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0))
    return np.array(s[n:n + 624], dtype=np.uint32)


@pytest.mark.parametrize("words", [1, 700, 5000, 17 * 16384 - 624])
def test_jump_polynomial_advances_the_window(words):
    """dn_mt19937_jump_poly(words) = x^words mod P: applied to a window by
    Horner (r <- f(r) ^ g_i W from the top coefficient down, f = one word of
    the transition) it gives the window stepped `words` words — the jump the
    speculated next draw starts from (DN_MT_SPEC beside the generation)."""
    g = _native.mt_jump_poly(words)
    bits = np.unpackbits(g.view(np.uint8), bitorder="little")[:19937]
    rng = np.random.default_rng(words)
    w = rng.integers(0, 1 << 32, 624, dtype=np.uint64).astype(np.uint32)
    top = int(np.nonzero(bits)[0].max())
    r = [0] * 624
    wl = [int(x) for x in w]
    for i in range(top, -1, -1):
        y = (r[0] & 0x80000000) | (r[1] & 0x7FFFFFFF)
        r = r[1:] + [r[397] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)]
        if bits[i]:
            r = [a ^ b for a, b in zip(r, wl)]
    assert np.array_equal(np.array(r, dtype=np.uint32), _mt_step_window(w, words))


def test_embedded_mt_jump_rows_pass_their_checks():
    """The build-time table of 2048 direct jump rows (csrc/gen_mt_rt_rows.cpp,
    embedded by csrc/mt_rt_rows14.S) carries its generator's checksum and
    passes it, the 64 tabulated rows and the recurrence at first use
    (csrc/host_gf2poly.cpp): a first 2^24 draw does not recompute it."""
    assert _native.lib().dn_mt19937_rt_rows_embedded() == 1
    blob = os.path.join(ROOT, "delta-node_amd", "lib", "mt_rt_rows14.bin")
    assert os.path.getsize(blob) == 8 * (2048 * 312 + 2)


def test_version_and_sizes():
    assert "gfx950" in _native.version()
    for n in (0, 1, 255, 256, 257, 1 << 20, (1 << 24) + 3):
        assert _native.vec_bytes(n) == field.vec_bytes(n) == 66 * 256 * ((n + 255) // 256)


def test_field_layout_roundtrip():
    rng = random.Random(3)
    vals = [rng.randrange(P) for _ in range(700)] + [0, 1, P - 1]
    vec = field.ints_to_vec(vals)
    assert vec.size == field.vec_bytes(len(vals))
    assert field.vec_to_ints(vec, len(vals)) == vals
    planes = field.vec_to_planes(vec, len(vals))
    assert field.limbs_to_ints(planes.T.copy()) == vals
    # tile structure: element 300 is element 44 of tile 1, limb 3 at lo[3][44]
    t = vec[field.TILE_BYTES:2 * field.TILE_BYTES]
    lo = t[:64 * 256].view("<u4").reshape(16, 256)
    assert lo[3, 44] == (vals[300] >> 96) & 0xFFFFFFFF
    assert t[64 * 256:].view("<u2")[44] == vals[300] >> 512


@pytest.mark.parametrize("key", ["f1", "f2"])
def test_native_mt_coefficients_match_reference(key):
    cfg = manifest()[key]
    z = load_npz(cfg["file"])
    r = random.Random(cfg["mt_seed"])
    block = _native.mt_draw_coeffs(r, cfg["N"], cfg["t"] - 1)
    got = np.stack([field.vec_to_limbs(block[j], cfg["N"]) for j in range(cfg["t"] - 1)], axis=1)
    assert np.array_equal(got, z["coeff_limbs"])
    # the Random object advanced exactly as the reference's calls advanced it
    r2 = random.Random(cfg["mt_seed"])
    for _ in range(cfg["N"] * (cfg["t"] - 1)):
        r2.randint(1, P - 1)
    assert r.getstate() == r2.getstate()
    assert r.getrandbits(64) == r2.getrandbits(64)


def test_native_mt_mid_stream_and_rejection_free_path():
    r = random.Random(77)
    r.getrandbits(32 * 100)  # start mid-buffer (index != 624)
    r.random()
    ref = random.Random()
    ref.setstate(r.getstate())
    block = _native.mt_draw_coeffs(r, 300, 2)
    want = [ref.randint(1, P - 1) for _ in range(600)]
    got = [field.vec_to_ints(block[j], 300) for j in range(2)]
    assert [got[j][e] for e in range(300) for j in range(2)] == want
    assert r.getstate() == ref.getstate()


def _lam_ref(xs):
    k = len(xs)
    out = []
    for i in range(k):
        num, den = 1, 1
        for j in range(k):
            if j != i:
                num *= -xs[j]
                den *= xs[i] - xs[j]
        out.append(op.div_mod(num % P, den, P))
    return out


def _lam_from_desc(w):
    lams = []
    k = w.k
    scale = 1
    if w.has_inv == 1:
        scale = sum(w.inv[j] << (32 * j) for j in range(17))
    elif w.has_inv == 2:
        d = w.d
        assert d % 2 == 1 and 3 <= d < 65536
        assert (w.d_inv32 * d) % 2**32 == 1 and (w.p_inv_d * P) % d == 1
        assert w.d_recip == (2**64 - 1) // d
        assert [w.w[i] for i in range(17)] == [pow(2, 32 * i, d) for i in range(17)]
        scale = op.inverse_mod(d, P)
    scale = scale * op.inverse_mod(pow(2, w.shift, P), P) % P
    for i in range(k):
        a = sum(w.a[i][j] << (32 * j) for j in range(w.a_limbs))
        if (w.neg >> i) & 1:
            a = -a
        lams.append(a * scale % P)
    return lams


@pytest.mark.parametrize("xs", [
    [1, 2, 3], [1, 3, 5], [2, 4, 5], [3, 4, 5], [5, 1, 3], [1, 2, 4, 5], [1, 2, 3, 4, 5], [1, 3, 5, 7, 9],
    [2, 3, 5, 8, 9], [7, 100, 255], [1, 256, 1000], [2, 3], list(range(1, 10)), list(range(1, 17)),
    [17, 33, 65, 129, 200, 250], [0, 5, 9], [1, 2**40, 2**63 + 7], [65535, 1, 300, 4096],
    list(range(100, 116)), [2**64 - 1, 2**64 - 2, 3],
])
def test_lagrange_descriptor_equals_reference_weights(xs):
    w = _native.lagrange(xs, 0)
    assert w.k == len(xs) and w.a_limbs in (1, 2, 17) and 0 <= w.shift < 32
    assert _lam_from_desc(w) == _lam_ref(xs)


def test_lagrange_fast_forms():
    w = _native.lagrange([1, 2, 3], 3)  # 3, -3, 1
    assert (w.a_limbs, w.has_inv, w.shift, w.neg) == (1, 0, 0, 0b010)
    w = _native.lagrange([1, 3, 5], 3)  # (15, -10, 3) / 8
    assert (w.a_limbs, w.has_inv, w.shift) == (1, 0, 3)
    w = _native.lagrange([2, 4, 5], 3)  # (10, -15, 8) / 3: exact division by 3
    assert (w.a_limbs, w.has_inv, w.shift, w.d) == (1, 2, 0, 3)


def test_lagrange_full_inverse_form(monkeypatch):
    """The full-width inverse form (tuning build, DN_EXACT_DIV=0) describes the
    same weights as the reference's."""
    monkeypatch.setenv("DN_EXACT_DIV", "0")
    with _native.library(_native.TUNING_LIB):
        for xs in ([2, 4, 5], [1, 2, 4, 5], [7, 100, 255], [2, 3, 5, 8, 9]):
            w = _native.lagrange(xs, 0)
            assert w.has_inv in (0, 1)
            assert _lam_from_desc(w) == _lam_ref(xs)


def test_product_library_reads_no_environment(monkeypatch):
    """The product library consults no DN_* knob (they exist only in the
    tuning build): it imports no getenv, and a set knob changes nothing."""
    import shutil
    import subprocess

    if shutil.which("nm"):
        und = subprocess.run(["nm", "-D", "--undefined-only", _native.lib_path()], capture_output=True, text=True,
                             check=True).stdout
        assert "getenv" not in und and "secure_getenv" not in und
        und_t = subprocess.run(["nm", "-D", "--undefined-only", _native.TUNING_LIB], capture_output=True, text=True,
                               check=True).stdout
        assert "getenv" in und_t
    want = _native.lagrange([2, 4, 5], 3)
    for k, v in (("DN_EXACT_DIV", "0"), ("DN_GRID_CAP", "7"), ("DN_TILE_MAP", "3"), ("DN_SPLIT_E", "4")):
        monkeypatch.setenv(k, v)
    got = _native.lagrange([2, 4, 5], 3)
    assert (got.has_inv, got.d, got.shift) == (want.has_inv, want.d, want.shift) == (2, 3, 0)
    with _native.library(_native.TUNING_LIB):
        assert _native.lagrange([2, 4, 5], 3).has_inv in (0, 1)  # the knob works where it exists


def test_lagrange_errors_mirror_reference():
    with pytest.raises(ValueError, match="need at least 3 shares"):
        _native.lagrange([1, 2], 3)
    with pytest.raises(ValueError, match="shares must be distinct"):
        _native.lagrange([1, 2, 1], 2)
    with pytest.raises(TypeError, match="reduce"):
        _native.lagrange([4], 1)
    with pytest.raises(NotImplementedError):
        _native.lagrange(list(range(1, 18)), 2)


def test_share_codec_matches_reference_bytes():
    f3 = load_json("f3_edge.json")
    for case in f3["cases"][:40]:
        for x, hx in enumerate(case["shares"], start=1):
            b = bytes.fromhex(hx)
            xx, y = shamir_mod._bytes_to_share(b)
            assert xx == x
            assert shamir_mod._share_to_bytes((xx, y)) == b


def test_serialize_and_op_mirror():
    for v in (0, 1, 255, 256, P, 2**64 - 1):
        assert serialize.int_to_bytes(v) == v.to_bytes((v.bit_length() + 7) // 8, "big")
        assert serialize.bytes_to_int(serialize.int_to_bytes(v)) == v
    # the reference's own cases (tests/serialize/hex_test.py:3-7)
    assert serialize.bytes_to_hex(bytes([255])) == "0xff"
    assert serialize.bytes_to_hex(bytes([255]), with0x=False) == "ff"
    assert serialize.bytes_to_hex(bytes([255]), length=2) == "0x00ff"
    assert serialize.bytes_to_hex(b"\x01\x02", length=4) == "0x00000102"
    assert serialize.hex_to_bytes("0x0102", length=3) == b"\x00\x01\x02"
    assert op.inverse_mod(3, P) * 3 % P == 1
    assert op.inverse_mod(-1, P) == P - 1
    with pytest.raises(ZeroDivisionError):
        op.inverse_mod(0, P)
    assert op.div_mod(10, 5, P) == 2


def test_surface_and_errors_before_device():
    assert shamir_mod.__all__ == ["Share", "PRIME", "SecretShare"]
    assert shamir.Share is shamir_mod.Share and shamir.SecretShare is shamir_mod.SecretShare
    assert shamir.PRIME == P
    ss = shamir.SecretShare(4)
    assert ss.threshold == 4 and ss.prime == P and isinstance(ss.random, random.Random)
    with pytest.raises(ValueError, match="threshold should be little equal than shares"):
        ss.make_shares(b"\x01", 3)
    sh = RefSecretShare(4).make_shares(b"\x05", 6)
    with pytest.raises(ValueError, match="need at least 4 shares"):
        ss.resolve_shares(sh[:3])
    with pytest.raises(ValueError, match="shares must be distinct"):
        ss.resolve_shares([sh[0], sh[1], sh[2], sh[1]])
    with pytest.raises(ValueError, match="not enough values to unpack"):
        ss.resolve_shares([])
    with pytest.raises(TypeError):
        shamir.SecretShare(1).resolve_shares(sh[:1])
    ss127 = shamir.SecretShare(3, prime=2**127 - 1)  # the byte API takes any prime (host path)
    assert ss127.resolve_shares(ss127.make_shares(b"\x01\x02", 4)[1:]) == b"\x01\x02"
    with pytest.raises(NotImplementedError):  # the vector (GPU) path is M521 only
        ss127.make_shares_vec(torch.arange(4, dtype=torch.int64), 4)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device failure mode")
def test_no_cpu_fallback():
    """The vector path needs the GPU (no CPU fallback); the byte API is the
    library's native host path by design (one secret per call)."""
    ss = shamir.SecretShare(2)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ss.make_shares_vec(torch.arange(10, dtype=torch.int64), 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ss.resolve_shares_vec([torch.zeros(66 * 256, dtype=torch.uint8)] * 2, [1, 2], 10)
    assert ss.resolve_shares(ss.make_shares(b"\x07", 3)[:2]) == b"\x07"


@pytest.mark.parametrize("start_words", [0, 5, 623, 624, 1000])
def test_mt19937_skip_matches_cpython(start_words):
    """dn_mt19937_skip (jump-ahead: Horner of x^J mod P on the 624-word window,
    polynomials from tools/gen_mt_jump.py) lands on exactly the state CPython
    reaches by generating the words — across the head of the current array,
    block boundaries, the first-digit windows (A_0, B_b) and the second digit
    (A_a, a >= 1: 64 L words and more) of the 17*2^14-word jump units."""
    L = 17 * (1 << 14)
    for words in (0, 1, 17, 600, 624, 625, 5000, L - 1, L, L + 624, 3 * L + 12345, 7 * L + 1, 14 * L + 9,
                  64 * L + 700, 70 * L + 3, 200 * L + 5):
        a = random.Random(99)
        a.getrandbits(32 * start_words) if start_words else None
        b = random.Random()
        b.setstate(a.getstate())
        _native.mt_skip(a, words)
        left = words
        while left:
            take = min(left, 1 << 20)
            b.getrandbits(32 * take)
            left -= take
        assert a.getstate() == b.getstate(), words
        assert a.getrandbits(64) == b.getrandbits(64)


def test_mt19937_skip_third_digit_composes():
    """Skips past 4097 jump units use the third radix-64 digit (C_c): one skip
    equals the same distance in two skips that stay below it, from two start
    indices; and it is additive across the C/A/B digit boundaries."""
    L = 17 * (1 << 14)
    for start in (0, 311):
        for total, first in ((4097 * L + 17, 2000 * L + 8), (9000 * L + 5, 4095 * L + 623), (4160 * L, 64 * L)):
            a = random.Random(7)
            a.getrandbits(32 * start) if start else None
            b = random.Random()
            b.setstate(a.getstate())
            _native.mt_skip(a, total)
            _native.mt_skip(b, first)
            _native.mt_skip(b, total - first)
            assert a.getstate() == b.getstate(), (start, total, first)


def test_mt_jump_job_builder_invariants(tmp_path):
    """The device MT draw's jump-job builder (host code in
    csrc/mt19937_device.hip), compiled for the host by tools/mt_levels_check.hip:
    every substream window produced exactly once, sources ready before their
    level, one table per workgroup, part rows in bounds and covering the
    polynomial in order — S up to 300 and boundary sizes to 65537, all three
    substream lengths."""
    import shutil
    import subprocess

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "mt_levels_check")
    subprocess.run([hipcc, "-O1", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(root, "include"),
                    "-I" + os.path.join(root, "delta-node_amd", "csrc"),
                    os.path.join(root, "tools", "mt_levels_check.hip"), "-o", exe], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "fails 0" in r.stdout


def test_mt_state_in_place_matches_getstate():
    """The device MT draws update the caller's random.Random in place when
    this interpreter's layout checks out (_native._mt_layout): the pointers
    read exactly getstate()'s 624 words and index, a write through them is what
    getstate() then returns, and a random.Random subclass (the reference's
    SecretShare.random is one instance of the class) has the same offsets."""
    if not _native._mt_layout():
        pytest.skip("this interpreter's _random layout is not the checked one: the marshal path serves it")

    class Sub(random.Random):
        pass

    for rng in (random.Random(11), Sub(12)):
        rng.getrandbits(32 * 333)
        state, index = _native._mt_inplace(rng)
        words = rng.getstate()[1]
        assert [state[i] for i in range(624)] == list(words[:624]) and index[0] == words[624]
        want = random.Random()
        want.setstate(rng.getstate())
        state[100] ^= 0xDEADBEEF
        index[0] = 5
        st = list(want.getstate()[1])
        st[100] ^= 0xDEADBEEF
        st[624] = 5
        assert list(rng.getstate()[1]) == st
    assert _native._mt_inplace(object()) is None


def test_mt_marshal_path_matches_in_place(monkeypatch):
    """With the in-place layout unavailable (another interpreter build), the
    host draw marshals through getstate / setstate and ends in the same state
    with the same coefficients as the in-place path."""
    a, b = random.Random(5), random.Random(5)
    want = _native.mt_draw_coeffs(a, 300, 2)
    monkeypatch.setattr(_native, "_MT_LAYOUT", False)
    assert _native._mt_inplace(b) is None
    got = _native.mt_draw_coeffs(b, 300, 2)
    assert np.array_equal(got, want) and a.getstate() == b.getstate()


def test_mt_paths_only_for_plain_mt19937():
    """The MT fast paths (jump-ahead, the state read in place) serve only a
    random.Random whose draw methods are CPython's: SystemRandom (os.urandom)
    and subclasses overriding randint / getrandbits / random are not MT19937
    draws, so the vector API calls them per coefficient as the reference does
    (shamir.py:59-61) — never reads their unused internal MT array."""
    class Plain(random.Random):
        pass

    class Rec(random.Random):
        def randint(self, a, b):
            return 7

    class Bits(random.Random):
        def getrandbits(self, k):
            return 3

    assert _native.mt_compatible(random.Random(1)) and _native.mt_compatible(Plain(1))
    for rng in (random.SystemRandom(), Rec(1), Bits(1), object()):
        assert not _native.mt_compatible(rng)
        assert _native._mt_inplace(rng) is None
    # the generic draw is the reference's own per-coefficient call sequence
    ss = shamir.SecretShare(3)
    ss.random = Rec(1)
    blk = shamir_mod._draw_coeffs_generic(ss.random, 5, 2)
    assert [field.vec_to_ints(blk[j], 5) for j in range(2)] == [[7] * 5, [7] * 5]
    r = random.Random(42)
    blk = shamir_mod._draw_coeffs_generic(Plain(42), 4, 2)
    want = [[r.randint(1, P - 1) for _ in range(2)] for _ in range(4)]
    assert [field.vec_to_ints(blk[j], 4) for j in range(2)] == [[w[j] for w in want] for j in range(2)]
    ss.random = random.SystemRandom()
    with pytest.raises(NotImplementedError, match="sharded draw needs a plain random.Random"):
        ss.draw_coeffs_vec(4, torch.device("cpu"), elem_offset=1, n_total=8)


@pytest.mark.parametrize("coeffs,x,prime", [
    ([5, 3, 2], 4, 101),                         # small prime
    ([5, 3, 2], 0, P),                           # x = 0
    ([123456789, 987654321, 5], 70000, P),       # x beyond the device range
    (list(range(1, 101)), 7, P),                 # 100 coefficients
    ([P + 5, -3, 2 * P - 1], 70001, P),          # unreduced and negative coefficients
    ([10, -4, 7], -3, 2**127 - 1),               # negative x
    ([10, 4, 7], 5, -13),                        # negative modulus (Python's sign of the divisor)
    ([1 << 600, 3], 1 << 70, 2**61 - 1),         # wide operands
    ([0, 0, 0], 12, 97),
])
def test_eval_at_any_integers_matches_reference_loop(coeffs, x, prime):
    """_eval_at (shamir.py:19-25) outside the device split's range runs the
    library's host Horner (dn_shamir_eval_at_host), equal to the reference's
    Python loop for any integers (checked against oracle/py_shamir.eval_at's
    restatement of that loop)."""
    from oracle.py_shamir import eval_at as ref_eval_at

    want = 0
    for c in coeffs[::-1]:
        want = (want * x + c) % prime
    assert shamir_mod._eval_at(coeffs, x, prime) == want
    if prime > 0:
        assert ref_eval_at(coeffs, x, prime) == want


def test_eval_at_edges():
    assert shamir_mod._eval_at([], 5, 97) == 0
    with pytest.raises(ZeroDivisionError):
        shamir_mod._eval_at([1, 2], 3, 0)
