"""BASELINE config 5 plumbing at a small size: a masked-result round from this
process (pack -> H2D -> split -> encode -> D2H -> HTTP) to a second local
process over loopback, which decodes shares 1, 3, 5 on its own HIP context,
reconstructs and checks the digest of the secrets (scripts/e2e_round.py)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _e2e():
    spec = importlib.util.spec_from_file_location("e2e_round", os.path.join(ROOT, "scripts", "e2e_round.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.gpu
@pytest.mark.parametrize("coeffs,seal", [("prng", False), ("mt", False), ("prng", True)])
def test_masked_result_round_over_loopback(coeffs, seal):
    """seal: every body travels as the receiver's AES envelope in JSON form
    ("0x" + hex(base64(nonce || AES-256-CTR))) and the peer opens it on its GPU."""
    e2e = _e2e()
    port = 18000 + os.getpid() % 1000 + (0 if coeffs == "prng" else 1000) + (2000 if seal else 0)
    proc = e2e.start_peer(port)
    try:
        e2e._wait_ready(port)
        st = e2e.run_round((1 << 14) + 77, port, coeffs=coeffs, seed=5, seal=seal)
    finally:
        e2e.stop_peer(proc, port)
    assert st["peer_verified"]
    assert st["bytes_posted"] > 5 * 66 * (1 << 14) * (2.6 if seal else 1)


@pytest.mark.gpu
def test_masked_result_round_full_size():
    """BASELINE config 5 at its own size: 2^24 int64 elements, MT19937
    coefficients in the reference's order (make_shares_vec, the drop-in path),
    every share vector posted to the peer, which reconstructs from shares 1, 3,
    5 and verifies the digest of the secrets."""
    e2e = _e2e()
    port = 21000 + os.getpid() % 1000
    proc = e2e.start_peer(port)
    try:
        e2e._wait_ready(port)
        st = e2e.run_round(1 << 24, port, coeffs="mt", seed=7, seal=False)
    finally:
        e2e.stop_peer(proc, port)
    assert st["peer_verified"]
    assert st["bytes_posted"] > 5 * 66 * (1 << 24)
