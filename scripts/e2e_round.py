#!/usr/bin/env python3
"""End-to-end masked-result round between two local delta-node processes
(BASELINE config 5): wall-clock from "pack" to the peer's last HTTP 200.

Runner side (this process), for a masked result {'w': {'w': int64[N]}}:
  pack    serialize.dump_agg_result as the reference does it (cloudpickle of
          the result dict; delta_node/serialize/agg.py:11 -> obj.py:10)
  H2D     the int64 array, pinned staging
  split   t-of-n Shamir split on the GPU (device ChaCha coefficients by
          default, `--coeffs mt` for the drop-in MT19937 draw on the host)
  encode  each share vector -> the reference's `_share_to_bytes` records
          (shamir.py:28-33) on the GPU, plus a uint8 record-length vector
  D2H     records + lengths into pinned host buffers
  seal    (--seal) each share's body sealed for its receiver as the reference
          sends shares: "0x" + hex(base64(nonce || AES-256-CTR(key, body)))
          (crypto/aes/aes.py:8-14 + serialize.bytes_to_hex,
          runner/horizontal/commu.py:23-49), on the GPU
  HTTP    one POST per share x to the peer (octet-stream), each share on its
          own keep-alive connection and sender thread, overlapped with the
          next share's encode + D2H
Peer side (`--serve`, a second process with its own HIP context): stores the
bodies; after the timed round it decodes the records of shares xs (GPU),
reconstructs and checks the xxh64 digest of the secrets the runner sent.

MB/s = 8 N bytes of int64 input / wall-clock.  One JSON line per round.
"""
from __future__ import annotations

import argparse
import http.client
import http.server
import json
import os
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "delta-node_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# ----------------------------------------------------------------- peer side
class _Peer(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    store: dict = {}
    bufs: dict = {}

    def log_message(self, *a):  # quiet
        pass

    def _reply(self, obj, code=200):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _body(self, slot=None):
        """Read the request body into a buffer that is not zero-filled first
        (np.empty), reused per share slot across rounds."""
        import numpy as np

        n = int(self.headers["Content-Length"])
        buf = self.bufs.get(slot) if slot is not None else None
        if buf is None or buf.size < n:
            buf = np.empty(n, dtype=np.uint8)
            if slot is not None:
                self.bufs[slot] = buf
        buf = buf[:n]
        view = memoryview(buf)
        got = 0
        while got < n:
            r = self.rfile.readinto(view[got:])
            if not r:
                raise ConnectionError("short body")
            got += r
        return buf

    def do_GET(self):
        if self.path == "/ping":
            return self._reply({"ok": True})
        return self._reply({"error": "not found"}, 404)

    def do_POST(self):
        if self.path.startswith("/secret_shares/"):
            x = int(self.path.rsplit("/", 1)[1])
            body = self._body(slot=x)
            self.store[x] = (body, int(self.headers["X-Records-Bytes"]), int(self.headers["X-Elements"]),
                             self.headers.get("X-Sealed") == "1")
            return self._reply({"x": x, "bytes": len(body)})
        if self.path == "/verify":
            req = json.loads(bytes(self._body()))
            return self._reply(_verify(self.store, req))
        if self.path == "/shutdown":
            self._reply({"ok": True})
            threading.Thread(target=self.server.shutdown, daemon=True).start()
            return None
        return self._reply({"error": "not found"}, 404)


def _verify(store: dict, req: dict) -> dict:
    """Decode the stored records of shares xs on the GPU, reconstruct, digest."""
    import numpy as np
    import torch
    import xxhash

    from delta_node.crypto import aes, shamir
    from delta_node.crypto.shamir import codec

    n, xs, t = int(req["n"]), [int(x) for x in req["xs"]], int(req["t"])
    keys = [bytes.fromhex(k) for k in req.get("keys", [])]
    dev = torch.device("cuda", 0)
    vecs = []
    for x in xs:
        body, rec_bytes, n_el, sealed = store[x]
        assert n_el == n
        if sealed:  # the receiver's side: hex_to_bytes + aes.decrypt (runner/horizontal/agg.py:258-266)
            raw = aes.decrypt_vec(keys[x - 1], torch.from_numpy(body).to(dev), hex=True)
        else:
            raw = torch.from_numpy(body)
        packed = raw[:rec_bytes].to(dev)
        lens = raw[rec_bytes:rec_bytes + n].to(dev).to(torch.int64)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=offsets[1:])
        vec, xv = codec.decode_share_vec(packed, offsets, n)
        if not bool((xv == x).all()):
            return {"ok": False, "why": f"share {x}: wrong abscissa in records"}
        vecs.append(vec)
    rec = shamir.SecretShare(t).resolve_shares_vec(vecs, xs, n)
    digest = xxhash.xxh64(rec.cpu().numpy().view(np.uint8)).hexdigest()
    return {"ok": digest == req["digest"], "digest": digest}


def serve(port: int) -> None:
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", port), _Peer)
    print(json.dumps({"serving": port}), flush=True)
    srv.serve_forever()


# --------------------------------------------------------------- runner side
def _wait_ready(port: int, timeout: float = 180.0) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
            c.request("GET", "/ping")
            if c.getresponse().status == 200:
                c.close()
                return
        except OSError:
            time.sleep(0.2)
    raise RuntimeError("peer did not come up")


def _post(conn: http.client.HTTPConnection, path: str, body, headers=None) -> dict:
    h = {"Content-Type": "application/octet-stream", "Content-Length": str(len(body))}
    h.update(headers or {})
    conn.request("POST", path, body=body, headers=h)
    r = conn.getresponse()
    data = r.read()
    if r.status != 200:
        raise RuntimeError(f"{path}: HTTP {r.status} {data[:200]!r}")
    return json.loads(data)


def run_round(n_elem: int, port: int, t: int = 3, n_shares: int = 5, coeffs: str = "prng",
              verify_xs=(1, 3, 5), seed: int = 0, seal: bool = False) -> dict:
    """One timed round; returns the stage timings and the peer's verification.
    seal: each body goes out as the receiver's AES envelope in JSON form."""
    import cloudpickle
    import numpy as np
    import torch
    import xxhash

    from delta_node.crypto import aes, shamir
    from delta_node.crypto.shamir import codec

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(seed)
    arr = rng.integers(0, 1 << 62, size=n_elem, dtype=np.int64)  # a masked result (fixed point + masks)
    result = {"w": {"w": arr}}
    ss = shamir.SecretShare(t)
    ss.random.seed(seed)
    # pinned staging, allocated once per runner (untimed)
    sec_pin = torch.empty(n_elem, dtype=torch.int64, pin_memory=True)
    cap = int(codec._lib().dn_m521_encoded_capacity(n_elem, n_shares))
    body_cap = cap + n_elem
    if seal:  # "0x" + hex(base64(nonce || body)); per-receiver keys (the runner's ECDH keys in the reference)
        body_cap = 2 + int(aes.aes._lib().dn_aes_encrypt_len(cap + n_elem, 1))
        keys = [np.random.default_rng([seed, x]).bytes(32) for x in range(1, n_shares + 1)]
    stage = [torch.empty(body_cap, dtype=torch.uint8, pin_memory=True) for _ in range(n_shares)]
    copy_stream = torch.cuda.Stream()
    conns = [http.client.HTTPConnection("127.0.0.1", port, timeout=600) for _ in range(n_shares)]
    pool = ThreadPoolExecutor(n_shares)
    torch.cuda.synchronize()

    st = {}
    t0 = time.perf_counter()
    packed_obj = cloudpickle.dumps(result)  # reference: serialize.dump_agg_result
    st["pack_s"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    src = result["w"]["w"]
    sec_pin.numpy()[:] = src
    dsec = sec_pin.to(dev, non_blocking=True)
    torch.cuda.synchronize()
    st["h2d_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    if coeffs == "mt":
        shares = ss.make_shares_vec(dsec, n_shares)
    else:
        shares, _key = ss.make_shares_vec_prng(dsec, n_shares)
    torch.cuda.synchronize()
    st["split_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    pending = []
    enc_s = 0.0
    for x in range(1, n_shares + 1):
        buf = stage[x - 1]
        te = time.perf_counter()
        recs, offs = codec.encode_share_vec(shares[x - 1], n_elem, x)
        lens = (offs[1:] - offs[:-1]).to(torch.uint8)
        nb = recs.numel()
        if seal:
            plain = torch.empty(nb + n_elem, dtype=torch.uint8, device=dev)
            plain[:nb].copy_(recs)
            plain[nb:].copy_(lens)
            text = aes.encrypt_vec(keys[x - 1], plain, hex=True)
            parts, size = [(0, text)], text.numel()
        else:
            parts, size = [(0, recs), (nb, lens)], nb + n_elem
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_stream(torch.cuda.current_stream())
            for off, part in parts:
                buf[off:off + part.numel()].copy_(part, non_blocking=True)
        copy_stream.synchronize()
        enc_s += time.perf_counter() - te
        body = memoryview(buf.numpy())[:size]
        pending.append(pool.submit(_post, conns[x - 1], f"/secret_shares/{x}", body,
                                   {"X-Records-Bytes": str(nb), "X-Elements": str(n_elem),
                                    "X-Sealed": "1" if seal else "0"}))
    replies = [p.result() for p in pending]
    wall = time.perf_counter() - t0
    st["encode_d2h_s"] = enc_s
    st["post_tail_s"] = time.perf_counter() - t1 - enc_s
    st["wall_s"] = wall
    st["bytes_posted"] = int(sum(r["bytes"] for r in replies))
    st["packed_bytes"] = len(packed_obj)
    st["input_MBps"] = 8 * n_elem / wall / 1e6
    st["elems_per_s"] = n_elem / wall
    st["http_GBps"] = st["bytes_posted"] / wall / 1e9
    digest = xxhash.xxh64(src.view(np.uint8)).hexdigest()
    req = {"n": n_elem, "xs": list(verify_xs), "t": t, "digest": digest}
    if seal:
        req["keys"] = [k.hex() for k in keys]
    ver = _post(conns[0], "/verify", json.dumps(req).encode())
    st["peer_verified"] = bool(ver.get("ok"))
    for c in conns:
        c.close()
    pool.shutdown()
    return st


def start_peer(port: int) -> subprocess.Popen:
    return subprocess.Popen([sys.executable, os.path.abspath(__file__), "--serve", str(port)],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def stop_peer(proc: subprocess.Popen, port: int) -> None:
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        c.request("POST", "/shutdown", body=b"", headers={"Content-Length": "0"})
        c.getresponse().read()
    except OSError:
        pass
    try:
        proc.wait(timeout=30)
    except subprocess.TimeoutExpired:
        proc.kill()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--serve", type=int, default=0, help="run the peer on this port")
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--port", type=int, default=18931)
    ap.add_argument("--coeffs", choices=("prng", "mt"), default="prng")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seal", action="store_true", help="send each body as the receiver's AES envelope (JSON form)")
    ap.add_argument("--cold", action="store_true", help="no warm-up round: the first round of a fresh runner "
                    "and peer (the peer is up and listening, nothing else)")
    args = ap.parse_args()
    if args.serve:
        serve(args.serve)
        return 0
    proc = start_peer(args.port)
    try:
        _wait_ready(args.port)
        if not args.cold:  # warm-up: contexts, kernels, connections
            run_round(1 << 12, args.port, coeffs=args.coeffs, seal=args.seal)
        ok = True
        for r in range(args.rounds):
            st = run_round(1 << args.log2n, args.port, coeffs=args.coeffs, seed=r + 1, seal=args.seal)
            st.update({"round": r, "N": 1 << args.log2n, "t": 3, "n": 5, "coeffs": args.coeffs, "sealed": args.seal,
                       "cold": args.cold and r == 0})
            print(json.dumps(st), flush=True)
            ok = ok and st["peer_verified"]
    finally:
        stop_peer(proc, args.port)
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
