#!/usr/bin/env python3
"""Headline benchmark: device-resident Shamir 3-of-5 split + reconstruct over
GF(2^521 - 1) of one 2^24-element int64 vector (BASELINE.json `metric`, configs 2+3).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`python bench.py --gpus N` with N > 1 and no launcher environment starts
`torch.distributed.run` with N ranks as a child process and relays rank 0's
line; under a launcher, --gpus must equal WORLD_SIZE.

One step = `dn_m521_split_u64` (t=3, n=5) over the rank's N elements, then
`dn_m521_reconstruct` of shares xs (default 1,3,5) back to int64, inputs
resident in HBM before the timed region (secrets + MT19937 coefficients drawn
exactly as the reference's `make_shares` would draw them).  The steps rotate
over --placements separately allocated share buffers, and the line reports
the split's rate per buffer (`roofline.placement`).  Strong scaling, as
the metric names it: ONE 2^24-element vector, rank r splitting its tile-aligned
shard (dist.shard_range); value = 2^24 / max-over-ranks time per step.  At
N > 1 the line also carries `weak_scaling` (2^24 elements per GPU).

Prints ONE JSON line (rank 0) with `roofline` for the dominant kernel (split;
its average launch time from HIP events on the launch stream, algorithmic
bytes 470 B/element) and `cpu_baseline` (the pure-Python restatement of the
reference, oracle/py_shamir.py, 1 core, a time-bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "delta-node_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
# 32-bit VALU: 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz (MI355X_MICROARCH.md: a wave64
# VALU instruction issues over 2 cycles on its SIMD) = 78.6 T lane-ops/s
PEAK_VALU_GOPS = 256 * 4 * 32 * 2.4


# ds_read_b32 with every CU streaming (MI355X_MICROARCH.md §LDS: ≈75 TB/s)
PEAK_LDS_B32_GBPS = 75000.0


def roof(bound: str, achieved: float, note: str) -> dict:
    peak, unit = {"hbm": (PEAK_HBM_GBPS, "GB/s"), "lds": (PEAK_LDS_B32_GBPS, "GB/s")}.get(
        bound, (PEAK_VALU_GOPS, "Gop/s"))
    return {"bound": bound, "achieved": achieved, "peak": peak, "unit": unit, "frac": achieved / peak,
            "per_unit": note}
FE_BYTES = 66           # ceil(521 / 8): one field element in the tiled layout


class TimingEvent:
    """A HIP timing event created with hipEventDisableSystemFence, with the
    record / elapsed_time surface of torch.cuda.Event.  torch's events are
    hipEventDefault: recording one performs a system-scope fence — an L2
    write-back and invalidate between the kernels it sits between — which is a
    cost of the measurement, not of the path (hip_runtime_api.h: the flag
    "can improve the accuracy of timing measurements by avoiding the cost of
    cache writeback and invalidation").  Same stream, so the order of the
    kernels and the events is unchanged.  The HIP runtime is the one torch
    loaded (the SONAME resolves to the library already in the process)."""
    _hip = None
    FLAGS = 0x20000000  # hipEventDisableSystemFence

    @classmethod
    def hip(cls):
        if cls._hip is None:
            import ctypes

            maps = {ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln}
            if len(maps) != 1:
                raise RuntimeError(f"expected one HIP runtime in the process, found {sorted(maps)}")
            h = ctypes.CDLL(maps.pop())
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventSynchronize.argtypes = [ctypes.c_void_p]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._hip = h
        return cls._hip

    def __init__(self):
        import ctypes

        self.ev = ctypes.c_void_p()
        if self.hip().hipEventCreateWithFlags(ctypes.byref(self.ev), self.FLAGS) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def record(self, stream):
        if self.hip().hipEventRecord(self.ev, ctypes_stream(stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end) -> float:
        import ctypes

        h = self.hip()
        if h.hipEventSynchronize(end.ev) != 0:
            raise RuntimeError("hipEventSynchronize failed")
        ms = ctypes.c_float()
        if h.hipEventElapsedTime(ctypes.byref(ms), self.ev, end.ev) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def __del__(self):
        if self._hip is not None and self.ev:
            self._hip.hipEventDestroy(self.ev)


def ctypes_stream(stream):
    import ctypes

    return ctypes.c_void_p(stream.cuda_stream)


def warm(fn, seconds: float = 0.15) -> None:
    """Run fn back to back for `seconds` of wall time (at least 3 calls): the
    GPU clock ramps up over tens of milliseconds of sustained work after an
    idle stretch, and the VALU-heavy rows are timed at the steady clock."""
    t0 = time.perf_counter()
    k = 0
    while k < 3 or time.perf_counter() - t0 < seconds:
        fn()
        k += 1
        if k % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def secrets_int64(seed: int, n: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.integers(-(1 << 63), (1 << 63) - 1, size=n, endpoint=True, dtype=np.int64)


def cpu_baseline(t: int, n: int, xs, budget_s: float, procs: int = 16) -> dict:
    """Reference algorithm restated in pure Python (oracle/py_shamir.py), per
    element make_shares + resolve_shares, time-bounded samples: on one core
    (the reference runs these calls synchronously on its event loop — the
    `value`), and sharded over `procs` worker processes (the box's CPU share)."""
    import multiprocessing as mp

    from oracle.py_shamir import time_elements, time_elements_star

    half = budget_s / 2
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    done, dt = time_elements(t, n, xs, half, seed=7)
    out = {"value": done / dt, "unit": "elements/s", "cores": 1, "kind": "port",
           "sample": f"{done} elements x (make_shares t={t} n={n} + resolve_shares xs={list(xs)}), "
                     f"pure-Python restatement of delta_node/crypto/shamir, {dt:.1f} s on 1 core",
           "cpu_model": cpu_model, "host_cpus": os.cpu_count()}
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(time_elements_star, [(t, n, list(xs), half, 100 + i) for i in range(procs)])
        out["sharded"] = {"value": sum(d / s for d, s in res), "unit": "elements/s", "cores": procs,
                          "sample": f"{sum(d for d, _ in res)} elements over {procs} processes, {half:.1f} s each"}
    except Exception as e:  # a box without spare cores: report the 1-core figure only
        out["sharded"] = {"error": repr(e)}
    out["c_port"] = c_port_baseline(t, n, xs, half, procs)
    return out


def c_port_baseline(t: int, n: int, xs, budget_s: float, threads: int) -> dict:
    """SURVEY §8(d)(iii), the fair-CPU comparison: the same per-element work
    in C (oracle/m521_oracle.c: CPython MT19937 draw of the coefficients, the
    reference's Horner with a literal % p, its Lagrange sequence — 9x64-bit
    limbs) on 1 thread and on `threads` threads (ctypes drops the GIL), chunks
    of 2^14 elements, time-bounded."""
    import concurrent.futures as cf

    from oracle import c_oracle

    chunk = 1 << 14
    rng = np.random.default_rng(3)
    sec = rng.integers(-2 ** 62, 2 ** 62, chunk, dtype=np.int64)

    def work(seed: int, budget: float):
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            co = c_oracle.draw_coeffs(seed + done, chunk, t - 1)
            sh = c_oracle.split(sec, co, t, n)
            c_oracle.reconstruct(sh[[x - 1 for x in xs]], xs)
            done += chunk
        return done, time.perf_counter() - t0

    d1, s1 = work(11, budget_s / 4)
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(lambda i: work(1000 * i, budget_s / 2), range(threads)))
    wall = time.perf_counter() - t0
    total = sum(d for d, _ in res)
    return {"value": total / wall, "unit": "elements/s", "cores": threads, "kind": "port",
            "one_thread": d1 / s1,
            "sample": f"{total} elements over {threads} threads (chunks of {chunk}: MT19937 draw + split t={t} "
                      f"n={n} + reconstruct xs={list(xs)}), C restatement, {wall:.1f} s wall"}


def caller_blocks_row(sec, coeffs, N: int, t: int, n: int, nblocks: int, stream, split_bytes: int, want,
                      reps: int = 4) -> dict:
    """The headline split on share blocks a caller allocates itself
    (torch.empty, the C-ABI's caller-owned memory, dn_shamir.h): the same
    kernel and inputs as the timed steps, `nblocks` separately allocated
    blocks, the mean of `reps` launches on each after a first touch — what a
    caller passing its own `out` gets, beside the probed pool blocks."""
    from delta_node.crypto.shamir import _native

    blocks = [torch.empty((n, want.shape[1]), dtype=torch.uint8, device=sec.device) for _ in range(nblocks)]
    ms = []
    for b in blocks:
        _native.split_u64(sec, coeffs, b, N, t, n)
        evs = [(TimingEvent(), TimingEvent()) for _ in range(reps)]
        for e0, e1 in evs:
            e0.record(stream)
            _native.split_u64(sec, coeffs, b, N, t, n)
            e1.record(stream)
        torch.cuda.synchronize()
        ms.append(float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs])))
    equal = all(bool(torch.equal(b, want)) for b in blocks)
    del blocks
    fr = [split_bytes / (m * 1e-3) / 1e9 / PEAK_HBM_GBPS for m in ms]
    return {"allocator": "torch.empty (one hipMalloc each, not probed)", "blocks": nblocks,
            "launches_per_block": reps, "split_ms": ms, "frac": fr, "frac_min": min(fr),
            "frac_median": float(np.median(fr)), "frac_max": max(fr), "frac_mean_time": split_bytes / (
                float(np.mean(ms)) * 1e-3) / 1e9 / PEAK_HBM_GBPS, "equal_to_timed_block": equal}


def stream_ceiling(ins, in_bpt, outs, out_bpt, ntiles: int, reps: int = 5) -> dict:
    """dn_diag_tile_stream (lib/libdn_diag.so): per tile, 16-B non-temporal
    loads of `in_bpt[i]` bytes from every input buffer, then 16-B stores of
    `out_bpt[j]` bytes to every output buffer, no arithmetic; the fastest of
    four grid sizes.  Overwrites the outputs."""
    import ctypes

    diag = ctypes.CDLL(os.path.join(ROOT, "delta-node_amd", "lib", "libdn_diag.so"))
    vp = ctypes.c_void_p
    ip = (vp * 16)(*[t.data_ptr() for t in ins])
    ib = (ctypes.c_uint32 * 16)(*in_bpt)
    op = (vp * 16)(*[t.data_ptr() for t in outs])
    ob = (ctypes.c_uint32 * 16)(*out_bpt)
    stream = torch.cuda.current_stream()

    def launch(grid):
        rc = diag.dn_diag_tile_stream(ip, ib, len(ins), op, ob, len(outs), ctypes.c_uint64(ntiles), grid,
                                      vp(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dn_diag_tile_stream rc={rc}")

    best = None
    for grid in (256, 1024, 4096, 16384):
        launch(grid)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(reps):
            launch(grid)
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        if best is None or ms < best["ms"]:
            best = {"ms": ms, "grid": grid}
    return best


def measure_ceiling(dev, sec, coeffs, shares, N: int, t: int, n: int, reps: int = 5) -> dict:
    """Same-buffer HBM ceiling of the split: the split's exact bytes per tile —
    the rank's secrets, t-1 coefficient rows read, n share rows written — over
    the SAME buffers (so the same physical pages, whose placement sets this
    part's write rate: DESIGN.md §5.1).  Overwrites `shares`."""
    from delta_node.crypto.shamir import field

    if N % field.TILE:
        return None
    best = stream_ceiling([sec] + [coeffs[j] for j in range(t - 1)], [8 * field.TILE] + [field.TILE_BYTES] * (t - 1),
                          [shares[x] for x in range(n)], [field.TILE_BYTES] * n, N // field.TILE, reps)
    best["kernel"] = ("dn_diag_tile_stream: the split's bytes over the same buffers, 16-B nt loads then stores "
                      "per tile, no arithmetic (fastest of grids 256/1024/4096/16384)")
    return best


def measure_recon_ceiling(share_rows, rec, N: int, reps: int = 5) -> dict:
    """Same-buffer ceiling of the reconstruct: its k share rows read, the int64
    output written, per tile, over the same buffers.  Overwrites `rec`."""
    from delta_node.crypto.shamir import field

    if N % field.TILE:
        return None
    best = stream_ceiling(list(share_rows), [field.TILE_BYTES] * len(share_rows), [rec], [8 * field.TILE],
                          N // field.TILE, reps)
    best["kernel"] = "dn_diag_tile_stream: the reconstruct's bytes over the same buffers, no arithmetic"
    return best


def config4_bench(dev, world: int, rank: int, log2n_total: int = 26, reps: int = 5, dist_on: bool = False) -> dict:
    """BASELINE config 4: 5-of-9 split of a 2^26-element vector sharded by
    element across the ranks (rank r: `dist.shard_range`), then one RCCL
    all-gather of the per-rank share blocks (world > 1), timed separately.
    Coefficients are the reference's own MT19937 stream for the whole vector,
    each rank drawing its shard on the GPU (so the gathered shares are the
    unsharded reference split's); the timed kernel reads them (866 B/element).  Parity: every rank reconstructs its shard from shares
    1,3,5,7,9 and compares with its secrets; after the gather, the full vector's
    slice of every rank equals that rank's own block."""
    from delta_node.crypto.shamir import _native, dist as sdist, field

    t, n = 5, 9
    N_total = 1 << log2n_total
    lo, hi = sdist.shard_range(N_total, rank, world)
    nl = hi - lo
    B = sdist.shard_tiles(N_total, world) * field.TILE_BYTES
    vb = field.vec_bytes(nl)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    sec = torch.randint(-(1 << 62), 1 << 62, (nl,), dtype=torch.int64, device=dev, generator=g)
    # the reference's MT19937 coefficient stream of ONE 2^26-element draw, each
    # rank drawing only its shard on its GPU (jump-ahead; dist.draw_coeffs_sharded)
    from delta_node.crypto import shamir as _shamir

    ss = _shamir.SecretShare(t)
    ss.random.seed(4321)
    if dist_on:
        cb = sdist.draw_coeffs_sharded(ss, N_total, dev)
        coeffs = cb[:, :vb].contiguous() if cb.shape[1] != vb else cb
    else:
        coeffs = ss.draw_coeffs_vec(N_total, dev)
    # the split writes into a share block as make_shares_vec returns one
    # (memory.share_block); the all-gather's padded send block is separate
    from delta_node.crypto.shamir import memory as _memory

    shares = _memory.share_block((n, vb), dev)
    block = torch.zeros((n, B), dtype=torch.uint8, device=dev) if dist_on else None
    stream = torch.cuda.current_stream()
    for _ in range(2):
        _native.split_u64(sec, coeffs, shares, nl, t, n)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(stream)
        _native.split_u64(sec, coeffs, shares, nl, t, n)
        b.record(stream)
    torch.cuda.synchronize()
    split_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if block is not None:
        block[:, :vb].copy_(shares)
    xs = [1, 3, 5, 7, 9]
    rec = torch.empty(nl, dtype=torch.int64, device=dev)
    _native.reconstruct([shares[x - 1] for x in xs], _native.lagrange(xs, t), out_u64=rec, n=nl)
    ok = bool(torch.equal(rec, sec))
    per_elem = 8 + (t - 1) * FE_BYTES + n * FE_BYTES
    split_max_ms = split_ms
    out = {"workload": f"{t}-of-{n} split of 2^{log2n_total} int64 elements sharded over {world} GPU(s), "
                       f"2^{log2n_total} / {world} per GPU",
           "elements_per_gpu": nl, "split_ms": split_ms,
           "roofline": roof("hbm", nl * per_elem / (split_ms * 1e-3) / 1e9,
                            f"8 B secret + {t - 1} x 66 B coefficients + {n} x 66 B shares per element"),
           "roundtrip_equal": ok}
    if dist_on:
        import torch.distributed as tdist

        cdev = dev if tdist.get_backend() == "nccl" else torch.device("cpu")
        tt = torch.tensor([split_ms], dtype=torch.float64, device=cdev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        split_max_ms = float(tt.item())
        full = sdist.allgather_share_blocks(block, N_total)  # warm-up (RCCL channels)
        del full
        tdist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(3):
            full = sdist.allgather_share_blocks(block, N_total)
        torch.cuda.synchronize()
        tdist.barrier()
        gdt = (time.perf_counter() - g0) / 3
        same = bool(torch.equal(full[:, rank * B: rank * B + vb], block[:, :vb]))
        del full
        flags = torch.tensor([int(ok and same)], dtype=torch.int32, device=cdev)
        tdist.all_reduce(flags, op=tdist.ReduceOp.MIN)
        recv = block.numel() * (world - 1)
        out["allgather"] = {"ms": gdt * 1e3, "bytes_received_per_gpu": recv, "GBps_per_gpu": recv / gdt / 1e9,
                            "blocks_equal": same, "all_ranks_ok": bool(flags.item())}
    out["split_elems_per_s_aggregate"] = N_total / (split_max_ms * 1e-3)
    ceil = measure_ceiling(dev, sec, coeffs, shares, nl, t, n)
    if ceil:
        out["roofline"]["ceiling_measured"] = {**ceil, "GBps": nl * per_elem / (ceil["ms"] * 1e-3) / 1e9,
                                               "split_frac_of_ceiling": ceil["ms"] / split_ms}
    del block, shares, coeffs, sec, rec
    torch.cuda.empty_cache()
    return out


def config5_bench(log2n: int, rounds: int = 2) -> dict:
    """BASELINE config 5: end-to-end masked-result round between this process
    and a second local delta-node process over loopback HTTP
    (scripts/e2e_round.py: pack -> H2D -> split -> GPU share encode -> D2H ->
    POST per share; the peer decodes + reconstructs and checks a digest after
    each round).  Both coefficient sources: the reference's MT19937 stream
    drawn on the GPU (bit-exact drop-in) and the device ChaCha20 form."""
    import importlib.util
    import socket

    spec = importlib.util.spec_from_file_location("e2e_round", os.path.join(ROOT, "scripts", "e2e_round.py"))
    e2e = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(e2e)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    proc = e2e.start_peer(port)
    out = {"workload": f"masked result {{'w': {{'w': int64[2^{log2n}]}}}} -> 3-of-5 shares as _share_to_bytes records, "
                       "POSTed to a second local process over loopback HTTP; wall-clock pack start -> last HTTP 200",
           "unit": "MB/s of int64 input"}
    try:
        e2e._wait_ready(port)
        e2e.run_round(1 << 12, port, coeffs="prng")  # warm-up (peer imports torch, kernels load)
        for coeffs in ("mt", "prng"):
            runs = [e2e.run_round(1 << log2n, port, coeffs=coeffs, seed=r + 1) for r in range(rounds)]
            best = max(runs, key=lambda r: r["input_MBps"])
            out[coeffs] = {"input_MBps": best["input_MBps"], "wall_s": best["wall_s"],
                           "wall_s_all": [r["wall_s"] for r in runs],
                           "stages_s": {k: best[k] for k in ("pack_s", "h2d_s", "split_s", "encode_d2h_s",
                                                             "post_tail_s")},
                           "http_GBps": best["http_GBps"], "bytes_posted": best["bytes_posted"],
                           "peer_verified": all(r["peer_verified"] for r in runs)}
    finally:
        e2e.stop_peer(proc, port)
    return out


def envelope_row(recs, reps: int, s, e) -> dict:
    """Share envelope (second half): one receiver's packed
    records -> "0x" + hex(base64(nonce || AES-256-CTR)) = the ASCII of
    serialize.bytes_to_hex(aes.encrypt(key, records)) (crypto/aes/aes.py:8-14,
    runner/horizontal/commu.py:23-49) and back.  LDS roofline: 14 rounds x 16
    T-table lookups (4 B, conflict-free ds_read_b32) per 16-byte block."""
    import base64
    import shutil
    import subprocess

    from delta_node.crypto import aes
    from oracle import c_oracle

    key, nonce = bytes(range(32)), bytes(range(16, 32))
    n = recs.numel()
    env = aes.encrypt_vec(key, recs, nonce=nonce, hex=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        env = aes.encrypt_vec(key, recs, nonce=nonce, hex=True)
    e.record()
    torch.cuda.synchronize()
    enc_alloc_ms = s.elapsed_time(e) / reps
    # the API call on a reused buffer (encrypt_buffer): the kernel + one 2-byte "0x" copy
    obuf = aes.encrypt_buffer(n, True, recs.device)
    env2 = aes.encrypt_vec(key, recs, nonce=nonce, hex=True, out=obuf)
    warm(lambda: aes.encrypt_vec(key, recs, nonce=nonce, hex=True, out=obuf))
    s.record()
    for _ in range(reps):
        env2 = aes.encrypt_vec(key, recs, nonce=nonce, hex=True, out=obuf)
    e.record()
    torch.cuda.synchronize()
    enc_ms = s.elapsed_time(e) / reps
    out_equal = bool(torch.equal(env2, env))
    del env2, obuf
    back = aes.decrypt_vec(key, env, hex=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        back = aes.decrypt_vec(key, env, hex=True)
    e.record()
    torch.cuda.synchronize()
    dec_ms = s.elapsed_time(e) / reps
    # the encrypt kernel alone: the C entry point on a preallocated text buffer
    # (the API call above also allocates its 3 GB output and writes "0x"),
    # events on its stream, best of 3 rounds of `reps` launches
    import ctypes as _ct

    from delta_node.crypto.aes import aes as _aes_mod
    from delta_node.crypto.shamir import _native as _cn

    AL = _aes_mod._lib()
    kbuf = torch.empty(16 + int(AL.dn_aes_encrypt_len(n, 1)), dtype=torch.uint8, device=recs.device)
    stream = torch.cuda.current_stream()

    def k_enc():
        _cn.check(AL.dn_aes_encrypt(key, len(key), nonce, recs.data_ptr(), n, kbuf.data_ptr() + 16, 1,
                                    stream.cuda_stream))

    kern = []
    warm(k_enc)
    for _ in range(3):
        s.record(stream)
        for _ in range(reps):
            k_enc()
        e.record(stream)
        torch.cuda.synchronize()
        kern.append(s.elapsed_time(e) / reps)
    enc_kernel_ms = min(kern)
    kernel_equal = bool(torch.equal(kbuf[16:], env[2:]))
    # the decrypt kernels alone (decode + in-place CTR, csrc/aes_envelope.hip) on the
    # "0x"-prefixed text as the JSON carries it, into a preallocated output
    tl = env.numel() - 2
    cap = int(AL.dn_aes_decrypt_capacity(tl, 1))
    dbuf = torch.empty(cap + 16, dtype=torch.uint8, device=recs.device)
    olen = torch.zeros(1, dtype=torch.int64, device=recs.device)
    dbad = torch.zeros(1, dtype=torch.int32, device=recs.device)

    def k_dec():
        _cn.check(AL.dn_aes_decrypt(key, len(key), env.data_ptr() + 2, tl, 1, dbuf.data_ptr(), cap + 16,
                                    olen.data_ptr(), dbad.data_ptr(), stream.cuda_stream))

    dkern = []
    warm(k_dec)
    for _ in range(3):
        s.record(stream)
        for _ in range(reps):
            k_dec()
        e.record(stream)
        torch.cuda.synchronize()
        dkern.append(s.elapsed_time(e) / reps)
    dec_kernel_ms = min(dkern)
    dec_kernel_equal = bool(torch.equal(dbuf[:n], recs)) and int(olen.item()) == n and int(dbad.item()) == 0
    del kbuf, dbuf
    units = 4096  # the first 4096 thread units (196 KB) against the oracle
    m = base64.b64decode(bytes.fromhex(bytes(env[2:2 + 128 * units].cpu().numpy()).decode()))
    oracle_ok = m[:16] == nonce and m[16:] == c_oracle.aes_ctr(key, nonce, bytes(recs[:len(m) - 16].cpu().numpy()))
    text_bytes = env.numel()
    lds_bytes = (n + 15) // 16 * 14 * 16 * 4
    row = {"workload": f"packed records of share x=3 ({n / 1e9:.2f} GB) <-> '0x' + hex(base64(nonce || AES-256-CTR)) "
                       f"({text_bytes / 1e9:.2f} GB)",
           "encrypt_ms": enc_ms, "decrypt_ms": dec_ms, "encrypt_alloc_ms": enc_alloc_ms,
           "encrypt_over_kernel": enc_ms / enc_kernel_ms, "encrypt_out_equal": out_equal,
           "encrypt_kernel_ms": enc_kernel_ms, "encrypt_kernel_equal_api": kernel_equal,
           "decrypt_kernel_ms": dec_kernel_ms, "decrypt_kernel_roundtrip": dec_kernel_equal,
           "timing": "encrypt_ms: the Python API call on a reused buffer (out=encrypt_buffer(n, hex)), "
                     "after >= 0.15 s of warm-up; encrypt_alloc_ms: the API call allocating its 3 GB output; "
                     "decrypt_ms: the API call (output allocation, the length read-back), mean of one round; "
                     "encrypt_kernel_ms: dn_aes_encrypt on a preallocated buffer, >= 0.15 s warm-up, best of "
                     "3 rounds; the rooflines use the kernel time",
           "encrypt_plaintext_GBps": n / (enc_ms * 1e-3) / 1e9, "decrypt_plaintext_GBps": n / (dec_ms * 1e-3) / 1e9,
           "roofline_lds": roof("lds", lds_bytes / (enc_kernel_ms * 1e-3) / 1e9,
                                "14 rounds x 16 Te lookups x 4 B per 16-byte block (encrypt kernel)"),
           "roofline_hbm": roof("hbm", (n + text_bytes) / (enc_kernel_ms * 1e-3) / 1e9,
                                "record bytes in + 2.67 x text bytes out (encrypt kernel)"),
           "roofline_lds_decrypt": roof("lds", lds_bytes / (dec_kernel_ms * 1e-3) / 1e9,
                                        "14 rounds x 16 Te lookups x 4 B per 16-byte block (decode + CTR kernels)"),
           "bound": "lds + valu (T-table AES-256; base64 and hex fused)",
           "roundtrip_equal": bool(torch.equal(back, recs)), "oracle_prefix_equal": bool(oracle_ok)}
    del env, back
    if shutil.which("openssl"):
        # the reference's stack on one core: OpenSSL AES-256-CTR (what `cryptography` wraps; its CLI
        # here) + CPython base64.b64encode + bytes.hex, on a 2^26-byte sample of the same records
        sample = bytes(recs[: 1 << 26].cpu().numpy())
        t0 = time.perf_counter()
        ct = subprocess.run(["openssl", "enc", "-aes-256-ctr", "-K", key.hex(), "-iv", nonce.hex(), "-nosalt"],
                            input=sample, capture_output=True, check=True).stdout
        text = "0x" + base64.b64encode(nonce + ct).hex()
        dt = time.perf_counter() - t0
        row["cpu_baseline"] = {"plaintext_GBps": len(sample) / dt / 1e9, "cores": 1, "kind": "port",
                               "sample": "2^26 record bytes: openssl enc -aes-256-ctr (AES-NI) + base64.b64encode "
                                         "+ bytes.hex, 1 core",
                               "text_prefix_equal": text[:2 + 8 * 4096] == "0x" + base64.b64encode(m[:3 * 4096]).hex()}
    return row


MASK_MIX_BOUND = 1.0 / (23.5 / 3.6e13 + 22.0 / 6.1e13)  # draws/s the draw loop's instruction mix allows


def mask_row(dev, log2n: int) -> dict:
    """mask PRG + fixed-point masking = fix_precision(val) + seed mask + 9
    pairwise masks (runner/horizontal/agg.py:284-318 with |u2| = 10), one
    dn_bounded_i64_accumulate launch over 10 generators."""
    import os as _os

    from delta_node.utils import masked_sum
    from oracle import py_mask as pm

    n = 1 << log2n
    val = torch.randn(n, dtype=torch.float64, device=dev) * 1e3
    terms = [(_os.urandom(32), 1)] + [(_os.urandom(32), (-1) ** i) for i in range(9)]
    out = torch.empty(n, dtype=torch.int64, device=dev)
    masked_sum(val, terms, precision=8, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    s.record()
    for _ in range(reps):
        masked_sum(val, terms, precision=8, out=out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    # the kernel alone (dn_bounded_i64_accumulate over the 10 seeded generators,
    # float64 base), events on its launch stream: masked_sum's call time above
    # also holds the host SeedSequence seeding and the rejection-flag read-back
    from delta_node.utils import _mask_native as mn

    gens = [mn.pcg64(sd) for sd, _ in terms]
    sg = [int(x) for _, x in terms]
    flags = torch.zeros(len(gens), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    mn.accumulate(gens, sg, out, n, 0, 2 ** 47 - 2, base_f64=val, precision=8, rejects=flags)
    s.record(stream)
    for _ in range(reps):
        mn.accumulate(gens, sg, out, n, 0, 2 ** 47 - 2, base_f64=val, precision=8, rejects=flags)
    e.record(stream)
    torch.cuda.synchronize()
    kms = s.elapsed_time(e) / reps
    # parity on a prefix vs numpy (the reference's generator)
    k = 1 << 14
    vh = val[:k].cpu().numpy()
    want = pm.fix_precision(vh, 8)
    for sd, sg in terms:
        want = want + sg * pm.make_mask_numpy(sd, (k,))  # a prefix of the length-n mask
    ok = bool(np.array_equal(out[:k].cpu().numpy(), want))
    # CPU baseline: the reference's numpy calls on a 2^20 sample, 1 thread of numpy
    m = 1 << 20
    vs = np.random.default_rng(0).standard_normal(m) * 1e3
    t0 = time.perf_counter()
    acc = pm.fix_precision(vs, 8)
    for sd, sg in terms:
        acc = acc + sg * pm.make_mask_numpy(sd, vs.shape)
    cpu_dt = time.perf_counter() - t0
    return {
        "workload": f"fix_precision(2^{log2n} float64) + 10 make_mask(32-byte seed) with signs, int64",
        "ms": ms, "kernel_ms": kms, "elems_per_s": n / (ms * 1e-3), "draws_per_s": 10 * n / (ms * 1e-3),
        "kernel_draws_per_s": 10 * n / (kms * 1e-3),
        "roofline": roof("hbm", 16 * n / (kms * 1e-3) / 1e9, "8 B float64 in + 8 B int64 out per element (kernel)"),
        "bound": "valu (PCG64 128-bit LCG step + XSL-RR + Lemire per draw)",
        # ISA of bounded_acc_kernel<true>'s paired-generator loop body (2 x 8
        # draws): 45.5 VALU per draw, 23.5 of them VOP3 (v_mad_u64_u32,
        # v_mul_lo_u32, 64-bit shifts / adds) and 22 VOP1/VOP2; measured issue
        # rates (tools/valu_rates.hip): VOP3 3.6e13, VOP1/2 6.1e13
        # lane-ops/s -> the mix allows 1 / (23.5 / 3.6e13 + 22 / 6.1e13) draws/s
        "roofline_valu": roof("valu", 10 * n / (kms * 1e-3) * 45.5 / 1e9,
                              "45.5 VALU instructions per draw (ISA count), 10 draws per element (kernel)"),
        "mix_bound": {"draws_per_s": MASK_MIX_BOUND, "frac": 10 * n / (kms * 1e-3) / MASK_MIX_BOUND,
                      "per_draw": "23.5 VOP3 @ 3.6e13/s + 22 VOP1/2 @ 6.1e13/s (draw loop only; tile jumps, "
                                  "base conversion and stores are extra instructions)"},
        "numpy_prefix_equal": ok,
        "cpu_numpy": {"elems_per_s": m / cpu_dt, "sample": f"2^20 elements x 10 masks, numpy 1 thread"}}


def rows_bench(dev, log2n: int) -> dict:
    """SURVEY §8(f) rows measured beside the headline (device-resident inputs):
    mask PRG + fixed-point masking = fix_precision(val) + seed mask + 9
    pairwise masks (runner/horizontal/agg.py:284-318 with |u2| = 10)."""
    n = 1 << log2n
    rows = {}
    reps = 5
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # share wire codec: encode / decode share x=3 of a 2^log2n vector (reference _share_to_bytes records)
    from delta_node.crypto.shamir import codec, field as _field

    ss = __import__("delta_node.crypto.shamir", fromlist=["SecretShare"]).SecretShare(3)
    ss.random.seed(5)
    blk = ss.make_shares_vec(torch.from_numpy(secrets_int64(3, n)), 5)
    packed, offs = codec.encode_share_vec(blk[2], n, 3)
    torch.cuda.synchronize()
    # the API calls: allocating their outputs (the decoder's bad-record
    # read-back per call) and on caller buffers (the decoder's check deferred
    # to one read-back after the loop: decode_share_vec(..., bad=flag))
    s.record()
    for _ in range(reps):
        packed, offs = codec.encode_share_vec(blk[2], n, 3, trim=False)
    e.record()
    torch.cuda.synchronize()
    enc_alloc_ms = s.elapsed_time(e) / reps
    total = int(offs[n].item())
    s.record()
    for _ in range(reps):
        vec, _xs = codec.decode_share_vec(packed, offs, n)
    e.record()
    torch.cuda.synchronize()
    dec_alloc_ms = s.elapsed_time(e) / reps
    cpk, cof = torch.empty_like(packed), torch.empty_like(offs)
    cvec, cxs = torch.empty_like(vec), torch.empty(n, dtype=torch.int64, device=dev)
    cbad = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.encode_share_vec(blk[2], n, 3, trim=False, out=cpk, offsets=cof)
    codec.decode_share_vec(packed, offs, n, out=cvec, xs=cxs, bad=cbad)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        codec.encode_share_vec(blk[2], n, 3, trim=False, out=cpk, offsets=cof)
    e.record()
    torch.cuda.synchronize()
    enc_call_ms = s.elapsed_time(e) / reps
    s.record()
    for _ in range(reps):
        codec.decode_share_vec(packed, offs, n, out=cvec, xs=cxs, bad=cbad)
    e.record()
    torch.cuda.synchronize()
    dec_call_ms = s.elapsed_time(e) / reps
    codec.check_bad(cbad)
    buffers_equal = bool(torch.equal(cvec, blk[2])) and bool(torch.equal(cpk[:total], packed[:total]))
    del cpk, cof, cvec, cxs
    # the kernels: the C entry points on preallocated buffers, events on their stream
    import ctypes as _ct

    CL = codec._lib()
    cap = int(CL.dn_m521_encoded_capacity(n, 3))
    kout = torch.empty(cap, dtype=torch.uint8, device=dev)
    koffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ksb = int(CL.dn_m521_codec_scratch_bytes(n))
    kscr = torch.empty(ksb, dtype=torch.uint8, device=dev)
    kvec = torch.empty(_field.vec_bytes(n), dtype=torch.uint8, device=dev)
    kxs = torch.empty(n, dtype=torch.int64, device=dev)
    kbad = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    from delta_node.crypto.shamir import _native as _cn

    def k_enc():
        _cn.check(CL.dn_m521_encode_shares(blk[2].data_ptr(), n, 3, koffs.data_ptr(), kout.data_ptr(), cap,
                                           kscr.data_ptr(), ksb, _ct.c_void_p(stream.cuda_stream)))

    def k_dec():
        _cn.check(CL.dn_m521_decode_shares(packed.data_ptr(), packed.numel(), offs.data_ptr(), n, kvec.data_ptr(),
                                           kxs.data_ptr(), kbad.data_ptr(), _ct.c_void_p(stream.cuda_stream)))

    kt = {}
    for name, fn in (("enc", k_enc), ("dec", k_dec)):
        fn()
        s.record(stream)
        for _ in range(reps):
            fn()
        e.record(stream)
        torch.cuda.synchronize()
        kt[name] = s.elapsed_time(e) / reps
    enc_ms, dec_ms = kt["enc"], kt["dec"]
    kernels_equal = (bool(torch.equal(koffs, offs)) and bool(torch.equal(kout[:total], packed[:total]))
                     and bool(torch.equal(kvec, blk[2])) and int(kbad.item()) == 0)
    del kout, koffs, kscr, kvec, kxs
    # CPU: the reference's per-share codec (shamir.py:28-45) restated, on a 2^16 sample of the same shares
    from oracle.py_shamir import parse_share, share_to_bytes

    k = 1 << 16
    ys = _field.vec_to_ints(blk[2, : _field.vec_bytes(k)].cpu().numpy(), k)
    t0 = time.perf_counter()
    recs = [share_to_bytes(3, y) for y in ys]
    cpu_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    back_ys = [parse_share(r)[1] for r in recs]
    cpu_dec = time.perf_counter() - t0
    enc_bytes = n * 66 + total + 8 * (n + 1)
    dec_bytes = total + 8 * (n + 1) + n * 66 + 8 * n
    rows["share_codec"] = {"workload": f"share x=3 of 2^{log2n} elements <-> packed _share_to_bytes records",
                           "encode_ms": enc_ms, "decode_ms": dec_ms, "bytes_out": total,
                           "encode_call_ms": enc_call_ms, "decode_call_ms": dec_call_ms,
                           "encode_call_alloc_ms": enc_alloc_ms, "decode_call_alloc_ms": dec_alloc_ms,
                           "decode_call_over_kernel": dec_call_ms / dec_ms,
                           "api_buffers_equal": buffers_equal,
                           "timing": "encode_ms / decode_ms: the C entry points on preallocated buffers (kernels); "
                                     "*_call_ms: the Python API calls on caller buffers (out=, offsets=, xs=; the "
                                     "decoder's bad-record check deferred: bad=flag, one check after the loop); "
                                     "*_call_alloc_ms: the API calls allocating their outputs, the decoder "
                                     "checking per call (a read-back each)",
                           "kernels_equal_api": kernels_equal,
                           "encode_elems_per_s": n / (enc_ms * 1e-3), "decode_elems_per_s": n / (dec_ms * 1e-3),
                           "roundtrip_equal": bool(torch.equal(vec, blk[2])),
                           "reference_bytes_equal_sample": bool(
                               b"".join(recs[:4096]) == bytes(packed[: int(offs[4096].item())].cpu().numpy())
                               and back_ys == ys),
                           "roofline_encode": roof("hbm", enc_bytes / (enc_ms * 1e-3) / 1e9,
                                                   "66 B vector + record bytes + 8 B offset per element"),
                           "roofline_decode": roof("hbm", dec_bytes / (dec_ms * 1e-3) / 1e9,
                                                   "record bytes + 8 B offset in, 66 B + 8 B x out per element"),
                           "cpu_baseline": {"encode_elems_per_s": k / cpu_enc, "decode_elems_per_s": k / cpu_dec,
                                            "cores": 1, "kind": "port",
                                            "sample": "2^16 shares, _share_to_bytes / _bytes_to_share restated "
                                                      "(oracle/py_shamir.py), 1 core"}}
    rows["share_envelope"] = envelope_row(packed[:total], reps, s, e)
    del packed, vec
    # device-PRNG split (dn_m521_split_prng, SURVEY §8(d) config 2'): coefficients generated in-kernel
    from delta_node.crypto.shamir import _native as _nat

    from delta_node.crypto.shamir import memory as _memory

    # make_shares_vec_prng's own output blocks (memory.share_block)
    shs = [_memory.share_block((5, _field.vec_bytes(n)), dev) for _ in range(3)]
    sec = torch.from_numpy(secrets_int64(3, n)).to(dev)
    prng = {}
    # The rows before this one end in host-only work (the CPU baselines), and
    # the GPU clock falls while it idles: the VALU-heavy ChaCha20 split then
    # reads ~20 % slow for its first tens of milliseconds (scripts/prng_row_probe.py,
    # profiles/r03/ab/prng_clock/).  So: `warm` (>= 150 ms of the same call),
    # then per output buffer (three placements, as the draw_split row) the best
    # of three rounds of `reps` launches; the median over the buffers is quoted.
    for rounds in (20, 8):
        by_buf, rounds_ms = [], []
        warm(lambda: _nat.split_prng(sec, bytes(range(32)), 0, rounds, 0, shs[0], n, 3, 5))
        for sh in shs:
            rms = []
            for _ in range(3):
                s.record()
                for _ in range(reps):
                    _nat.split_prng(sec, bytes(range(32)), 0, rounds, 0, sh, n, 3, 5)
                e.record()
                torch.cuda.synchronize()
                rms.append(s.elapsed_time(e) / reps)
            by_buf.append(min(rms))
            rounds_ms.append(rms)
        pm = float(np.median(by_buf))
        sh = shs[-1]
        back = ss.resolve_shares_vec([sh[1], sh[2], sh[4]], [2, 3, 5], n)
        ops = (2 * 17 / 16) * (12 * 4 * rounds + 32)  # ChaCha lane-ops per element (2.125 blocks)
        prng[f"chacha{rounds}"] = {"ms": pm, "ms_by_buffer": by_buf, "ms_rounds": rounds_ms,
                                   "elems_per_s": n / (pm * 1e-3),
                                   "roofline_hbm": roof("hbm", n * (8 + 5 * 66) / (pm * 1e-3) / 1e9,
                                                        "8 B secret + 5 x 66 B shares per element"),
                                   "roofline_valu": roof("valu", n * ops / (pm * 1e-3) / 1e9,
                                                         f"{ops:.0f} ChaCha lane-ops per element (2.125 blocks)"),
                                   "roundtrip_equal": bool(torch.equal(back, sec))}
    rows["split_prng"] = {"workload": f"3-of-5 split of 2^{log2n} int64, coefficients generated on the device "
                                      f"(338 B/elem HBM)",
                          "timing": "median over three output buffers of the best of three rounds of "
                                    f"{reps} launches each, after >= 0.15 s of warm-up launches", **prng}
    del shs, sh, sec, back
    # coordinator member sum: 10 int64 members
    from delta_node.utils import sum_int64

    mem = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device=dev) for _ in range(10)]
    outs = torch.empty(n, dtype=torch.int64, device=dev)
    sum_int64(mem, out=outs)
    s.record()
    for _ in range(reps):
        sum_int64(mem, out=outs)
    e.record()
    torch.cuda.synchronize()
    sm = s.elapsed_time(e) / reps
    k = 1 << 22  # CPU: make_masked_results' numpy accumulation (coord/horizontal/agg.py:227-251), 1 core
    memh = [m[:k].cpu().numpy() for m in mem]
    t0 = time.perf_counter()
    acc = memh[0].copy()
    for mh in memh[1:]:
        acc += mh
    cpu_sum = time.perf_counter() - t0
    rows["member_sum"] = {"workload": f"10 members x 2^{log2n} int64 masked results", "ms": sm,
                          "roofline": roof("hbm", 11 * 8 * n / (sm * 1e-3) / 1e9, "10 x 8 B in + 8 B out per element"),
                          "equal_torch_sum": bool(torch.equal(outs, torch.stack(mem).sum(0))),
                          "equal_numpy_sample": bool(np.array_equal(outs[:k].cpu().numpy(), acc)),
                          "cpu_baseline": {"elems_per_s": k / cpu_sum, "cores": 1, "kind": "port",
                                           "sample": "2^22 elements x 10 members, numpy += (the reference's loop)"}}
    # MiMC7 data commitment (utils/mimc7.py:63-92): 2^15 rows x (9 features + label), 256 Merkle roots
    from delta_node.utils import mimc7
    from oracle import py_mimc7

    drng = np.random.default_rng(11)
    data = drng.standard_normal((1 << 15, 10))
    data[:, -1] = drng.integers(0, 2, 1 << 15)
    ddev = torch.from_numpy(data).to(dev)
    roots = mimc7.calc_data_commitment(ddev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        roots = mimc7.calc_data_commitment(ddev)
    mm = (time.perf_counter() - t0) / 3 * 1e3
    t0 = time.perf_counter()
    want = py_mimc7.data_commitment(data[:256])
    cdt = time.perf_counter() - t0
    mulmods = (1 << 15) * 10 * 13 * 4 + 256 * 127 * 2 * 13 * 4  # x^7 = 4 Montgomery products per round
    # the same at 2^20 rows: enough rows to fill the chip (throughput- rather than latency-bound)
    big = drng.standard_normal((1 << 20, 10))
    big[:, -1] = drng.integers(0, 2, 1 << 20)
    bdev = torch.from_numpy(big).to(dev)
    broots = mimc7.calc_data_commitment(bdev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        broots = mimc7.calc_data_commitment(bdev)
    bm = (time.perf_counter() - t0) / 3 * 1e3
    bwant = py_mimc7.data_commitment(big[:128])
    big_row = {"ms": bm, "rows_per_s": (1 << 20) / (bm * 1e-3),
               "mont_mul_per_s": ((1 << 20) * 10 * 13 * 4 + 8192 * 127 * 2 * 13 * 4) / (bm * 1e-3),
               "oracle_prefix_equal": broots[:1] == bwant}
    del bdev
    # calc_weight_commitment (mimc7.py:58-60): one sequential chain, host core (dn_mimc7_weight_commitment_host)
    # beside the same chain on one device lane (dn_mimc7_weight_chain) and the Python restatement
    wts = drng.standard_normal(1 << 17) * 0.1
    t0 = time.perf_counter()
    wc = mimc7.calc_weight_commitment(wts)
    wh = time.perf_counter() - t0
    wdev = torch.from_numpy(wts[:4096]).to(dev)
    mimc7.weight_commitment_device(wdev[:16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wd = mimc7.weight_commitment_device(wdev)
    wdt = time.perf_counter() - t0
    t0 = time.perf_counter()
    wp = py_mimc7.weight_commitment(wts[:4096])
    wpt = time.perf_counter() - t0
    weight_row = {"workload": "calc_weight_commitment of 2^17 float64 weights (52 dependent products each)",
                  "host_us_per_weight": wh / (1 << 17) * 1e6,
                  "device_lane_us_per_weight": wdt / 4096 * 1e6,
                  "cpu_python_us_per_weight": wpt / 4096 * 1e6,
                  "oracle_equal_4096": wd == wp and mimc7.calc_weight_commitment(wts[:4096]) == wp,
                  "commitment_prefix": wc.hex()[:16]}
    rows["mimc7_commitment"] = {"workload": "calc_data_commitment, 2^15 rows x 10 cols -> 256 roots",
                                "ms": mm, "rows_per_s": (1 << 15) / (mm * 1e-3),
                                "mont_mul_per_s": mulmods / (mm * 1e-3),
                                "parallelism": "one lane per row (512 waves for 1024 SIMDs), then one wave per "
                                               "128-row Merkle block: latency-bound chains at this size",
                                "oracle_prefix_equal": roots[:2] == want, "bound": "valu (BN254 Montgomery mul)",
                                "cpu_python": {"rows_per_s": 256 / cdt, "sample": "256 rows, Python ints 1 thread"},
                                "at_2e20_rows": big_row, "weight_commitment": weight_row}
    rows["mask_masking"] = mask_row(dev, log2n)
    return rows


def draw_split_row(dev, log2n: int, reps: int = 3) -> dict:
    """make_shares_vec(values, 5) with the reference's coefficients (t = 3):
    MT19937 draws on the GPU (jump-ahead substreams) fused with the split
    (dn_mt19937_split_device), vs the coefficient block drawn then split.
    Wall time per call (the call synchronises: it returns CPython's final MT
    state).  Bytes: 8 + 5 x 66 per element fused (no coefficient block), vs
    2 x 66 written + 470 for draw then split."""
    import random

    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import _native, field, memory

    n = 1 << log2n
    sec = torch.from_numpy(secrets_int64(5, n)).to(dev)
    # the fused call's generation writes the shares at the rate of their pages'
    # placement: three separately allocated outputs, the
    # best of `reps` calls on each, the median of the three quoted
    # (the share blocks make_shares_vec allocates itself when out is None: memory.share_block)
    outs = [memory.share_block((5, field.vec_bytes(n)), dev) for _ in range(3)]
    fused_by_buf, unfused = [], []
    ok = True
    wss = shamir.SecretShare(3)
    warm(lambda: wss.make_shares_vec(sec, 5, out=outs[0]))
    for bi, out in enumerate(outs):
        fused = []
        for r in range(reps + 1):
            a, b = shamir.SecretShare(3), shamir.SecretShare(3)
            a.random.seed(77 + r)
            b.random.seed(77 + r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            got = a.make_shares_vec(sec, 5, out=out)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if r:  # the first call on each buffer warms up
                fused.append(t1 - t0)
            if bi == 0:  # draw then split, and the parity check, once
                co = b.draw_coeffs_vec(n, dev)
                want = torch.empty_like(out)
                _native.split_u64(sec, co, want, n, 3, 5)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                if r:
                    unfused.append(t2 - t1)
                ok = ok and bool(torch.equal(got, want)) and a.random.getstate() == b.random.getstate()
                del co, want
        fused_by_buf.append(min(fused))
    fm, um = float(np.median(fused_by_buf)), min(unfused)
    del outs
    # back to back in a loop, as a caller splitting vector after vector does:
    # the product default (out=None: each call's block from memory.share_block,
    # the previous one back to the pool) and a caller's own torch.empty block
    loop = {}
    spec0 = _native.mt_spec_stats()
    for name in ("pooled_default_out", "caller_out"):
        ss = shamir.SecretShare(3)
        ss.random.seed(91)
        mine = torch.empty((5, field.vec_bytes(n)), dtype=torch.uint8, device=dev) if name == "caller_out" else None
        for _ in range(3):
            r = ss.make_shares_vec(sec, 5, out=mine)
            del r
        torch.cuda.synchronize()
        reps_l = 10
        t0 = time.perf_counter()
        for _ in range(reps_l):
            r = ss.make_shares_vec(sec, 5, out=mine)
            del r
        torch.cuda.synchronize()
        loop[name] = (time.perf_counter() - t0) / reps_l * 1e3
        del mine
    spec1 = _native.mt_spec_stats()
    # calls of the loops that used windows speculated by the call before
    # (DN_MT_SPEC: a call continuing its predecessor computes the next one's
    # jump levels on a side stream beside its generation)
    loop["speculated_calls"] = spec1["hits"] - spec0["hits"]
    loop["calls"] = 2 * (3 + 10)
    words = 17 * 2 * n
    # smaller vectors take shorter MT substreams (2^10 / 2^12 / 2^14 draws: dn_mt19937_split_device)
    by_size = {}
    for lg in (12, 16, 20, 22):
        if lg > log2n:
            break
        m = 1 << lg
        ss = shamir.SecretShare(3)
        ss.random.seed(lg)
        sm = sec[:m]
        o2 = torch.empty((5, field.vec_bytes(m)), dtype=torch.uint8, device=dev)
        for _ in range(3):  # (the third call waits for the first speculation's side work)
            ss.make_shares_vec(sm, 5, out=o2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            ss.make_shares_vec(sm, 5, out=o2)
        torch.cuda.synchronize()
        by_size[f"2^{lg}"] = (time.perf_counter() - t0) / 20 * 1e3
        del o2
    return {"workload": f"make_shares_vec(2^{log2n} int64, 5) on SecretShare(3), coefficients = the reference's "
                        "MT19937 draws (shamir.py:59-61), bit-exact", "unit": "elements/s",
            "fused_ms": fm * 1e3, "fused_elems_per_s": n / fm, "draw_then_split_ms": um * 1e3,
            "draw_then_split_elems_per_s": n / um, "mt_words_per_s_fused": words / fm,
            "roofline_fused": roof("hbm", n * (8 + 5 * 66) / fm / 1e9,
                                   "8 B secret + 5 x 66 B shares per element (wall time of the whole call)"),
            "fused_ms_by_buffer": [x * 1e3 for x in fused_by_buf],
            "timing": "wall time per call; fused_ms: lone calls (a fresh SecretShare each: nothing to speculate "
                      f"on), the median over three output buffers of the best of {reps} calls on each (after >= "
                      "0.15 s of warm-up calls); loop_ms_per_call: back-to-back calls on one SecretShare, where "
                      "each call's jump level was speculated by the call before (DN_MT_SPEC); fused_ms_by_size: "
                      "20 back-to-back calls on one SecretShare per size after 3 (a loop, speculated from 2^16 "
                      "coefficients where the levels fit beside the generation)",
            "equal_draw_then_split_and_state": ok, "fused_ms_by_size": by_size,
            "loop_ms_per_call": loop}


def reference_digest_equal(block, n: int, name: str) -> bool:
    """SHA-256 checksum of checksums of a share block's limb planes against
    the reference-generated digest `name` (tests/golden/make_golden.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden.fixtures import chunk_digests, combine_digests, manifest

    from delta_node.crypto.shamir import field

    want = [d for d in manifest()["digests"] if d["name"] == name][0]["digest"]
    h = block.cpu().numpy()
    planes = np.stack([field.vec_to_planes(h[s], n) for s in range(h.shape[0])])
    del h
    return combine_digests(chunk_digests(planes)) == want


def _child_json(cmd, timeout: float) -> dict:
    """Run `cmd` as a fresh child process; its last JSON line (or the failure)."""
    import subprocess

    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"error": f"timeout after {timeout} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not lines:
        return {"error": f"exit {r.returncode}: {r.stderr[-400:]}"}
    return json.loads(lines[-1])


def cold_row(log2n: int) -> dict:
    """The first make_shares_vec of a fresh process (scripts/cold_call.py), and
    BASELINE config 5's first round in a fresh runner/peer pair
    (scripts/e2e_round.py --cold): what a reference round, which splits once
    (runner/horizontal/agg.py:142-153), actually pays.  Every other row is warm."""
    py = sys.executable
    e2e = _child_json([py, "scripts/cold_call.py", "--log2n", str(log2n), "--mode", "e2e"], 300)
    phases = _child_json([py, "scripts/cold_call.py", "--log2n", str(log2n), "--mode", "phases"], 300)
    # every probe try misses the keep bar (a fresh process told the fastest rate
    # is unreachable): the share block's tries run until PROBE_TIME_BUDGET
    worst = _child_json([py, "scripts/cold_call.py", "--log2n", str(log2n), "--mode", "e2e", "--force-miss"], 300)
    c5 = _child_json([py, "scripts/e2e_round.py", "--cold", "--rounds", "1", "--coeffs", "mt",
                      "--log2n", str(log2n), "--port", str(free_port())], 600)
    return {"workload": f"first make_shares_vec(2^{log2n} int64, 5) of a fresh process, secrets already on "
                        "the device; wall time to return",
            "cold_ms": e2e.get("first_ms"), "warm_after_ms": e2e.get("second_ms"), "first_call": e2e,
            "cold_worst_ms": worst.get("first_ms"), "cold_worst": worst,
            "phases": phases,
            "config5_first_round": {k: c5.get(k) for k in ("wall_s", "input_MBps", "pack_s", "h2d_s", "split_s",
                                                           "encode_d2h_s", "post_tail_s", "peer_verified", "error")
                                    if k in c5}}


def byte_api_row(budget_s: float = 2.0) -> dict:
    """The call sites the reference actually has (runner/horizontal/agg.py:142-153,
    coord/horizontal/agg.py:296,330,362): make_shares of one 32-byte secret into
    n = 5 / 9 shares and resolve_shares from t of them, per call, beside the
    reference algorithm restated in pure Python on 1 core."""
    import os as _os

    from delta_node.crypto import shamir
    from oracle import py_shamir

    def per_call(fn, budget):
        fn()
        k, t0 = 0, time.perf_counter()
        while True:
            fn()
            k += 1
            dt = time.perf_counter() - t0
            if dt > budget or k >= 20000:
                return dt / k * 1e6

    out = {"unit": "us per call"}
    secret = _os.urandom(32)
    for t, n in ((3, 5), (5, 9)):
        ss = shamir.SecretShare(t)
        ref = py_shamir.RefSecretShare(t, seed=1)
        sh = ss.make_shares(secret, n)
        rsh = ref.make_shares(secret, n)
        ok = ss.resolve_shares(sh[:t]) == ref.resolve_shares(rsh[:t]) == secret.lstrip(b"\0")
        out[f"t{t}n{n}"] = {
            "make_shares_us": per_call(lambda: ss.make_shares(secret, n), budget_s / 8),
            "resolve_shares_us": per_call(lambda: ss.resolve_shares(sh[:t]), budget_s / 8),
            "cpu_reference_make_shares_us": per_call(lambda: ref.make_shares(secret, n), budget_s / 8),
            "cpu_reference_resolve_shares_us": per_call(lambda: ref.resolve_shares(rsh[:t]), budget_s / 8),
            "roundtrip_ok": bool(ok)}
    # the share envelope of the same call sites (runner/horizontal/agg.py:192-196
    # encrypt per share per peer, :258 / :265 decrypt): the byte API on the host
    # (csrc/host_aes.cpp) beside the device route it replaced (H2D, one launch, D2H)
    from delta_node.crypto import aes
    from delta_node.crypto.aes import aes as aes_mod

    key = _os.urandom(32)
    ae = {"unit": "us per call", "host_cipher": aes.host_impl(), "host_max_bytes": aes.HOST_MAX_BYTES}
    for nb in (68, 33):
        data = _os.urandom(nb)
        text = aes.encrypt(key, data)
        dev_text = lambda: bytes(aes.encrypt_vec(key, aes_mod._to_device(data)).cpu().numpy())  # noqa: E731
        ok = aes.decrypt(key, text) == data and aes.decrypt(key, dev_text()) == data
        ae[f"{nb}B"] = {"encrypt_us": per_call(lambda: aes.encrypt(key, data), budget_s / 8),
                        "decrypt_us": per_call(lambda: aes.decrypt(key, text), budget_s / 8),
                        "device_route_encrypt_us": per_call(dev_text, budget_s / 8),
                        "roundtrip_ok": bool(ok)}
    out["aes"] = ae
    return out


def load_traffic(path: str):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launcher_cmd(gpus: int, argv, port: int) -> list:
    """The command `bench.py --gpus N` (N > 1, not already under a launcher)
    runs as a CHILD process: one rank per GPU of this node, rendezvous on
    127.0.0.1, every rank running this file with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(gpus: int, argv) -> int:
    """Run N ranks through torch.distributed.run as a child process (never
    exec), pass its output through, and print rank 0's JSON line as the one
    line on stdout.  Returns the child's exit code.  The parent launches no
    kernel and allocates nothing on a GPU; counting devices may initialise
    the HIP runtime in it (torch.cuda.device_count falls back to
    hipGetDeviceCount without amdsmi), which is harmless because the ranks
    are a separate child process, not an exec of this one."""
    import subprocess

    backend = os.environ.get("DN_DIST_BACKEND", "nccl")
    visible = torch.cuda.device_count()  # may initialise HIP here (see above)
    if backend == "nccl" and gpus > visible:
        print(f"bench.py: --gpus {gpus} with RCCL needs {gpus} visible GPUs, this node has {visible} "
              "(DN_DIST_BACKEND=gloo rehearses the ranks on fewer GPUs)", file=sys.stderr)
        return 2
    proc = subprocess.Popen(launcher_cmd(gpus, argv, free_port()), stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for ln in proc.stdout:
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if line:
        print(line, flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) on this node; without a launcher's WORLD_SIZE, N > 1 starts "
                         "torch.distributed.run with N ranks as a child process")
    ap.add_argument("--placements", type=int, default=5,
                    help="share buffers the timed steps rotate over (separate allocations: the split's rate "
                         "depends on the physical pages of its share buffer, DESIGN.md §5.1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2n", type=int, default=24, help="elements of the vector = 2^log2n (sharded over the ranks)")
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--shares", type=int, default=5)
    ap.add_argument("--xs", type=str, default="1,3,5")
    ap.add_argument("--cpu-budget", type=float, default=16.0,
                    help="seconds of CPU baseline sampling, half 1-core, half 16-process (0 = skip)")
    ap.add_argument("--allgather", action="store_true", help="also time the RCCL all-gather of share blocks (N>1)")
    ap.add_argument("--rows", type=int, default=1, help="also measure the SURVEY §8(f) rows built so far")
    ap.add_argument("--traffic", type=str, default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--config4", type=int, default=1, help="also run BASELINE config 4 (5-of-9 split of 2^26 "
                                                            "sharded over the ranks + RCCL all-gather)")
    ap.add_argument("--config4-log2n", type=int, default=26, help="config 4 total elements = 2^this")
    ap.add_argument("--config5", type=int, default=1, help="also run BASELINE config 5 (end-to-end round over "
                                                            "loopback HTTP to a second process; N=1 only)")
    ap.add_argument("--events", choices=("nofence", "torch"), default="nofence",
                    help="timing events of the timed steps: HIP events without the system-scope fence "
                         "(TimingEvent, default) or torch.cuda.Event (a fence, i.e. an L2 write-back, per record)")
    ap.add_argument("--cold", type=int, default=1, help="also time the first make_shares_vec / config-5 round "
                                                         "of fresh processes (with --rows; N=1 only)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if (args.gpus or 1) > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under a launcher the ranks form a process group even at WORLD_SIZE=1, so
    # the collective code paths (RCCL under nccl) run at every N
    dist_on = "WORLD_SIZE" in os.environ
    if dist_on:
        import torch.distributed as dist

        # DN_DIST_BACKEND=gloo rehearses the multi-rank control flow on a
        # 1-GPU box (ranks share cuda:0); the product path is nccl (RCCL).
        backend = os.environ.get("DN_DIST_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", torch.cuda.current_device())
    # small control-plane tensors (timings, parity flags): device under nccl, host under gloo
    cdev = dev if not dist_on or torch.distributed.get_backend() == "nccl" else torch.device("cpu")

    from delta_node.crypto import shamir
    from delta_node.crypto.shamir import _native, field, memory
    from delta_node.crypto.shamir import dist as sdist

    N_total = 1 << args.log2n
    t, n = args.t, args.shares
    xs = [int(x) for x in args.xs.split(",")]
    # Strong scaling (BASELINE metric: ONE 2^24 vector): rank r
    # owns the tile-aligned range shard_range(N_total, r, world) of it.
    lo, hi = sdist.shard_range(N_total, rank, world) if world > 1 else (0, N_total)
    N = hi - lo

    def barrier():
        if dist_on:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # ---- inputs resident in HBM (untimed) ---------------------------------
    # secrets: one synthetic vector; coefficients: the reference's MT19937
    # stream for the WHOLE vector (N make_shares calls on one instance), each
    # rank drawing only its shard on its GPU (dist.draw_coeffs_sharded)
    ss = shamir.SecretShare(t)
    ss.random.seed(1)
    sec_h = secrets_int64(1, N_total)[lo:hi].copy()
    sec = torch.from_numpy(sec_h).to(dev)
    vb = field.vec_bytes(N)
    if dist_on:
        coeffs = sdist.draw_coeffs_sharded(ss, N_total, dev)[:, :vb].contiguous()
    else:
        coeffs = ss.draw_coeffs_vec(N_total, dev)
    # The steps rotate over `nbuf` separately allocated share buffers (step i
    # writes buffer i mod nbuf and reconstructs from it): the split's rate is
    # a property of its share buffer's physical pages, so
    # the timed average is over several placements, not one allocation's.
    nbuf = max(1, args.placements)
    # each the block make_shares_vec returns for out=None (memory.share_block:
    # pooled 16 MiB physical chunks; torch.empty below 64 MiB)
    share_bufs = [memory.share_block((n, vb), dev) for _ in range(nbuf)]
    rec = torch.empty(N, dtype=torch.int64, device=dev)
    w = _native.lagrange(xs, t)
    row_sets = [[sb[x - 1] for x in xs] for sb in share_bufs]
    for sb in share_bufs:  # first touch of every buffer, before the warm-up
        _native.split_u64(sec, coeffs, sb, N, t, n)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    # HIP events on the launch stream bracket every kernel of the timed steps:
    # three per step (before the split, between split and reconstruct, after
    # the reconstruct), so each kernel's time excludes the host's launch gap
    # before the next step (reported apart as step_gap_ms).  They
    # are TimingEvents (no system-scope fence per record: torch's events cost
    # ~4-5 us of stream time each at 2^21, r05g).
    def step(i, ev=None):
        b = i % nbuf
        if ev:
            ev[0].record(stream)
        _native.split_u64(sec, coeffs, share_bufs[b], N, t, n)
        if ev:
            ev[1].record(stream)
        _native.reconstruct(row_sets[b], w, out_u64=rec, n=N)
        if ev:
            ev[2].record(stream)

    def timed_steps(fn, steps):
        for i in range(args.warmup):
            fn(i)
        barrier()
        mk = TimingEvent if args.events == "nofence" else (lambda: torch.cuda.Event(enable_timing=True))
        evs = [[mk() for _ in range(3)] for _ in range(steps)]
        end = mk()
        barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i, evs[i])
        end.record(stream)
        barrier()
        el = time.perf_counter() - t0
        if dist_on:
            tt = torch.tensor([el], dtype=torch.float64, device=cdev)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            el = float(tt.item())
        return el, evs + [[end]]

    elapsed, evs = timed_steps(step, args.steps)
    split_each = [evs[i][0].elapsed_time(evs[i][1]) for i in range(args.steps)]
    split_ms = float(np.mean(split_each))
    recon_ms = float(np.mean([evs[i][1].elapsed_time(evs[i][2]) for i in range(args.steps)]))
    # stream time between one step's reconstruct and the next step's split (host launch gaps)
    gap_ms = float(np.mean([evs[i][2].elapsed_time(evs[i + 1][0]) for i in range(args.steps - 1)])) \
        if args.steps > 1 else None
    split_by_buf = [float(np.mean(split_each[b::nbuf])) for b in range(min(nbuf, args.steps))]

    # ---- parity of what was timed (cheap, size-independent + sampled) -----
    last = (args.steps - 1) % nbuf if args.steps else 0
    shares = share_bufs[last]
    share_rows = row_sets[last]
    roundtrip = bool(torch.equal(rec, sec))
    sample = min(2048, N)
    from oracle import c_oracle

    co_h = np.stack([field.vec_to_limbs(coeffs[j, : field.vec_bytes(sample)].cpu().numpy(), sample)
                     for j in range(t - 1)], axis=1)
    want = c_oracle.split(sec_h[:sample], co_h, t, n)
    got = np.stack([field.vec_to_limbs(shares[x, : field.vec_bytes(sample)].cpu().numpy(), sample) for x in range(n)])
    oracle_ok = bool(np.array_equal(got, want))
    bufs_equal = all(bool(torch.equal(sb, shares)) for sb in share_bufs)
    # the headline workload IS the reference's split_t3n5_2e24 digest case
    # (secrets_int64(1, 2^24), random.seed(1)): the timed share block's digest
    # against the one the reference itself produced (tests/golden/manifest.json)
    ref_digest_ok = None
    if world == 1 and N_total == (1 << 24) and (t, n) == (3, 5):
        ref_digest_ok = reference_digest_equal(shares, N, "split_t3n5_2e24")
    all_ok = roundtrip and oracle_ok and bufs_equal and ref_digest_ok is not False
    if dist_on:  # every rank's parity, not only rank 0's
        fl = torch.tensor([int(all_ok)], dtype=torch.int32, device=cdev)
        torch.distributed.all_reduce(fl, op=torch.distributed.ReduceOp.MIN)
        all_ok = bool(fl.item())

    # ---- same-buffer ceilings: the split's bytes through the same pages ----
    split_bytes = N * (8 + (t - 1) * FE_BYTES + n * FE_BYTES)
    placement = None
    ceiling = recon_ceiling = None
    if N >= (1 << 20):
        fr = [split_bytes / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS for ms in split_by_buf]
        # the same split into blocks a caller allocates (before the ceiling
        # probes, which overwrite the timed blocks: the equality check needs them)
        caller = caller_blocks_row(sec, coeffs, N, t, n, nbuf, stream, split_bytes, shares) if world == 1 else None
        ceils = [measure_ceiling(dev, sec, coeffs, share_bufs[b], N, t, n) for b in range(len(split_by_buf))]
        placement = {"buffers": len(split_by_buf), "steps_per_buffer": args.steps // max(1, nbuf),
                     "split_ms": split_by_buf, "frac": fr, "frac_min": min(fr), "frac_median": float(np.median(fr)),
                     "frac_max": max(fr), "n_frac_ge_0_70": sum(f >= 0.70 for f in fr),
                     "ceiling_ms": [c["ms"] for c in ceils],
                     "split_frac_of_ceiling": [c["ms"] / ms for c, ms in zip(ceils, split_by_buf)],
                     # memory.share_block's allocation-time fill probe of each block (TB/s; None: not probed)
                     "probed_write_TBps": [(memory.block_rate(sb) or 0.0) / 1e12 or None for sb in share_bufs],
                     "pool": memory.pool_stats()}
        # over the same buffers the timed average covers: mean of their ceilings
        ceiling = {"ms": float(np.mean([c["ms"] for c in ceils])), "grid": [c["grid"] for c in ceils],
                   "kernel": ceils[0]["kernel"], "buffers": len(ceils)}
        recon_ceiling = measure_recon_ceiling(share_rows, rec, N)
        if caller:
            placement["caller_blocks"] = caller
    del share_bufs, row_sets

    # ---- N > 1: the weak-scaling figure (2^log2n elements per GPU) --------
    weak = None
    if world > 1:
        del shares, coeffs, share_rows, rec, sec
        torch.cuda.empty_cache()
        ssw = shamir.SecretShare(t)
        ssw.random.seed(1 + rank)
        wsec = torch.from_numpy(secrets_int64(1 + rank, N_total)).to(dev)
        wco = ssw.draw_coeffs_vec(N_total, dev)
        wsh = torch.empty((n, field.vec_bytes(N_total)), dtype=torch.uint8, device=dev)
        wrec = torch.empty(N_total, dtype=torch.int64, device=dev)
        wrows = [wsh[x - 1] for x in xs]

        def wstep(i, ev=None):
            _native.split_u64(wsec, wco, wsh, N_total, t, n)
            _native.reconstruct(wrows, w, out_u64=wrec, n=N_total)

        wel, _ = timed_steps(wstep, args.steps)
        wok = torch.tensor([int(torch.equal(wrec, wsec))], dtype=torch.int32, device=cdev)
        torch.distributed.all_reduce(wok, op=torch.distributed.ReduceOp.MIN)
        weak = {"value": N_total * world * args.steps / wel, "unit": "elements/s", "elements_per_gpu": N_total,
                "ms_per_step": wel / args.steps * 1e3, "scaling": "weak", "roundtrip_all_ranks": bool(wok.item())}
        del wsec, wco, wsh, wrec, wrows
        torch.cuda.empty_cache()

    # ---- optional: RCCL all-gather of share blocks (reported separately) --
    allgather = None
    if args.allgather and world > 1:
        shb = torch.zeros((n, sdist.shard_tiles(N_total, world) * field.TILE_BYTES), dtype=torch.uint8, device=dev)
        for _ in range(2):
            sdist.allgather_share_blocks(shb, N_total)
        barrier()
        g0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            full = sdist.allgather_share_blocks(shb, N_total)
        barrier()
        gdt = (time.perf_counter() - g0) / reps
        recv = shb.numel() * (world - 1)
        allgather = {"ms": gdt * 1e3, "bytes_received_per_gpu": recv, "GBps_per_gpu": recv / gdt / 1e9}
        del full, shb

    # ---- report -------------------------------------------------------------
    value = N_total * args.steps / elapsed
    split_bytes = N * (8 + (t - 1) * FE_BYTES + n * FE_BYTES)
    recon_bytes = N * (len(xs) * FE_BYTES + 8)
    achieved = split_bytes / (split_ms * 1e-3) / 1e9
    traffic = load_traffic(args.traffic)
    line = {
        "metric": "elements/s device-resident Shamir 3-of-5 split+recombine, 2^24 vec, 1/2/4/8 GPU",
        "value": value,
        "unit": "elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic int64 secrets (numpy PCG64) + MT19937 coefficients drawn as make_shares draws them",
        "config": {"workload": f"{t}-of-{n} split + reconstruct(xs={xs}) of one 2^{args.log2n}-element int64 "
                               f"vector, GF(2^521-1), sharded by element over {world} GPU(s)",
                   "elements_total": N_total, "elements_per_gpu": N, "threshold": t, "shares": n, "xs": xs,
                   "parallelism": f"element-shard x{world}",
                   "share_blocks": "memory.share_block (make_shares_vec's own output allocation: pooled 16 MiB "
                                   "physical chunks)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBPS,
                     # PMC bytes of the headline launch (2^24, 3-of-5) from the committed counter
                     # passes (not collected by this run); null for other sizes
                     "traffic": ((traffic or {}).get("split_bytes_per_launch")
                                 if abs((traffic or {}).get("split_bytes_per_launch", 0) - split_bytes)
                                 < 0.01 * split_bytes else None),
                     "traffic_source": (traffic or {}).get("source", os.path.relpath(args.traffic, ROOT)),
                     "kernel": "dn::split_kernel<3, false, false, false, 2>",
                     "algorithmic_bytes_per_launch": split_bytes, "avg_launch_ms": split_ms,
                     "avg_over": f"{args.steps} timed launches rotating over {nbuf} share buffers",
                     "events": ("HIP events with hipEventDisableSystemFence on the launch stream"
                                if args.events == "nofence" else "torch.cuda.Event (system-scope fence per record)"),
                     "placement": placement,
                     # blocks memory.share_block mapped, probed and rejected for this run's share
                     # blocks (the probe-and-discard cost of the fractions above)
                     "probe_rejected_blocks": placement and placement["pool"]["rejected"],
                     "caller_blocks_frac_mean_time": placement and placement.get("caller_blocks", {}).get(
                         "frac_mean_time"),
                     "ceiling_measured": ceiling and {
                         **ceiling, "GBps": split_bytes / (ceiling["ms"] * 1e-3) / 1e9,
                         "split_frac_of_ceiling": ceiling["ms"] / split_ms}},
        "kernels": {"split_ms": split_ms, "reconstruct_ms": recon_ms, "step_gap_ms": gap_ms,
                    "split_GBps": achieved, "reconstruct_GBps": recon_bytes / (recon_ms * 1e-3) / 1e9,
                    "split_elems_per_s": N / (split_ms * 1e-3), "reconstruct_elems_per_s": N / (recon_ms * 1e-3),
                    "reconstruct_ceiling_measured": recon_ceiling and {
                        **recon_ceiling, "GBps": recon_bytes / (recon_ceiling["ms"] * 1e-3) / 1e9,
                        "reconstruct_frac_of_ceiling": recon_ceiling["ms"] / recon_ms}},
        "parity": {"roundtrip_equal": roundtrip, "c_oracle_sample_equal": oracle_ok, "sample": sample,
                   "reference_digest_equal": ref_digest_ok, "all_ranks_ok": all_ok},
        # share blocks memory.share_block mapped, write-probed and freed to place
        # this run's timed blocks (their fractions: roofline.placement; the same
        # split on caller-allocated blocks: roofline.placement.caller_blocks)
        "probe_rejected_blocks": placement and placement["pool"]["rejected"],
    }
    if weak:
        line["weak_scaling"] = weak
    if allgather:
        line["allgather"] = allgather
    if args.config4:
        if world == 1:
            del shares, coeffs, share_rows
        torch.cuda.empty_cache()
        line["config4"] = config4_bench(dev, world, rank, args.config4_log2n, dist_on=dist_on)
    if args.rows and world == 1:
        line["rows"] = rows_bench(dev, args.log2n)
        line["rows"]["draw_split"] = draw_split_row(dev, args.log2n)
        if args.cold:
            line["rows"]["draw_split"]["cold"] = cold_row(args.log2n)
        line["rows"]["byte_api"] = byte_api_row()
    if args.config5 and world == 1:
        line["config5"] = config5_bench(args.log2n)
    if args.cpu_budget > 0:
        # the reference CPU path timed on this host in the same run, at every
        # N (north_star): after all GPU work, rank 0 only, while the other
        # ranks wait at a barrier (their GPU work is done; their cores idle)
        if dist_on:
            barrier()
        if rank == 0:
            procs = min(16, max(1, (os.cpu_count() or 16) // world))
            line["cpu_baseline"] = cpu_baseline(t, n, xs, args.cpu_budget, procs=procs)
            line["cpu_baseline"]["run_at_world_size"] = world
        if dist_on:
            barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()
    if not all_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
