#!/usr/bin/env python3
"""ISA checks over the product kernels (run by `make -C delta-node_amd isa-check`).

For every device source, compile to gfx950 assembly and flag
  * waterfall loops around memory instructions: a v_readfirstlane shortly
    before a buffer/global access that is followed by an exec-mask loop back
    edge — the compiler could not prove an address or buffer descriptor
    wave-uniform (cost 1.4x on the fused draw + split before it was fixed);
  * scratch (private segment) use and the VGPR count of every kernel.
Exit status 1 if any waterfall loop is found.
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "delta-node_amd")
SRCS = ["shamir_m521", "codec_m521", "aes_envelope", "mask_pcg64", "sum_i64", "mimc7_bn254", "mt19937_device"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def scan(asm: str):
    lines = asm.split("\n")
    kern, hits, info = None, {}, {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z[^:\s]+):", l)
        if m:
            kern = m.group(1)
        m = re.match(r"^\s*\.set (_Z\S+)\.(num_vgpr|private_seg_size), (\d+)", l)
        if m:
            info.setdefault(m.group(1), {})[m.group(2)] = int(m.group(3))
        t = l.strip()
        if kern and t.startswith(("buffer_", "global_", "flat_")):
            nxt = " ".join(x.strip() for x in lines[i + 1:i + 4])
            back = " ".join(x.strip() for x in lines[max(0, i - 12):i])
            if ("s_xor_b64 exec" in nxt or "s_cbranch_execnz" in nxt) and "v_readfirstlane" in back:
                hits[kern] = hits.get(kern, 0) + 1
    return hits, info


def main() -> int:
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for src in SRCS:
            out = os.path.join(td, src + ".s")
            subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(PKG, "..", "include"),
                            "-I" + os.path.join(PKG, "csrc"), "-S", "--cuda-device-only",
                            os.path.join(PKG, "csrc", src + ".hip"), "-o", out], check=True)
            hits, info = scan(open(out).read())
            for k, v in sorted(info.items()):
                flag = " SCRATCH" if v.get("private_seg_size") else ""
                print(f"{src:16s} vgpr={v.get('num_vgpr', '?'):>3} scratch={v.get('private_seg_size', 0):>4}{flag} {k[:90]}")
            for k, n in hits.items():
                print(f"WATERFALL {src}: {n} memory instructions in exec-mask loops in {k[:90]}")
                bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
