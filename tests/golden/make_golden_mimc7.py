#!/usr/bin/env python3
"""Extract the MiMC7 known-answer vectors of the reference's tests (data only).

The reference cannot run here (delta_node/utils/mimc7.py imports gmpy2, which
is not installed), so its own KATs — tests/mimc7_test.py:5-97: mimc7_hash(1, 0),
the weight commitment of 3 floats and the data commitment of a 32x4 dataset —
pin the oracle (oracle/py_mimc7.py).  This script reads the literal inputs
and expected outputs out of that test file with `ast` and writes them to
tests/golden/mimc7_kat.json; nothing of the reference's code is kept.
"""
import ast
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/tests/mimc7_test.py"


def main():
    tree = ast.parse(open(SRC).read())
    consts, arrays = [], []
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and len(node.value) > 40:
            consts.append(node.value)
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "array":
            arrays.append(ast.literal_eval(node.args[0]))
        if isinstance(node, ast.Assign) and isinstance(node.value, ast.List) and \
                getattr(node.targets[0], "id", "") == "weight":
            weight = ast.literal_eval(node.value)
    x, y = arrays[0], arrays[1]
    kat = {
        "source": "reference tests/mimc7_test.py (values only)",
        "hash_1_0": consts[0],
        "weight": weight, "weight_commitment": consts[1],
        "data_x": x, "data_y": y, "data_commitment": consts[2],
    }
    json.dump(kat, open(os.path.join(HERE, "mimc7_kat.json"), "w"), indent=1)
    print({k: (v if not isinstance(v, list) else f"{len(v)} items") for k, v in kat.items()})


if __name__ == "__main__":
    main()
