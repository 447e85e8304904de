"""Load the reference `delta_node.crypto.shamir` by file path (fixture generation only).

Used ONLY by `make_golden.py`, in the build container where `/root/reference`
exists.  Nothing on the GPU box imports this: the reference never travels.

Why a shim: `import delta_node.crypto.shamir` fails in the reference because
`delta_node/serialize/__init__.py:1` -> `serialize/agg.py:6` imports the absent
`delta` (delta-task) package.  The hot path itself only needs
`serialize/hex.py:44-50` (`int_to_bytes`/`bytes_to_int`), `crypto/shamir/op.py`
and `crypto/shamir/shamir.py`, so those three files are loaded directly and
registered under the module names `shamir.py` imports them by
(`from delta_node import serialize`, `from . import op`).
"""
import importlib.util
import sys
import types

REF = "/root/reference/delta_node"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference_shamir():
    """Return the reference `delta_node.crypto.shamir.shamir` module."""
    if "delta_node.crypto.shamir.shamir" in sys.modules:
        return sys.modules["delta_node.crypto.shamir.shamir"]
    pkg = types.ModuleType("delta_node")
    pkg.__path__ = [REF]
    sys.modules["delta_node"] = pkg
    ser = _load("delta_node.serialize", f"{REF}/serialize/hex.py")
    pkg.serialize = ser
    crypto = types.ModuleType("delta_node.crypto")
    crypto.__path__ = [f"{REF}/crypto"]
    sys.modules["delta_node.crypto"] = crypto
    sh = types.ModuleType("delta_node.crypto.shamir")
    sh.__path__ = [f"{REF}/crypto/shamir"]
    sys.modules["delta_node.crypto.shamir"] = sh
    crypto.shamir = sh
    op = _load("delta_node.crypto.shamir.op", f"{REF}/crypto/shamir/op.py")
    sh.op = op
    mod = _load("delta_node.crypto.shamir.shamir", f"{REF}/crypto/shamir/shamir.py")
    return mod
