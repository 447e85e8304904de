from .shamir import *  # noqa: F401,F403  (reference: delta_node/crypto/shamir/__init__.py:1)
