"""MI355X-native drop-in for delta-node's secret-sharing hot path.

Only the packages on that path and either side of it exist here:
`delta_node.crypto.shamir` (the reference surface,
delta_node/crypto/shamir/__init__.py:1), `delta_node.crypto.aes` (the share
envelope, crypto/aes/aes.py:8-23), `delta_node.serialize` (serialize/hex.py)
and `delta_node.utils` (masks, fixed point, member sums, MiMC7).
"""
