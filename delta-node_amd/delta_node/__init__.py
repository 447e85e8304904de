"""MI355X-native drop-in for delta-node's secret-sharing hot path.

Only the packages on that path exist here: `delta_node.crypto.shamir` (the
reference surface, delta_node/crypto/shamir/__init__.py:1) and the two
`delta_node.serialize` helpers it depends on (delta_node/serialize/hex.py:44-50).
"""
