"""`delta_node.crypto` subset: the Shamir secret-sharing hot path and the AES share envelope."""
