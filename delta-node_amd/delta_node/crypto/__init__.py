"""`delta_node.crypto` subset: the Shamir secret-sharing hot path only."""
