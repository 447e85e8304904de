"""`delta_node.utils` subset on the masking path.

Reference: delta_node/utils/__init__.py re-exports arr.py (make_mask) and
precision.py (fix_precision / unfix_precision) among others; the
commitment / MiMC7 helpers are not provided here.
"""
from .agg import allreduce_sum, sum_int64, sum_member_results
from .arr import make_mask, make_mask_tensor
from .mask import masked_sum, unmasked_values
from .precision import fix_precision, unfix_precision

__all__ = ["make_mask", "make_mask_tensor", "fix_precision", "unfix_precision", "masked_sum", "unmasked_values",
           "sum_int64", "sum_member_results", "allreduce_sum"]
