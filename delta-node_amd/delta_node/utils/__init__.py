"""`delta_node.utils` (reference: delta_node/utils/__init__.py:1-15).

Same exports as the reference: make_mask, fix_precision, unfix_precision,
calc_commitment, constant, calc_weight_commitment, calc_data_commitment —
plus this package's device-side helpers of the masking / aggregation path
(make_mask_tensor, masked_sum, unmasked_values, sum_int64,
sum_member_results, allreduce_sum) and the npz helpers load_arr / dump_arr.
"""
from . import constant
from .agg import allreduce_sum, sum_int64, sum_member_results
from .arr import dump_arr, load_arr, make_mask, make_mask_tensor
from .commitment import calc_commitment
from .mask import masked_sum, unmasked_values
from .mimc7 import calc_data_commitment, calc_weight_commitment
from .precision import fix_precision, unfix_precision

__all__ = ["make_mask", "fix_precision", "unfix_precision", "calc_commitment", "constant",
           "calc_weight_commitment", "calc_data_commitment",
           "make_mask_tensor", "masked_sum", "unmasked_values", "sum_int64", "sum_member_results", "allreduce_sum",
           "load_arr", "dump_arr"]
