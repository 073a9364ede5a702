"""ctypes binding of libtuplewise.so (the C ABI declared in include/tuplewise.h).

This module is the only place the package touches the native library.  It fails loudly:
there is no CPU fallback for any hot-path computation — a missing library or a machine
without a HIP device raises instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import sys

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
# TW_LIB_PATH: an A/B build of the same library (tools/ab_barrier.py), never the product default
LIB_PATH = pathlib.Path(os.environ["TW_LIB_PATH"]) if os.environ.get("TW_LIB_PATH") else (
    _HERE / "libtuplewise.so")

TW_OK, TW_ERR_ARG, TW_ERR_HIP = 0, 1, 2
TW_F64, TW_I64 = 0, 1
TW_PRED_GT, TW_PRED_HALF, TW_PRED_SUBGT = 0, 1, 2
TW_KERN_PROD, TW_KERN_GINI, TW_KERN_HINGE, TW_KERN_LOGISTIC = 0, 1, 2, 3
TW_LOSS_HINGE, TW_LOSS_LOGISTIC = 0, 1

_vp, _i64, _i32, _u64, _f64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                               ctypes.c_uint64, ctypes.c_double)

# name -> argtypes (all return int status unless listed in _RESTYPES)
_SIGNATURES = {
    "tw_last_error": [],
    "tw_version": [],
    "tw_device_count": [_vp],
    "tw_count_pairs": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _i32, _vp, _vp],
    "tw_count_pairs_step": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _i32, _vp, _i64, _vp,
                            _u64, _i64, _vp, _u64, _vp, _i32, _vp],
    "tw_count_step_set_plan": [_i32, _i32, _i32],
    "tw_count_set_scalar_mix": [_i32],
    "tw_count_set_plan": [_i32, _i64],
    "tw_rank_images_work_bytes": [_i64, _i64],
    "tw_rank_images": [_vp, _i64, _vp, _i64, _i32, _vp, _i64, _vp, _vp, _vp],
    "tw_count_pairs_rank_step": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _vp, _i64, _vp, _u64,
                                 _i64, _vp, _u64, _vp, _i32, _vp],
    "tw_gather_records": [_vp, _vp, _i64, _vp, _vp],
    "tw_count_rank_set_plan": [_i32, _i64],
    "tw_count_rank_set_next": [_i32],
    "tw_rank_set_plan": [_i32, _i32],
    "tw_rank_set_small": [_i32, _i32, _i32],
    "tw_rank_images_query": [_vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _vp, _i64, _vp, _vp,
                             _vp],
    "tw_chain_emit": [_vp, _i64, _vp, _i64, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32,
                      _i64, _i64, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp],
    "tw_chain_unpack": [_vp, _i32, _i32, _i64, _i32, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp,
                        _vp],
    "tw_count_pairs_chain": [_vp, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i64, _i64, _i32, _vp,
                             _vp],
    "tw_count_pairs_chain_bucket": [_vp, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i64, _i64,
                                    _i32, _vp, _vp],
    "tw_count_chain_set_plan": [_i32, _i64],
    "tw_chain_set_emit": [_i32, _i32],
    "tw_chain_scatter": [_vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp],
    "tw_chain_gather": [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp,
                        _vp, _vp],
    "tw_chain_gather2": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _i32,
                         _vp, _vp, _vp, _vp, _vp, _vp],
    "tw_count_pairs_sorted_work_bytes": [_i32, _i64],
    "tw_count_sorted_set_chunk": [_i64],
    "tw_count_pairs_sorted": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _i32, _vp, _vp, _vp],
    "tw_count_pairs_idx": [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _vp],
    "tw_count_idx_set_parts": [_i32],
    "tw_count_idx_set_variant": [_i32],
    "tw_count_pairs_idx_ws": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _i64, _i32,
                              _i32, _vp, _i64, _vp, _vp],
    "tw_count_pairs_idx32": [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _vp],
    "tw_count_pairs_idx32_ws": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _i64, _i32,
                                _i32, _vp, _i64, _vp, _vp],
    "tw_count_pairs_rng": [_vp, _vp, _vp, _vp, _i32, _i64, _u64, _u64, _i32, _i32, _vp, _vp],
    "tw_count_pairs_rng_work_bytes": [_i32, _i64, _i64, _i32, _i32],
    "tw_count_rng_set_codes": [_i32],
    "tw_count_img_set_plan": [_i32, _i32],
    "tw_count_sorted_set_bucket": [_i32],
    "tw_count_pairs_rng_ws": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _u64, _u64, _i32, _i32,
                              _vp, _i64, _vp, _vp],
    "tw_count_pairs_sorted_steps_work_bytes": [_i64, _i64, _i32, _i64, _i32, _i32],
    "tw_count_pairs_sorted_steps": [_vp, _vp, _i64, _i64, _vp, _vp, _i32, _i64, _i64, _i64, _i64,
                                    _i32, _i32, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _vp, _vp],
    "tw_count_pairs_sorted_step": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _i32, _vp, _vp,
                                   _i64, _vp, _u64, _i64, _vp, _u64, _vp, _i32, _vp],
    "tw_count_pairs_rng_step": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _u64, _u64, _i32,
                                _i32, _vp, _i64, _vp, _i64, _vp, _u64, _i64, _vp, _u64, _vp,
                                _i32, _vp],
    "tw_pair_sum_work_per_shard": [_i64, _i64],
    "tw_pair_sum_f64": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _f64, _vp, _vp, _vp],
    "tw_pair_sum_idx_work_per_shard": [_i64],
    "tw_pair_sum_idx_f64": [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _f64, _vp, _vp, _vp],
    "tw_pair_sum_idx32_f64": [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _f64, _vp, _vp, _vp,
                              _vp],
    "tw_hinge_grad": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i64, _vp, _f64,
                      _vp, _vp],
    "tw_pair_grad": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i64, _vp, _f64, _i32,
                     _vp, _vp],
    "tw_pair_grad_audit": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i64, _vp, _f64,
                           _i32, _vp, _vp, _vp],
    "tw_pair_grad_complete_work_bytes": [_i32, _i64, _i64, _i64],
    "tw_pair_grad_complete_set_search": [_i32],
    "tw_pair_grad_complete": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _vp, _f64, _i32, _vp,
                              _vp, _vp],
    "tw_pair_grad_rng": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _vp, _f64, _i32, _u64,
                         _vp, _i32, _vp, _vp],
    "tw_hinge_grad_rng": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _vp, _f64, _u64,
                          _vp, _i32, _vp, _vp],
    "tw_hinge_set_variant": [_i32],
    "tw_swr_rows_rng": [_vp, _i32, _i64, _i64, _u64, _vp, _i32, _i32, _vp],
    "tw_sgd_update": [_vp, _vp, _vp, _i32, _i64, _f64, _f64, _f64, _vp, _vp],
    "tw_sgd_update_to": [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _f64, _f64, _f64, _vp, _i32, _vp],
    "tw_sgd_step_fusable": [_i64, _i32],
    "tw_sgd_step": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i64, _f64, _i32, _u64,
                    _vp, _i32, _i32, _vp, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _vp],
    "tw_count_rng_img_set_unroll": [_i32],
    "tw_sgd_segment_narrow_ok": [_i64, _i32, _i64],
    "tw_sgd_segment_narrow": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32, _i64,
                              _f64, _i32, _u64, _vp, _i32, _i32, _vp, _vp, _f64, _f64, _f64, _vp,
                              _vp, _vp, _vp, _vp, _vp],
    "tw_sgd_segment_narrow_tables": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i64,
                                     _i64, _vp, _vp, _i64, _i32, _i64, _f64, _i32, _u64, _vp,
                                     _i32, _i32, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _vp,
                                     _vp, _vp],
    "tw_pair_grad_rng_swr": [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i64, _vp, _f64,
                             _i32, _u64, _vp, _i32, _i64, _u64, _vp, _vp],
    "tw_sgd_segment_narrow_swr": [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i64, _f64,
                                  _i32, _u64, _vp, _i32, _i32, _i64, _u64, _vp, _vp, _f64,
                                  _f64, _f64, _vp, _vp, _vp, _vp, _vp, _vp],
    "tw_peer_buffer_bytes": [_i32, _i64],
    "tw_peer_alloc": [_i64, _vp, _vp],
    "tw_peer_free": [_vp],
    "tw_peer_handle": [_vp, _vp],
    "tw_peer_open": [_vp, _vp],
    "tw_peer_close": [_vp],
    "tw_peer_hello": [_vp, _i32, _i32, _u64, _vp],
    "tw_peer_check": [_vp, _i32, _u64, _vp],
    "tw_peer_step": [_vp, _i64, _i64, _vp, _i32, _i32, _i32, _i64, _i32, _vp, _vp, _f64, _f64,
                     _f64, _vp, _vp, _vp],
    "tw_peer_step_cols": [_vp, _i64, _i64, _vp, _i32, _i32, _i32, _i64, _i32, _vp, _vp, _f64,
                          _f64, _f64, _vp, _vp, _vp],
    "tw_sgd_segment_narrow_peer": [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32,
                                   _i64, _f64, _i32, _u64, _vp, _i32, _i32, _i64, _i64, _i64,
                                   _vp, _vp, _f64, _f64, _f64, _vp, _vp, _i32, _i32, _i32, _vp],
    "tw_gemv_f64": [_vp, _i64, _i64, _vp, _vp, _vp],
    "tw_gemv_set_variant": [_i32],
    "tw_pair_hinge_sum_sorted_work_bytes": [_i32, _i64, _i64],
    "tw_pair_hinge_sum_sorted": [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _f64, _vp, _vp, _vp],
    "tw_permute_scatter": [_vp, _vp, _i64, _u64, _vp],
    "tw_permute_pair": [_vp, _vp, _i64, _u64, _vp, _vp, _i64, _u64, _vp],
    "tw_perm_index": [_vp, _i64, _i64, _i64, _u64, _vp],
    "tw_rank_histogram": [_vp, _i64, _i64, _i32, _vp, _vp],
    "tw_source_histogram": [_i64, _i64, _i64, _u64, _i64, _i32, _vp, _vp],
    "tw_bucket_scatter": [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _i64, _vp, _vp],
    "tw_scatter_records": [_vp, _i64, _vp, _vp],
    "tw_exchange_set_grid": [_i32],
    "tw_exchange_counts": [_i64, _i64, _i32, _i32, _u64, _u64, _vp, _vp, _vp],
    "tw_exchange_pack": [_vp, _i64, _vp, _i64, _i32, _i32, _u64, _u64, _vp, _vp, _vp, _vp],
    "tw_exchange_pack_fixed": [_vp, _i64, _vp, _i64, _i32, _i32, _u64, _u64, _i64, _vp, _vp, _vp,
                               _vp],
    "tw_scatter_buckets": [_vp, _i32, _i64, _vp, _i64, _vp, _vp],
    "tw_row_route_counts": [_vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp],
    "tw_row_pack": [_vp, _i64, _i64, _i64, _i64, _i32, _vp, _i64, _vp, _vp, _vp, _vp],
    "tw_row_unpack": [_vp, _i64, _i64, _vp, _vp],
    "tw_row_route_remote_counts": [_vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _vp],
    "tw_row_pack_remote": [_vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _i64, _vp, _vp, _vp,
                           _vp, _vp],
    "tw_row_table_local": [_vp, _i64, _i64, _i64, _vp, _vp],
    "tw_row_table_remote": [_vp, _i32, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp,
                            _vp],
    "tw_comm_init": [_i32, _vp, _vp],
    "tw_comm_destroy": [_i32],
    "tw_allgather_u64": [_i32, _vp, _vp, _i64, _vp],
    "tw_allgather_f64": [_i32, _vp, _vp, _i64, _vp],
    "tw_comm_wait": [_i32, _vp, _i64],
    "tw_comm_set_timeout": [_i64],
    "tw_comm_set_prior_timeout": [_i64],
    "tw_np_randint_batch": [_vp, _vp, _i32, _vp, _vp, _vp, _vp],
    "tw_np_mt_next32": [_vp, _vp, _i64, _vp],
    "tw_np_randint_pairs": [_vp, _vp, _i32, _i64, _i64, _i64, _vp, _vp],
    "tw_np_randint_pairs_steps": [_vp, _vp, _i32, _i32, _i64, _i64, _i64, _vp],
    "tw_np_randint_pairs_steps_u16": [_vp, _vp, _i32, _i32, _i64, _i64, _i64, _vp],
    "tw_widen_u16": [_vp, _i64, _vp, _vp],
    "tw_np_randint_pairs_steps_u8": [_vp, _vp, _i32, _i32, _i64, _i64, _i64, _vp],
    "tw_widen_u8": [_vp, _i64, _vp, _vp],
    "tw_eval_small_work": [_i64, _i64, _i64],
    "tw_eval_small": [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _i64,
                      _vp, _i32, _f64, _vp, _vp, _vp, _vp, _vp, _vp],
    "tw_ship_draws": [_vp, _i32, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _vp],
    "tw_draw_pipe_start": [_vp, _vp, _i32, _vp, _vp, _i64, _i32, _i64, _i64, _i64, _i64, _i64,
                           _i32, _i32, _vp, _vp, _i32, _i32, _vp],
    "tw_ship_draws_tables": [_vp, _i32, _i64, _vp, _vp, _i32, _i32, _i64, _vp, _i64, _vp, _vp],
    "tw_np_randint_batch_u16": [_vp, _vp, _i32, _vp, _vp, _vp, _vp],
    "tw_draw_pipe_wait": [_vp, _i32],
    "tw_draw_pipe_shipped": [_vp, _i32, _vp],
    "tw_draw_pipe_stop": [_vp],
    "tw_copy_words": [_vp, _i64, _vp, _vp],
    "tw_stage_eval": [_vp, _i32, _vp, _i32, _vp, _vp, _vp],
    "tw_host_device_pointer": [_vp, _vp],
    "tw_chain_final_pack": [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i64, _vp, _vp, _vp,
                            _vp],
    "tw_chain_final_scatter": [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "tw_chain_walk": [_i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _vp],
    "tw_chain_unpack_count": [_vp, _i32, _i32, _i64, _i32, _i64, _i64, _i64, _i64, _i32, _vp,
                              _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp],
    "tw_chain_unpack_exact": [_vp, _i32, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "tw_count_pairs_chain_rng": [_vp, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i64, _i64, _i64,
                                 _u64, _u64, _vp, _vp],
    "tw_words_checksum": [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i64, _vp],
    "tw_words_checksum_acc_words": [],
    "tw_np_shuffle_pair": [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _i64, _vp],
    "tw_np_shuffle_draws32": [_vp, _vp, _i64, _vp],
    "tw_np_shuffle_draws32_range": [_vp, _vp, _i64, _i64, _i64, _vp],
    "tw_shuffle_swaps_work_bytes": [_i64, _i64],
    "tw_shuffle_swaps_rounds": [_i64, _i64],
    "tw_shuffle_swaps_set_rounds": [_i32],
    "tw_shuffle_swaps_set_tail": [_i32],
    "tw_shuffle_swaps": [_vp, _i64, _vp, _i64, _vp, _vp, _i32, _i32, _vp, _vp, _vp],
    "tw_shuffle_swaps_windows": [],
    "tw_shuffle_swaps_part": [_vp, _i64, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp],
}
_RESTYPES = {
    "tw_last_error": ctypes.c_char_p,
    "tw_count_pairs_sorted_work_bytes": ctypes.c_int64,
    "tw_rank_images_work_bytes": ctypes.c_int64,
    "tw_peer_buffer_bytes": ctypes.c_int64,
    "tw_count_pairs_rng_work_bytes": ctypes.c_int64,
    "tw_count_pairs_sorted_steps_work_bytes": ctypes.c_int64,
    "tw_pair_sum_work_per_shard": ctypes.c_int64,
    "tw_pair_sum_idx_work_per_shard": ctypes.c_int64,
    "tw_pair_grad_complete_work_bytes": ctypes.c_int64,
    "tw_pair_hinge_sum_sorted_work_bytes": ctypes.c_int64,
    "tw_shuffle_swaps_work_bytes": ctypes.c_int64,
    "tw_eval_small_work": ctypes.c_int64,
    "tw_words_checksum_acc_words": ctypes.c_int64,
}

_lib = None


class _NoTensor:  # stands in for torch.Tensor until lib() has imported torch
    pass


_TENSOR = _NoTensor  # torch.Tensor once lib() has run: call() converts such arguments
_getrefcount = sys.getrefcount


class TuplewiseError(RuntimeError):
    """A HIP runtime failure inside libtuplewise.so."""


def lib() -> ctypes.CDLL:
    """Load libtuplewise.so once (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64/libhsa-runtime64, and
        # libtuplewise.so's NEEDED libamdhip64.so.7 must bind to that copy.  Loading our
        # library first would pull /opt/rocm's runtime in beside torch's (two HSA runtimes,
        # one of which then sees no device), so torch is imported before the dlopen.
        import torch as _torch
        global _TENSOR
        _TENSOR = _torch.Tensor
        if not LIB_PATH.exists():
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g;"
                " g.build()'` (hipcc --offload-arch=gfx950).  There is no CPU fallback.")
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = handle
    return _lib


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int) -> None:
    """Map a C-ABI status to the exception family the reference would raise."""
    if rc == TW_OK:
        return
    msg = lib().tw_last_error().decode(errors="replace")
    if rc == TW_ERR_ARG:
        raise ValueError(msg)
    raise TuplewiseError(msg)


def call(name: str, *args) -> None:
    """Run one C-ABI entry point.  A torch tensor may be passed in place of its `ptr()`: it is
    converted here and, being an element of `args`, stays referenced until the entry point has
    returned (and, since every launch is stream-ordered after the caller's allocations, until
    the caching allocator can no longer hand its block to a later temporary of the same
    argument list — the round-5 aperture violation's class, learning.py:443-475)."""
    fn = getattr(lib(), name)
    T = _TENSOR
    for a in args:
        if isinstance(a, T):
            args = tuple(ctypes.c_void_p(a.data_ptr()) if isinstance(a, T) else a for a in args)
            break
    check(fn(*args))


# ----------------------------------------------------------------------------- device memory
def torch():
    import torch as _torch  # imported lazily: the C ABI itself has no torch dependency
    return _torch


def device():
    """The HIP device all package work runs on (current torch device)."""
    t = torch()
    if not t.cuda.is_available():
        raise TuplewiseError(
            "tuplewise: no HIP device is visible; the MI355X path has no CPU fallback")
    return t.device("cuda", t.cuda.current_device())


def stream_handle():
    """The current HIP stream of the current device as a raw handle (the C ABI's `stream`): the
    raw-stream accessor, not a torch.cuda.Stream object per call (~4x less host time in the
    learning loop's launches)."""
    C = torch()._C
    return ctypes.c_void_p(C._cuda_getCurrentRawStream(C._cuda_getDevice()))


def host_device_pointer(t):
    """The device address of a pinned host tensor's storage (None when it is not mapped)."""
    out = ctypes.c_void_p()
    if lib().tw_host_device_pointer(ctypes.c_void_p(t.data_ptr()), ctypes.byref(out)) != TW_OK:
        return None
    return out.value


def ptr(t) -> ctypes.c_void_p:
    """The device address of a tensor that someone else keeps alive.

    A bare address does not hold its tensor: `ptr(to_device(a))` frees the block as soon as
    this returns, so a later temporary of the same argument list can be handed the same block
    (round 5: aliased bucket starts and an aperture violation in k_row_table_remote).  Such an
    unreferenced temporary is refused here — by its reference count, which for an object only
    the caller's evaluation stack holds is 3 inside this frame (stack, parameter, getrefcount's
    argument), and for a view whose base nobody else holds the base's count is 2.  Pass the
    tensor itself to `call()` instead, or bind it to a name first."""
    if t is None:
        return ctypes.c_void_p(0)
    if _getrefcount(t) <= 3:
        b = t._base
        if b is None or _getrefcount(b) <= 3:  # 3 here: b, the view's own ref, the argument
            raise TuplewiseError(
                "tuplewise._lib.ptr: an unreferenced temporary tensor; its block would be freed "
                "before the native call runs — pass the tensor to call() or name it first")
    return ctypes.c_void_p(t.data_ptr())


def to_device(arr: np.ndarray, dtype=None):
    """Host ndarray -> contiguous device tensor (copy)."""
    t = torch()
    a = np.ascontiguousarray(arr if dtype is None else arr.astype(dtype, copy=False))
    return t.from_numpy(a).to(device())


def to_device_many(arrays, pinned: bool = False) -> list:
    """Several host arrays -> contiguous device tensors of the same dtypes through ONE H2D copy
    (the small drop-in calls were bound by one copy's fixed cost per array).  Each array starts
    at an 8-byte boundary of the staging buffer.  pinned: staged in page-locked memory (torch's
    caching host allocator) and copied asynchronously on the current stream — the host does
    not wait for the stream's earlier work (the drop-in's per-step counts)."""
    t = torch()
    arrs = [np.ascontiguousarray(a) for a in arrays]
    offs, total = [], 0
    for a in arrs:
        offs.append(total)
        total += (a.nbytes + 7) & ~7
    host = (t.empty((max(total, 8),), dtype=t.uint8, pin_memory=True) if pinned
            else t.from_numpy(np.empty(max(total, 8), dtype=np.uint8)))
    buf = host.numpy()
    for a, o in zip(arrs, offs):
        buf[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
    dev = host.to(device(), non_blocking=pinned)
    out = []
    for a, o in zip(arrs, offs):
        td = t.from_numpy(np.empty(0, dtype=a.dtype)).dtype
        out.append(dev[o:o + a.nbytes].view(td).reshape(a.shape))
    return out


def empty(shape, dtype):
    return torch().empty(shape, dtype=dtype, device=device())


def collectives_default(group, G: int) -> bool:
    """The collectives= default of ShardedSample / SGDEngine: the multi-rank branches exactly
    when the group has several ranks, or on any group when TW_FORCE_COLLECTIVES=1 (bench.py's
    world-size-1 RCCL rehearsal: every collective of the multi-GPU path on one GPU)."""
    if group is None:
        return False
    return G > 1 or os.environ.get("TW_FORCE_COLLECTIVES", "") == "1"


def capture(graph):
    """torch.cuda.graph(graph) in thread-local capture mode: other host threads (the RCCL
    process group's watchdog polling its events, the native draw thread) keep making HIP calls
    while a stream of this thread captures — in the default global mode those calls invalidate
    the capture and kill the watchdog (seen on a world-size-1 nccl group)."""
    return torch().cuda.graph(graph, capture_error_mode="thread_local")
