"""ctypes binding of ``librecsys_amd.so`` (the C ABI in ``include/recsys_amd.h``).

This is the "reference-side binding" for a Python reference: the host layer passes raw device
pointers, sizes and the current HIP stream; no torch types cross the boundary.  torch is imported
FIRST so the process has exactly one HIP runtime (torch's ``libamdhip64.so.7``; the library's
``DT_NEEDED libamdhip64.so.7`` then binds to it by soname).

The product path has no fallback: if the library is missing or a call fails, this raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: one HIP runtime per process)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG_DIR, "librecsys_amd.so")

RS_OK, RS_ERR_ARG, RS_ERR_UNSUPPORTED, RS_ERR_LAUNCH = 0, -1, -2, -3
_ERRS = {RS_ERR_ARG: "bad argument/shape", RS_ERR_UNSUPPORTED: "shape not compiled in",
         RS_ERR_LAUNCH: "kernel launch failed"}

_vp, _i32, _i64, _f32, _u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64

# name -> (restype, argtypes); must match include/recsys_amd.h exactly
SIGNATURES: dict[str, tuple] = {
    "rs_embedding_lookup_fwd": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _i32, _vp, _i64,
                                       _i32, _vp, _i64, _i64, _vp]),
    "rs_sequence_lookup_fwd": (_i32, [_vp, _vp, _vp, _i64, _i32, _i64, _i64, _i32, _vp, _i32, _vp,
                                      _i64, _i64, _vp, _i64, _vp, _vp]),
    "rs_sparse_grad_accumulate": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _i32, _i32,
                                         _vp, _vp, _vp, _vp, _i32]),
    "rs_sparse_push_workspace_bytes": (_i64, [_i64, _i32]),
    "rs_sparse_grad_accumulate_ws": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _i32, _i32,
                                            _vp, _vp, _vp, _vp, _i32, _vp, _i64]),
    "rs_sparse_push_group_workspace_bytes": (_i64, [_i32, _vp, _vp]),
    "rs_sparse_grad_accumulate_group": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp,
                                               _vp, _vp, _vp, _i32, _vp, _i64]),
    "rs_sparse_adam": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _f32, _f32, _f32,
                              _f32, _f32]),
    "rs_sparse_adagrad": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _f32, _f32]),
    "rs_sparse_compact": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _i32]),
    "rs_sparse_merge_rows": (_i32, [_vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _i32]),
    "rs_sparse_merge_rows_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp,
                                        _vp, _vp, _i32]),
    "rs_sparse_merge_rows_dev_stride": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32,
                                                _vp, _vp, _vp, _vp, _i32, _vp]),
    "rs_sparse_sorted_workspace_bytes": (_i64, [_i64]),
    "rs_sparse_grad_accumulate_sorted": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _i32,
                                                _i32, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _i64,
                                                _i64]),
    "rs_owner_route_workspace_bytes": (_i64, [_i64, _i32]),
    "rs_owner_route": (_i32, [_vp, _vp, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _i64]),
    "rs_owner_route_fixed": (_i32, [_vp, _vp, _i64, _i32, _i64, _i32, _vp, _vp, _vp, _vp, _i64]),
    "rs_gather_rows": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64]),
    "rs_scatter_rows": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64]),
    "rs_segment_expand": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _i32, _i32, _i32, _vp]),
    "rs_set_math_mode": (_i32, [_i32]),
    "rs_get_math_mode": (_i32, []),
    "rs_set_seed_offset": (_i32, [_vp]),
    "rs_il_set_variant": (_i32, [_i32]),
    "rs_ctr_metrics_state_doubles": (_i64, [_i32]),
    "rs_ctr_metrics_accumulate": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _vp]),
    "rs_ctr_metrics_result": (_i32, [_vp, _vp, _i32, _vp]),
    "rs_il_get_variant": (_i32, []),
    "rs_il_param_count": (_i32, [_i32, _i32]),
    "rs_il_fwd": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32,
                         _i32, _f32, _u64, _vp, _i64, _vp]),
    "rs_il_fwd_gather": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i64, _i32, _i32,
                                _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp,
                                _i64, _vp]),
    "rs_il_bwd_workspace_floats": (_i64, [_i64, _i32, _i32]),
    "rs_il_attn_save_floats": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "rs_il_fwd_saved": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                               _f32, _i32, _f32, _u64, _vp, _i64, _vp, _vp, _i64]),
    "rs_il_bwd_saved": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp,
                               _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp, _i32, _vp, _i32, _vp,
                               _i64, _vp, _i64]),
    "rs_il_bwd": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp,
                         _vp, _vp, _f32, _i32, _f32, _u64, _vp, _i32, _vp, _i32, _vp, _i64]),
    "rs_dense_fwd": (_i32, [_vp, _vp, _i64, _i32, _i64, _vp, _vp, _i32, _i32, _vp, _i64]),
    "rs_dense_bwd_data": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _i32, _i32, _vp, _i64,
                                 _i32]),
    "rs_dense_bwd_weight_workspace_floats": (_i64, [_i64, _i32, _i32]),
    "rs_dense_uses_library": (_i32, [_i64, _i32, _i32]),
    "rs_dense_uses_big": (_i32, [_i64, _i32, _i32]),
    "rs_dense_bwd_weight": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i64, _i32, _i32,
                                   _vp, _vp, _i32, _vp, _i64]),
    "rs_dense_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _i32, _i32, _vp,
                            _i64, _i32, _vp, _vp, _i32, _vp, _i64]),
    "rs_dense_fwd_grouped": (_i32, [_vp, _i32, _vp]),
    "rs_dense_bwd_data_grouped": (_i32, [_vp, _i32, _vp]),
    "rs_dense_bwd_weight_grouped_workspace_floats": (_i64, [_i32, _vp]),
    "rs_dense_bwd_weight_grouped": (_i32, [_vp, _i32, _vp, _vp, _i64]),
    "rs_bce_clip_loss": (_i32, [_vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32, _vp, _vp, _vp, _vp]),
    "rs_bce_clip_workspace_floats": (_i64, [_i64, _i32]),
    "rs_bce_clip_loss_ws": (_i32, [_vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32, _vp, _vp, _vp, _vp,
                                   _vp, _i64]),
    "rs_dense_adam": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _f32, _f32, _f32, _f32, _f32,
                             _i32]),
    "rs_dense_adam_done": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _f32, _f32, _f32, _f32, _f32,
                             _i32, _vp]),
    "rs_din_param_count": (_i32, [_i32, _i32]),
    "rs_din_bwd_workspace_floats": (_i64, [_i32, _i64, _i32, _i32]),
    "rs_din_fwd": (_i32, [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i64, _i32, _i32,
                          _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "rs_din_bwd": (_i32, [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i64, _i32, _i32,
                          _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp,
                          _vp, _i32, _vp, _i64]),
    "rs_din_bwd_strided": (_i32, [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i64, _i32,
                                  _i32, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                  _i64, _vp, _vp, _i64, _i32, _vp, _i32, _vp, _i64]),
    "rs_din_bwd_ex": (_i32, [_vp, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i64, _i32,
                             _i32, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                             _i64, _vp, _i64, _vp, _vp, _i64, _i32, _vp, _i32, _vp, _i64]),
    "rs_gate_mix_fwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp,
                               _vp, _i64, _vp, _i64]),
    "rs_gate_mix_bwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp,
                               _vp, _i64, _vp, _i64, _vp, _i64]),
    "rs_cross_bwd_workspace_floats": (_i64, [_i64, _i32, _i32]),
    "rs_cross_fwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _i64]),
    "rs_cross_bwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _i64, _vp, _i64, _i32,
                            _vp, _i32, _vp, _i64]),
    "rs_fm_fwd": (_i32, [_vp, _vp, _i64, _i64, _i64, _i32, _i32, _vp, _i64, _f32, _vp, _i64, _vp,
                         _i64, _vp, _i64]),
    "rs_fm_bwd": (_i32, [_vp, _vp, _i64, _i64, _i64, _i32, _i32, _vp, _i64, _f32, _vp, _i64, _vp, _i64,
                         _vp, _i64, _vp, _i64, _i64, _i32, _vp, _i64]),
    "rs_ffm_param_count": (_i64, [_i32, _i32, _i32, _i32]),
    "rs_ffm_bwd_workspace_floats": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "rs_ffm_fwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                          _vp, _i64, _vp, _i64]),
    "rs_ffm_bwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                          _vp, _i64, _vp, _i64, _vp, _i64, _i32, _vp, _i32, _vp, _i64]),
    "rs_mul_fwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _f32, _vp, _i64]),
    "rs_mul_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _f32, _vp, _i64, _vp, _i64, _vp,
                          _i64]),
    "rs_mul_fwd_grouped": (_i32, [_vp, _i32, _vp, _f32]),
    "rs_mul_bwd_grouped": (_i32, [_vp, _i32, _vp, _f32]),
    "rs_softmax_kl": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _i64, _vp, _i64, _vp, _f32, _f32,
                             _vp, _vp, _i64]),
    "rs_rowdot": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _i64, _vp,
                         _i64]),
    "rs_mse_rows": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _f32, _vp, _vp, _i64]),
    "rs_grouped_head_bwd_workspace_floats": (_i64, [_i64, _i32, _i32]),
    "rs_grouped_head_fwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _i32, _vp, _i64]),
    "rs_grouped_head_bwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _i64, _i32, _vp,
                                   _i64, _vp, _i64, _vp, _i32, _vp, _i64]),
    "rs_row_select": (_i32, [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i32, _vp, _i64, _vp, _vp, _vp]),
    "rs_l1l2_grad": (_i32, [_vp, _vp, _vp, _i64, _f32, _f32]),
    "rs_l1l2_grad_grouped": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "rs_act_fwd": (_i32, [_vp, _vp, _i64, _i32, _vp]),
    "rs_act_bwd": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "rs_bce_rows": (_i32, [_vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32, _vp, _f32, _vp, _vp]),
    "rs_weighted_row_sum": (_i32, [_vp, _vp, _i64, _i32, _f32, _f32, _f32, _f32, _f32, _f32, _vp]),
    "rs_staytime_labels": (_i32, [_vp, _vp, _vp, _i64, _vp, _i32, _f32, _f32, _f32, _vp, _i64,
                                  _vp, _vp, _vp]),
    "rs_mlp_head_param_floats": (_i64, [_i32, _i32, _i32, _i32, _i32]),
    "rs_mlp_head_workspace_floats": (_i64, [_i64, _i32, _i32, _i32, _i32, _i32]),
    "rs_mlp_head_partial_blocks": (_i32, [_i64]),
    "rs_mlp_head_train": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32,
                                 _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32,
                                 _f32, _vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64]),
    "rs_mlp_head_dz_workspace_floats": (_i64, [_i64, _i32, _i32, _i32, _i32, _i32]),
    "rs_mlp_head_train_dz": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32,
                                    _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32,
                                    _f32, _vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _vp, _i64]),
    "rs_partials_reduce_adam_rows": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _vp, _vp, _f32, _f32, _f32, _f32, _f32, _i32,
                                            _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32,
                                            _f32, _f32, _vp, _i64]),
    "rs_partials_reduce_adam_rows_ex": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                               _vp, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _f32,
                                               _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32,
                                               _f32, _f32, _f32, _f32, _vp, _i64, _i64, _vp, _i64,
                                               _i64]),
    "rs_partials_reduce_adam": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _f32, _f32, _f32, _f32, _f32, _i32]),
    "rs_partials_reduce_adam_scan": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _f32, _f32, _f32, _f32, _f32, _i32,
                                       _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32, _f32, _f32]),
    "rs_il_bwd_partial_blocks": (_i32, [_i64, _i32, _i32, _i32, _i32, _i64]),
    "rs_il_bwd_saved_partial_blocks": (_i32, [_i64, _i32, _i32, _i32, _i32, _i64]),
    "rs_sparse_adam_scan": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32, _f32,
                                   _f32, _f32]),
    "rs_sparse_adagrad_scan": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32]),
    "rs_sparse_adam_recover": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32,
                                      _f32, _f32, _f32]),
    "rs_sparse_adagrad_recover": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _f32, _f32]),
    "rs_sparse_compact_scan": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _i32]),
    "rs_sparse_pack_scan": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32]),
    "rs_sparse_merge_packed": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _i64, _i32]),
    "rs_sparse_merge_packed_stride": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _i64, _i32, _i32]),
    "rs_il_bwd_push": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp,
                              _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp, _vp, _vp, _vp, _vp,
                              _i32, _vp, _i64]),
    "rs_il_bwd_push_saved": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32,
                                    _vp, _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp, _vp, _vp, _vp,
                                    _vp, _i32, _vp, _i64, _vp, _i64]),
    "rs_il_xt_splits": (_i32, [_i64]),
    "rs_il_bwd_xt_supported": (_i32, [_i64, _i32, _i32, _i32, _i32, _i64]),
    "rs_il_bwd_saved_xt": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp,
                                  _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp, _i32, _vp, _i32, _vp,
                                  _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _vp]),
    "rs_il_bwd_push_saved_xt": (_i32, [_vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32,
                                       _i32, _vp, _vp, _vp, _vp, _f32, _i32, _f32, _u64, _vp, _vp,
                                       _vp, _vp, _vp, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                       _i64, _i32, _i32, _vp]),
    "rs_il_fwd_gather_saved": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i64, _i32,
                                      _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _i32, _f32,
                                      _u64, _vp, _i64, _vp, _vp, _i64]),
    "rs_gather_columns": (_i32, [_vp, _vp, _i64, _i64, _vp, _i32, _vp, _i64]),
    "rs_gather_sum_columns": (_i32, [_vp, _i32, _vp, _vp, _vp, _i64, _i32, _vp, _i64]),
    "rs_scatter_add_columns": (_i32, [_vp, _vp, _i64, _i64, _vp, _i32, _vp, _i64]),
    "rs_segment_mean": (_i32, [_vp, _vp, _i64, _i64, _vp, _i32, _vp, _i64]),
    "rs_field_scale_fwd": (_i32, [_vp, _vp, _i64, _i64, _vp, _i32, _vp, _i64, _f32, _vp, _i64]),
    "rs_field_scale_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _vp, _i32, _vp, _i64, _f32,
                                  _vp, _i64, _i32, _vp, _i64]),
    "rs_field_linear_fwd": (_i32, [_vp, _vp, _i64, _i64, _vp, _i32, _i32, _vp, _vp, _vp, _i64]),
    "rs_field_linear_workspace_floats": (_i64, [_i64, _i32, _i32, _i32]),
    "rs_field_linear_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i32, _i32, _i32,
                                   _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _i64]),
    "rs_can_fwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp]),
    "rs_can_bwd": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                          _i32, _vp, _i64]),
    "rs_fm_proj_fwd": (_i32, [_vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp]),
    "rs_fm_proj_workspace_floats": (_i64, [_i64, _i32, _i32]),
    "rs_fm_proj_bwd": (_i32, [_vp, _vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _i64, _i32,
                              _vp, _i32, _vp, _i64]),
}

_LIB = None


class RecsysKernelError(RuntimeError):
    pass


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the shared library.  Raises if it has not been built.
    RS_LIB_PATH overrides the in-tree library (kernel-variant experiments only)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("RS_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
        raise RecsysKernelError(
            f"{path} not found: build the HIP extension first (python -c "
            "'import __graft_entry__ as g; g.build()' or python recommendsystem_amd/build.py)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    v = os.environ.get("RS_IL_VARIANT")  # A/B runs: auto | wave | wide
    if v:
        lib.rs_il_set_variant(IL_VARIANTS[v])
    return lib


_TRACE = bool(os.environ.get("RS_TRACE_CALLS"))  # debugging: sync + name after every launch


def call(name: str, *args) -> int:
    rc = getattr(load(), name)(*args)
    if _TRACE and not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()
        print(f"[rs] {name} ok", flush=True)
    if SIGNATURES[name][0] is _i32 and rc != RS_OK and not name.endswith(("_count", "_blocks")):
        raise RecsysKernelError(f"{name} returned {rc} ({_ERRS.get(rc, 'hip error')})")
    return rc


def trace_point(what: str) -> None:
    """RS_TRACE_CALLS debugging: synchronise and name the step section that just completed
    (graph replays are not visible to `call`)."""
    if _TRACE and not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()
        print(f"[rs] {what} ok", flush=True)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle() -> int:
    """hipStream_t of torch's current stream on the current device."""
    return torch.cuda.current_stream().cuda_stream


def require_device(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RecsysKernelError("recommendsystem_amd kernels need tensors on a ROCm device "
                                    "(there is no CPU fallback)")


def c_array(ctype, values):
    """A ctypes array (keep a reference while the call runs) and its address for a `_vp` slot."""
    arr = (ctype * len(values))(*values)
    return arr, ctypes.addressof(arr)


def partials_reduce_adam(stream, segments, params=None, m=None, v=None, step=None, done=None,
                         lr=0.0, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0,
                         adam=False, scan_table=None, scan_grad_scale=1.0, scan_rows=None) -> int:
    """rs_partials_reduce_adam over a list of segments
    (part_ptr, ld, nrows, ncols, out_ptr, scale, adam_off); with ``scan_table`` (a scan-mode
    SparseTable with a SparseAdam optimizer) its sparse Adam runs in the same launch
    (rs_partials_reduce_adam_scan); with ``scan_rows`` = (rows, n) too, it walks those n looked-up
    rows instead of sweeping the flags (rs_partials_reduce_adam_rows: valid when they are the only
    rows marked); ``scan_rows`` = (rows_ptr, n, stride, counts_ptr, counts_stride, seg_len) walks
    strided entries of which each seg_len-long segment holds counts[seg] valid ones (the packed DP
    records after the exchange, rs_partials_reduce_adam_rows_ex)."""
    n = len(segments)
    keep = []

    def arr(ct, vals):
        a, addr = c_array(ct, vals)
        keep.append(a)
        return addr

    parts = arr(ctypes.c_void_p, [s[0] for s in segments])
    lds = arr(ctypes.c_int64, [s[1] for s in segments])
    nrows = arr(ctypes.c_int32, [s[2] for s in segments])
    ncols = arr(ctypes.c_int64, [s[3] for s in segments])
    outs = arr(ctypes.c_void_p, [s[4] for s in segments])
    scales = arr(ctypes.c_float, [s[5] for s in segments])
    offs = arr(ctypes.c_int64, [s[6] for s in segments])
    if scan_table is not None and scan_rows is not None:
        t, o = scan_table, scan_table.optimizer
        rows, nr, *packed = scan_rows
        stride, cptr, cstride, seg = packed if packed else (1, None, 0, 0)
        return call("rs_partials_reduce_adam_rows_ex", stream, n, parts, lds, nrows, ncols, outs,
                    scales, offs, ptr(params), ptr(m), ptr(v), ptr(step), ptr(done), lr, beta1,
                    beta2, eps, grad_scale, int(adam), ptr(t.weight), ptr(t.m), ptr(t.v),
                    ptr(t.grad), ptr(t.flag), t.rows, t.dim, o.learning_rate, o.beta1, o.beta2,
                    o.epsilon, scan_grad_scale,
                    rows if isinstance(rows, int) else ptr(rows), int(nr), int(stride), cptr,
                    int(cstride), int(seg))
    if scan_table is not None:
        t, o = scan_table, scan_table.optimizer
        return call("rs_partials_reduce_adam_scan", stream, n, parts, lds, nrows, ncols, outs,
                    scales, offs, ptr(params), ptr(m), ptr(v), ptr(step), ptr(done), lr, beta1,
                    beta2, eps, grad_scale, int(adam), ptr(t.weight), ptr(t.m), ptr(t.v),
                    ptr(t.grad), ptr(t.flag), t.rows, t.dim, o.learning_rate, o.beta1, o.beta2,
                    o.epsilon, scan_grad_scale)
    return call("rs_partials_reduce_adam", stream, n, parts, lds, nrows, ncols, outs, scales, offs,
                ptr(params), ptr(m), ptr(v), ptr(step), ptr(done), lr, beta1, beta2, eps,
                grad_scale, int(adam))


MATH_MODES = {"f32": 0, "bf16": 1}
# rs_il_set_variant: which InteractingLayer kernels run the E = U = 16, H = 2, F <= 32 shapes
IL_VARIANTS = {"auto": 0, "wave": 1, "wide": 2}


@contextlib.contextmanager
def il_variant(name: str):
    """rs_il_set_variant for the duration of the block ("auto" | "wave" = one wave per sample |
    "wide" = one 4-wave workgroup per sample; include/recsys_amd.h)."""
    if name not in IL_VARIANTS:
        raise ValueError(f"IL variant must be one of {sorted(IL_VARIANTS)}, got {name!r}")
    prev = load().rs_il_get_variant()
    call("rs_il_set_variant", IL_VARIANTS[name])
    try:
        yield
    finally:
        call("rs_il_set_variant", prev)


@contextlib.contextmanager
def math_mode(mode: str):
    """rs_set_math_mode for the duration of the block ("f32" | "bf16"; include/recsys_amd.h):
    launches issued -- or captured into a graph -- inside it use that mode."""
    if mode not in MATH_MODES:
        raise ValueError(f"math mode must be one of {sorted(MATH_MODES)}, got {mode!r}")
    prev = load().rs_get_math_mode()
    call("rs_set_math_mode", MATH_MODES[mode])
    try:
        yield
    finally:
        call("rs_set_math_mode", prev)


_SEED_OFFSET = [None]


@contextlib.contextmanager
def seed_offset(counter):
    """rs_set_seed_offset(counter) for the duration of the block: dropout launches issued (or
    captured) inside it add the device int64 `counter`'s value at run time to their seed."""
    if counter is not None and (counter.dtype != torch.int64 or not counter.is_cuda):
        raise ValueError("seed offset must be a device int64 tensor")
    prev = _SEED_OFFSET[0]
    call("rs_set_seed_offset", ptr(counter))
    _SEED_OFFSET[0] = counter
    try:
        yield
    finally:
        call("rs_set_seed_offset", ptr(prev))
        _SEED_OFFSET[0] = prev


def seed_offset_active() -> bool:
    return _SEED_OFFSET[0] is not None
