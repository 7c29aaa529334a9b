"""ctypes binding of include/bann.h (librsbann_amd.so, built in-tree).

The product path is the HIP library; there is no CPU fallback.  If the shared
library is missing, importing the compute API raises ``BannLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)                       # rs-bann_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("BANN_LIB") or os.path.join(PKG_ROOT, "librsbann_amd.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "bann.h")
HEADER_PATHS = [HEADER_PATH, os.path.join(REPO_ROOT, "include", "bann_net.h")]

BANN_OK = 0
STATUS = {0: "BANN_OK", -1: "BANN_E_HIP", -2: "BANN_E_SHAPE", -3: "BANN_E_OOM", -4: "BANN_E_STATE",
          -5: "BANN_E_ARG"}
ACTIVATIONS = {"tanh": 0, "relu": 1, "leaky_relu": 2, "silu": 3, "identity": 4}
PRIORS = {"ridge_ard": 0, "ridge_base": 1, "lasso_ard": 2, "lasso_base": 3, "std_normal": 4}
STEP_MODES = {"uniform": 0, "random": 1, "std_scaled": 2, "izmailov": 3, "injected": 100}
HMC_STATUS = {0: "accepted", 1: "rejected", 2: "rejected_early"}


class BannLibraryError(RuntimeError):
    pass


class BannError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


_P = C.c_void_p
_i32, _i64, _u64, _f32, _f64 = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_double
_pi8, _pu8 = C.POINTER(C.c_int8), C.POINTER(C.c_uint8)
_pi32, _pf32, _pf64 = C.POINTER(C.c_int32), C.POINTER(C.c_float), C.POINTER(C.c_double)



class PrecisionHyperparams(C.Structure):
    """bann_precision_hyperparams (NetworkPrecisionHyperparameters, params.rs:134-142)"""
    _fields_ = [("dense_shape", C.c_float), ("dense_scale", C.c_float), ("summary_shape", C.c_float),
                ("summary_scale", C.c_float), ("output_shape", C.c_float), ("output_scale", C.c_float)]


class McmcCfg(C.Structure):
    """bann_mcmc_cfg (the MCMCCfg fields of Net::train's HMC path, mcmc_cfg.rs:181-204)"""
    _fields_ = [("hmc_step_size_factor", C.c_float), ("hmc_max_hamiltonian_error", C.c_float),
                ("hmc_integration_length", C.c_int32), ("hmc_step_size_mode", C.c_int32),
                ("chain_length", C.c_int32), ("burn_in", C.c_int32), ("fixed_param_precisions", C.c_int32),
                ("sampled_output_bias", C.c_int32), ("trace", C.c_int32), ("trajectories", C.c_int32),
                ("joint_hmc", C.c_int32), ("gradient_descent", C.c_int32),
                ("gradient_descent_joint", C.c_int32), ("effect_sizes", C.c_int32)]


# bann_allreduce_fn: in-place sum over ranks of a host buffer (dtype 0 f32, 1 f64)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32)
UNIFORM_FN = C.CFUNCTYPE(C.c_double, C.c_void_p)
NORMAL_FN = C.CFUNCTYPE(C.c_double, C.c_void_p)
GAMMA_FN = C.CFUNCTYPE(C.c_double, C.c_void_p, C.c_double, C.c_double)


class RngHooks(C.Structure):
    """bann_rng_hooks: host random source of the network driver"""
    _fields_ = [("user", C.c_void_p), ("uniform", UNIFORM_FN), ("normal", NORMAL_FN), ("gamma", GAMMA_FN)]


class TrainSummary(C.Structure):
    """bann_train_summary (TrainingStats + global state)"""
    _fields_ = [("num_samples", C.c_uint64), ("num_accepted", C.c_uint64), ("num_early_rejected", C.c_uint64),
                ("num_records", C.c_int32), ("mse_train_last", C.c_float), ("lpd_last", C.c_float),
                ("output_bias", C.c_float), ("error_precision", C.c_float), ("output_layer_precision", C.c_float),
                ("output_reg_sum", C.c_float)]


# name -> (restype, argtypes); mirrors include/bann.h and include/bann_net.h one to one
SIGNATURES = {
    "bann_ctx_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "bann_ctx_destroy": (C.c_int, [_P]),
    "bann_last_error": (C.c_char_p, [_P]),
    "bann_version": (C.c_char_p, []),
    "bann_genotypes_upload": (C.c_int, [_P, _pi8, _i64, _i64]),
    "bann_genotypes_upload_bed": (C.c_int, [_P, _pu8, _i64, _i64]),
    "bann_genotypes_synthetic": (C.c_int, [_P, _i64, _i64, _u64]),
    "bann_genotypes_stats": (C.c_int, [_P, _pf32, _pf32]),
    "bann_genotypes_load_bed": (C.c_int, [_P, C.c_char_p]),
    "bann_bed_dims": (C.c_int, [C.c_char_p, C.POINTER(_i64), C.POINTER(_i64)]),
    "bann_grouping_read": (C.c_int, [C.c_char_p, _pi32, C.POINTER(_i64), C.POINTER(_i64), _pi32]),
    "bann_grouping_uniform": (C.c_int, [_i32, _i32, C.POINTER(_i64), _pi32]),
    "bann_phen_read": (C.c_int, [C.c_char_p, C.POINTER(_i64), _pf32]),
    "bann_phen_write": (C.c_int, [C.c_char_p, _pf32, _i64]),
    "bann_genotypes_set_stats": (C.c_int, [_P, _pf32, _pf32]),
    "bann_genotypes_download": (C.c_int, [_P, _pi32, _i32, _pi8]),
    "bann_branch_add": (C.c_int, [_P, _pi32, _i32, _pi32, _i32, _i32, _i32]),
    "bann_finalize": (C.c_int, [_P, _i32]),
    "bann_num_branches": (C.c_int, [_P]),
    "bann_num_params": (_i64, [_P, _i32]),
    "bann_num_precisions": (_i64, [_P, _i32]),
    "bann_branch_info": (C.c_int, [_P, _i32, _pi32, _pi32, _pi32, _i32, _pi32, _pi32]),
    "bann_branch_set_params": (C.c_int, [_P, _i32, _pf32]),
    "bann_branch_get_params": (C.c_int, [_P, _i32, _pf32]),
    "bann_branch_set_precisions": (C.c_int, [_P, _i32, _pf32]),
    "bann_branch_get_precisions": (C.c_int, [_P, _i32, _pf32]),
    "bann_branch_set_target": (C.c_int, [_P, _i32, _pf32]),
    "bann_set_target_all": (C.c_int, [_P, _pf32]),
    "bann_predict": (C.c_int, [_P, _i32, _pf32]),
    "bann_rss": (C.c_int, [_P, _i32, _pf64]),
    "bann_log_density_gradient": (C.c_int, [_P, _i32, _pf32, _pf64]),
    "bann_log_density": (C.c_int, [_P, _i32, _f64, _pf64]),
    "bann_log_density_gradient_many": (C.c_int, [_P, _pi32, _i32, _pf32, _pf64]),
    "bann_log_density_gradient_joint": (C.c_int, [_P, _i32, _pf32, _pf32, _pf64, _pf64]),
    "bann_forward_feed": (C.c_int, [_P, _i32, _pf32, _pf32]),
    "bann_effect_sizes": (C.c_int, [_P, _i32, _pf32]),
    "bann_population_effect_sizes": (C.c_int, [_P, _pi32, _i32, _pf32]),
    "bann_neg_hamiltonian": (C.c_int, [_P, _i32, _pf32, _pf64]),
    "bann_hmc_step": (C.c_int, [_P, _pi32, _i32, _i32, _f32, _i32, _f32, _pf32, _pf32, _u64, _pf32, _pi32, _pf64,
                                _pi32, _pf64]),
    "bann_hmc_step_joint": (C.c_int, [_P, _pi32, _i32, _i32, _f32, _i32, _f32, _pf32, _pf32, _u64, _pf32, _pf32,
                                      _pi32, _pf64, _pf64]),
    "bann_branch_set_output_stats": (C.c_int, [_P, _i32, _f32, _f32]),
    "bann_shard_branches": (C.c_int, [_pi32, _i32, _i32, _pi32]),
    "bann_comm_unique_id": (C.c_int, [_pu8]),
    "bann_ctx_comm_init": (C.c_int, [_P, _pu8, _i32, _i32]),
    "bann_ctx_comm_callback": (C.c_int, [_P, ALLREDUCE_FN, _P, _i32, _i32]),
    "bann_comm_info": (C.c_int, [_P, _pi32, _pi32, _pi32, _pi32]),
    "bann_residual_update_host": (C.c_int, [ALLREDUCE_FN, _P, _pf32, _pf32, _i64]),
    "bann_exchange_residual": (C.c_int, [_P, _pf32]),
    "bann_network_hmc_step": (C.c_int, [_P, _pf32, _f32, _f32, _i32, _f32, _i32, _f32, _pf32, _pf32, _u64, _pf32,
                                        _pi32, _pf64, _pf64]),
    "bann_exchange_residual_device": (C.c_int, [_P]),
    "bann_set_network_step_rule": (C.c_int, [_P, _i32, _f32]),
    "bann_network_step_rule_info": (C.c_int, [_P, _pf64]),
    "bann_set_network_adapt_trajectories": (C.c_int, [_P, _i32]),
    "bann_network_info": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "bann_network_step_rule_state": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "bann_residual_set": (C.c_int, [_P, _pf32]),
    "bann_residual_get": (C.c_int, [_P, _pf32]),
    "bann_residual_device": (C.c_int, [_P, C.POINTER(_pf32)]),
    "bann_residual_init": (C.c_int, [_P, _pf32, _f32, _pf64, _pf64]),
    "bann_residual_stats": (C.c_int, [_P, _pf64, _pf64]),
    "bann_residual_shift": (C.c_int, [_P, _f32, _pf64, _pf64]),
    "bann_residual_to_target": (C.c_int, [_P, _i32]),
    "bann_residual_from_target": (C.c_int, [_P, _i32, _pf64, _pf64]),
    "bann_rebuild_targets": (C.c_int, [_P, _pi32, _i32, _P]),
    "bann_set_launch_timing": (C.c_int, [_P, _i32]),
    "bann_launch_timing": (C.c_int, [_P, _pf32, _pf32, _pi32, _i32]),
    "bann_network_timing": (C.c_int, [_P, _pf32, _pf32, _pi32, _i32]),
    "bann_ctx_num_individuals": (_i64, [_P]),
    "bann_leapfrog_begin": (C.c_int, [_P, _pi32, _i32, _i32, _f32, _i32, _f32, _u64]),
    "bann_leapfrog_steps": (C.c_int, [_P, _i32]),
    "bann_leapfrog_end": (C.c_int, [_P, _pi32, _pi32]),
    "bann_leapfrog_predictions_device": (C.c_int, [_P, C.POINTER(_pf32)]),
    "bann_leapfrog_residual_delta_device": (C.c_int, [_P, _P]),
    "bann_leapfrog_residual_delta": (C.c_int, [_P, _P]),
    "bann_fused_kernel_name": (C.c_char_p, []),
    "bann_branch_get_step_sizes": (C.c_int, [_P, C.c_int32, _P]),
    "bann_predict_many": (C.c_int, [_P, _P, C.c_int32, _P]),
    "bann_synchronize": (C.c_int, [_P]),
    "bann_profile_session": (C.c_int, [_P, _i32, _pf32, _pf32]),
    "bann_branch_kernel_path": (C.c_int, [_P, _i32]),
    "bann_set_fused_enabled": (C.c_int, [_P, _i32]),
    "bann_set_hidden_gemm_bf16": (C.c_int, [_P, _i32]),
    "bann_packed_genotype_bytes": (_i64, [_P]),
    # bann_net.h: the Net::train driver and the Net<B> model file
    "bann_net_create": (C.c_int, [_P, C.POINTER(PrecisionHyperparams), _u64, C.POINTER(_P)]),
    "bann_net_destroy": (C.c_int, [_P]),
    "bann_net_set_rng_hooks": (C.c_int, [_P, C.POINTER(RngHooks)]),
    "bann_net_set_global": (C.c_int, [_P, _f32, _f32, _f32, _f32]),
    "bann_net_train": (C.c_int, [_P, _pf32, _i64, C.POINTER(McmcCfg), C.c_char_p]),
    "bann_net_train_single_branch": (C.c_int, [_P, _pf32, _i64, C.POINTER(McmcCfg), C.c_char_p]),
    "bann_net_perturb": (C.c_int, [_P, _i32, _f32, _i32, _f32]),
    "bann_net_predict": (C.c_int, [_P, _P, _pf32]),
    "bann_net_rss": (C.c_int, [_P, _P, _pf32, _i64, _pf64]),
    "bann_net_gradient": (C.c_int, [_P, _P, _pf32, _i64, _pf32]),
    "bann_net_branch_r2s": (C.c_int, [_P, _P, _pf32, _i64, _pf32]),
    "bann_net_activations": (C.c_int, [_P, _P, _i32, _pf32]),
    "bann_net_population_effect_sizes": (C.c_int, [_P, _P, _pf32]),
    "bann_net_summary": (C.c_int, [_P, C.POINTER(TrainSummary)]),
    "bann_net_records": (C.c_int, [_P, _pf32, _pf32, _i32]),
    "bann_net_residual": (C.c_int, [_P, _pf32]),
    "bann_net_set_test_data": (C.c_int, [_P, _P, _pf32, _i64]),
    "bann_net_records_test": (C.c_int, [_P, _pf32, _i32]),
    "bann_set_trajectory_recording": (C.c_int, [_P, _i32]),
    "bann_branch_get_trajectory": (C.c_int, [_P, _i32, _i32, _pi32, _pf32, _pf32, _pf64]),
    "bann_branch_get_trajectory_joint": (C.c_int, [_P, _i32, _i32, _pi32, _pf32, _pf32, _pf32, _pf64]),
    "bann_set_graph_replay": (C.c_int, [_P, _i32]),
    "bann_get_graph_replay": (C.c_int, [_P]),
    "bann_net_save": (C.c_int, [_P, C.c_char_p]),
    "bann_net_load": (C.c_int, [_P, C.c_char_p]),
    "bann_net_last_error": (C.c_char_p, [_P]),
}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load librsbann_amd.so and attach the signatures.  Raises loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise BannLibraryError(
            f"{path} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C rs-bann_amd/csrc).  There is no CPU fallback.")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
