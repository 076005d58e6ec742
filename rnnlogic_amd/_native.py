"""ctypes binding of the C-ABI library (include/rnnlogic_hip.h).

This is the only door from Python into the HIP path.  The library is built
in-tree (rnnlogic_amd/_build/librnnlogic_hip.so, see build()); if it is
missing, every GPU entry point raises — there is no silent fallback.
"""
import ctypes
import functools
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "librnnlogic_hip.so")

RNNL_OK, RNNL_ERR_INVALID, RNNL_ERR_HIP, RNNL_ERR_OVERFLOW, RNNL_ERR_NOMEM, RNNL_ERR_INTERNAL, RNNL_ERR_RANGE = \
    0, 1, 2, 3, 4, 5, 6
AGG_SUM, AGG_PNA = 0, 1
FEATURE_ADD, FEATURE_NONE = 0, 1
ROTATE_DIRECT, ROTATE_MFMA = 0, 1
FLAG_MIXED = 1
ERR_COUNT_WIDTH, ERR_NODE_RANGE, ERR_ACC_RANGE = 8, 16, 32

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32 = ctypes.c_float

# (name, restype, argtypes) for every symbol declared in include/rnnlogic_hip.h
SIGNATURES = [
    ("rnnl_last_error", ctypes.c_char_p, []),
    ("rnnl_version", ctypes.c_int, []),
    ("rnnl_graph_create", ctypes.c_int, [_P, _I64, _I32, _I32, _P]),
    ("rnnl_graph_destroy", ctypes.c_int, [_P]),
    ("rnnl_graph_info", ctypes.c_int, [_P, _P]),
    ("rnnl_rules_create", ctypes.c_int, [_P, _P, _P, _I32, _P]),
    ("rnnl_rules_destroy", ctypes.c_int, [_P]),
    ("rnnl_rules_info", ctypes.c_int, [_P, _P]),
    ("rnnl_rules_node_of_rule", ctypes.c_int, [_P, _P]),
    ("rnnl_rules_head_roots", ctypes.c_int, [_P, _P, _P]),
    ("rnnl_node_weights", ctypes.c_int, [_P, _P, _I32, _I32, _P, _P, _P]),
    ("rnnl_node_weights_size", ctypes.c_int, [_P, _I32, _P]),
    ("rnnl_node_weights_head", ctypes.c_int, [_P, _I32, _P, _I32, _I32, _P, _P, _P]),
    ("rnnl_lstm_train_sizes", ctypes.c_int, [_I32, _I32, _I32, _I32] + [ctypes.POINTER(ctypes.c_size_t)] * 4),
    ("rnnl_lstm_train_forward", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, _P, _I32, _P, _P, _P]),
    ("rnnl_lstm_train_backward", ctypes.c_int,
     [_P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _I32, _P]),
    ("rnnl_lstm_weight_grads_scratch", ctypes.c_int, [_I32, ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]),
    ("rnnl_lstm_weight_grads", ctypes.c_int, [_P, _P, _I32, ctypes.c_int64, _P, ctypes.c_size_t, _P, _P]),
    ("rnnl_lstm_encode_trie_scratch", ctypes.c_int, [_P, _I32, ctypes.POINTER(ctypes.c_size_t)]),
    ("rnnl_lstm_encode_trie", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _P, ctypes.c_size_t, _P]),
    ("rnnl_lstm_encode_trie_sum", ctypes.c_int,
     [_P, _P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _P, ctypes.c_size_t, _P, _P, _P]),
    ("rnnl_lstm_encode", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, _I32, _P, _I32, _P]),
    ("rnnl_forward_workspace_size", ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    ("rnnl_predictorplus_forward", ctypes.c_int,
     [_P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, ctypes.c_size_t, _I32, _P]),
    ("rnnl_predictorplus_ground", ctypes.c_int,
     [_P, _P, _I32, _P, _P, _P, _I32, _P, _P, ctypes.c_size_t, _I32, _I32, _P]),
    ("rnnl_predictorplus_score", ctypes.c_int,
     [_P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, ctypes.c_size_t, _I32, _I32, _I32, _P]),
    ("rnnl_predictorplus_forward_rotate", ctypes.c_int,
     [_P, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, ctypes.c_size_t, _I32, _I32, _I32, _I32, _P, _P, _P,
      _P]),
    ("rnnl_forward_rotate_zero", ctypes.c_int, [_P, ctypes.c_size_t, _P]),
    ("rnnl_forward_status", ctypes.c_int, [_P, _P]),
    ("rnnl_forward_status_totals", ctypes.c_int, [_P, _P, _P]),
    ("rnnl_forward_host_info", ctypes.c_int, [_P, _P]),
    ("rnnl_forward_header_bytes", ctypes.c_int, [_P]),
    ("rnnl_forward_status_host", ctypes.c_int, [_P, _P]),
    ("rnnl_forward_status_flags", ctypes.c_int, [_P, _P, _P, _P]),
    ("rnnl_forward_flags_host", ctypes.c_int, [_P, _P]),
    ("rnnl_ground", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _P, _P, ctypes.c_size_t, _I32, _P]),
    ("rnnl_ground_export_candidates", ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _P]),
    ("rnnl_ground_export_entries", ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _P]),
    ("rnnl_linear_node_weights_size", ctypes.c_int, [_P, _P]),
    ("rnnl_linear_node_weights", ctypes.c_int, [_P, _P, _I32, _P, _P]),
    ("rnnl_predictor_forward", ctypes.c_int,
     [_P, _P, _P, _I32, _P, _P, _P, _I32, _P, _P, _P, _P, ctypes.c_size_t, _I32, _P]),
    ("rnnl_predictor_ground", ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _P, _P, ctypes.c_size_t, _I32, _P]),
    ("rnnl_predictor_score", ctypes.c_int,
     [_P, _P, _P, _I32, _P, _P, _I32, _P, _P, _P, _P, ctypes.c_size_t, _I32, _P]),
    ("rnnl_predictor_rule_stats", ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P]),
    ("rnnl_predictor_backward", ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _I32, _P, _I32, _P, _P]),
    ("rnnl_debug_profile", ctypes.c_int, [_P]),
    ("rnnl_debug_clock", ctypes.c_int, [_P]),
    ("rnnl_debug_capacity", ctypes.c_int, [_I64, _I64, _I64]),
    ("rnnl_debug_sort_bits", ctypes.c_int, [_I32]),
    ("rnnl_debug_pair_memo", ctypes.c_int, [_I32]),
    ("rnnl_fill_rows", ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    ("rnnl_fill_value", ctypes.c_int, [_F32, _I64, _P, _P]),
    ("rnnl_rotate_table_sizes", ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P]),
    ("rnnl_rotate_entity_table", ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    ("rnnl_rotate_relation_table", ctypes.c_int, [_P, _I32, _I32, _F32, _P, _P]),
    ("rnnl_rotate_workspace_size", ctypes.c_int, [_I32, _I32, _I32, _I32, _P]),
    ("rnnl_multi_hot", ctypes.c_int, [_P, _P, _P, _I64, _P, _I32, _I32, _P, _P]),
    ("rnnl_train_batch", ctypes.c_int,
     [_P, _I64, _I32, _P, _P, _P, _I64, _P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P]),
    ("rnnl_filter_flags", ctypes.c_int, [_P, _P, _P, _I64, _P, _I32, _I32, _P, _P]),
    ("rnnl_filtered_ranks", ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _P, _P, _P]),
    ("rnnl_miner_create", ctypes.c_int, [_P, _I64, _I32, _I32, _P]),
    ("rnnl_miner_destroy", ctypes.c_int, [_P]),
    ("rnnl_rule_search", ctypes.c_int, [_P, _I32, _P, _I64, _P, _I64, _P, _P]),
    ("rnnl_rotate_score", ctypes.c_int,
     [_P, _P, _P, _I32, _F32, _P, _P, _I32, _I32, _P, _I32, _I32, _P, ctypes.c_size_t, _P]),
    ("rnnl_rotate_score_pieces", ctypes.c_int,
     [_P, _P, _P, _I32, _F32, _P, _P, _I32, _I32, _P, _I32, _I32, _P, ctypes.c_size_t, _I32, _F32, _P]),
    ("rnnl_rotate_backward", ctypes.c_int, [_P, _I32, _P, _P, _I32, _I32, _I32, _P, _P, _P]),
    ("rnnl_rotate_param_grads_scratch", ctypes.c_int, [_I32, _I32, _I32, _I32, ctypes.POINTER(ctypes.c_size_t)]),
    ("rnnl_rotate_param_grads", ctypes.c_int, [_P, _P, _I32, _P, ctypes.c_float, _P, _P, _I32, _I32, _I32, _I32, _P,
                                               _P, ctypes.c_size_t, _P, _P, _P]),
    ("rnnl_pack_weights_floats", ctypes.c_int, [_P]),
    ("rnnl_pack_weights", ctypes.c_int, [_P, _P, _P]),
    ("rnnl_nll_aux_bytes", ctypes.c_int, [_I32, _P]),
    ("rnnl_nll_forward", ctypes.c_int, [_P, _P, _P, _I32, _I32, _F32, _P, _P, _P, _P]),
    ("rnnl_nll_backward", ctypes.c_int, [_P, _P, _P, _I32, _I32, _F32, _P, _P, _P, _P, _P]),
    ("rnnl_ground_wide_scratch_bytes", ctypes.c_int, [_P, _I32, _P]),
    ("rnnl_ground_wide", ctypes.c_int,
     [_P, _P, _P, _P, _P, _P, _I32, _P, ctypes.c_size_t, _P, _P, _P, _P, _I64, _P, _P]),
    ("rnnl_forward_error_bits", ctypes.c_int, [_P, _P, _P]),
    ("rnnl_predictorplus_backward_size", ctypes.c_int, [_P, _I32, _P]),
    ("rnnl_predictorplus_backward_rows_size", ctypes.c_int, [_I32, _I64, _P]),
    ("rnnl_pna_features", ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                         _P]),
    ("rnnl_pna_features_backward_scratch", ctypes.c_int, [_P, _P]),
    ("rnnl_pna_features_backward", ctypes.c_int,
     [_P, _P, _P, _I32, _P, _I32, _I32, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _I32, _P, ctypes.c_size_t, _P,
      _P]),
    ("rnnl_predictorplus_backward", ctypes.c_int,
     [_P, _P, _P, _P, _I32, _P, _I32, _P, _P, _I64, _P, ctypes.c_size_t, _I32, _I32, _P, ctypes.c_size_t, _P,
      ctypes.c_size_t, _P, _P]),
]


class PredictorParams(ctypes.Structure):
    """rnnl_predictor_params (include/rnnlogic_hip.h)."""
    _fields_ = [("aggregator", _I32), ("feature", _I32), ("node_w", _P), ("add_w", _P), ("add_b", _P),
                ("ln_w", _P), ("ln_b", _P), ("s0_w", _P), ("s0_b", _P), ("s1_w", _P), ("s1_b", _P),
                ("rel_emb", _P), ("base_row", _P), ("packed", _P)]


class SumGrads(ctypes.Structure):
    """rnnl_sum_grads (include/rnnlogic_hip.h)."""
    _fields_ = [("emb", _P), ("emb_ld", _I32), ("add_w", _P), ("add_b", _P), ("ln_w", _P), ("ln_b", _P),
                ("s0_w", _P), ("s0_b", _P), ("s1_w", _P), ("s1_b", _P), ("rel_emb", _P)]


class RotateArgs(ctypes.Structure):
    """rnnl_rotate_args (include/rnnlogic_hip.h)."""
    _fields_ = [("eemb", _P), ("etab", _P), ("rtab", _P), ("dim", _I32), ("n_entities", _I32), ("gamma", _F32),
                ("mode", _I32), ("workspace", _P), ("workspace_bytes", ctypes.c_size_t), ("pieces", _I32),
                ("first_share", _F32)]


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("rnnlogic_hip error %d: %s" % (code, msg))
        self.code = code


_lib = None


def build(verbose=False):
    """Compile the library for gfx950 with hipcc (cross-compiles without a GPU)."""
    out = subprocess.run(["make", "-C", os.path.join(HERE, "csrc"), "-j4"], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RuntimeError("building librnnlogic_hip.so failed:\n%s%s" % (out.stdout or "", out.stderr or ""))
    return LIB_PATH


def lib():
    """The loaded library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("HIP library %s is missing: run rnnlogic_amd._native.build() "
                               "(or __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            # (an older A/B build loaded by tools/ab_run.py may lack newer entry
            # points: those raise when called; tests/test_host.py checks that
            # the shipped library exports every symbol of the header)
            f = getattr(L, name, None)
            if f is None:
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != RNNL_OK:
        raise NativeError(rc, lib().rnnl_last_error().decode(errors="replace"))
    return rc


def call(name, *args):
    return check(getattr(lib(), name)(*args))


def _run_on(index, fn, args, kw):
    import torch
    if index is None or index == torch.cuda.current_device():
        return fn(*args, **kw)
    with torch.cuda.device(index):
        return fn(*args, **kw)


def on_input_device(fn):
    """Run a method with the current device set to the device of its first
    tensor argument.  torch's default stream is the null stream (handle 0),
    which HIP resolves against the *current* device, and the library's side
    streams belong to the current device too: a caller whose tensors live on
    cuda:k but whose current device is another (the reference trainer picks
    cuda:k from `gpus` without set_device) would otherwise launch there."""
    import torch

    @functools.wraps(fn)
    def wrapped(*args, **kw):
        index = None
        for a in args:
            if isinstance(a, torch.Tensor):
                index = a.device.index if a.is_cuda else None
                break
        return _run_on(index, fn, args, kw)
    return wrapped


def on_self_device(fn):
    """on_input_device for methods of objects with a `device` attribute
    (TrainerPredictor, the device batch builders)."""
    @functools.wraps(fn)
    def wrapped(self, *args, **kw):
        dev = getattr(self, "device", None)
        index = dev.index if dev is not None and dev.type == "cuda" else None
        return _run_on(index, fn, (self,) + args, kw)
    return wrapped
