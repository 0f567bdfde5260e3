"""ctypes binding of libccmpc.so (include/ccmpc.h).

The library is built in-tree (``cc-mpc_amd/csrc/Makefile`` -> ``cc-mpc_amd/ccmpc/libccmpc.so``)
so it travels with the repository snapshot.  There is no fallback: if the library is missing or
its ABI does not match, every entry point raises.
"""
import ctypes
import os

import numpy as np

LIB_PATH = os.environ.get(
    "CCMPC_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libccmpc.so"))
ABI_VERSION = 2

CCMPC_OK = 0
CCMPC_F64 = 0
CCMPC_F32 = 1
GMM_PER_LATENT, GMM_PER_PARTICLE = 0, 1

STATUS = {
    0: "ok", -1: "invalid argument", -2: "kernel launch failed", -3: "workspace too small",
    -4: "unsupported configuration", -10: "singular", -11: "no tangent", -12: "non-finite",
    -13: "not PD", -14: "not PSD",
}

REC_SINGULAR, REC_NO_TANGENT, REC_NONFINITE, REC_NOT_PD, REC_NOT_PSD = -10, -11, -12, -13, -14

# record layouts (ccmpc_halfspace / ccmpc_affine_rec, 128 bytes each)
HALFSPACE_DTYPE = np.dtype([
    ("n0", "<f8"), ("n1", "<f8"), ("d", "<f8"),
    ("q00", "<f8"), ("q01", "<f8"), ("q11", "<f8"),
    ("r00", "<f8"), ("r01", "<f8"), ("r11", "<f8"),
    ("beta1", "<f8"), ("beta2", "<f8"), ("lower_bound", "<f8"),
    ("mean0", "<f8"), ("mean1", "<f8"),
    ("which", "<i4"), ("side", "<i4"), ("status", "<i4"), ("t_tau", "<i4"),
])
AFFINE_DTYPE = np.dtype([
    ("n0", "<f8"), ("n1", "<f8"), ("d", "<f8"), ("margin", "<f8"), ("rhs", "<f8"),
    ("mean0", "<f8"), ("mean1", "<f8"),
    ("c00", "<f8"), ("c01", "<f8"), ("c11", "<f8"),
    ("s00", "<f8"), ("s01", "<f8"), ("s11", "<f8"), ("m", "<f8"),
    ("which", "<i4"), ("side", "<i4"), ("status", "<i4"), ("t", "<i4"),
])
assert HALFSPACE_DTYPE.itemsize == 128 and AFFINE_DTYPE.itemsize == 128

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_U64 = ctypes.c_uint64
_D = ctypes.c_double
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); the exact export list of include/ccmpc.h
SIGNATURES = {
    "ccmpc_abi_version": (ctypes.c_int, []),
    "ccmpc_last_error": (ctypes.c_char_p, []),
    "ccmpc_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "ccmpc_copy_async": (ctypes.c_int, [_P, _P, _SZ, _P]),
    "ccmpc_copy_kernel_async": (ctypes.c_int, [_P, _P, _SZ, _P]),
    "ccmpc_graph_capture_begin": (ctypes.c_int, [_P]),
    "ccmpc_graph_capture_end": (ctypes.c_int, [_P, _P]),
    "ccmpc_graph_launch": (ctypes.c_int, [_P, _P]),
    "ccmpc_signal_host": (ctypes.c_int, [_P, _P, _P]),
    "ccmpc_copy_signal_async": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P]),
    "ccmpc_graph_destroy": (ctypes.c_int, [_P]),
    "ccmpc_moments_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "ccmpc_moments": (ctypes.c_int, [_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _I64, _I64, _P,
                                     _SZ, _P, _P, _P]),
    "ccmpc_minkowski": (ctypes.c_int, [_P, _P, _I64, _I64, _P, _P, _P, _D, _D, _I32, _P, _P,
                                       _P]),
    "ccmpc_affine": (ctypes.c_int, [_P, _P, _I64, _I64, _P, _P, _P, _D, _P, _P]),
    "ccmpc_minkowski_cycle_args": (ctypes.c_int, [_P]),
    "ccmpc_cycle_args_size": (_SZ, []),
    "ccmpc_minkowski_cycle": (ctypes.c_int, [_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _I64,
                                             _I64, _P, _SZ, _P, _P, _P, _D, _D, _I32, _P, _P,
                                             _P, _P, _P]),
    "ccmpc_ideal_minkowski_cycle": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _P, _U64,
                                                   _P, _P, _SZ, _P, _P, _P, _D, _D, _I32, _P,
                                                   _P, _P, _P, _P, _P]),
    "ccmpc_ideal_minkowski_cycle_ex": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _P,
                                                      _U64, _P, _P, _P, _SZ, _P, _P, _P, _D, _D,
                                                      _I32, _P, _P, _P, _P, _P, _P]),
    "ccmpc_sample_unicycle": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _D, _U64, _I64,
                                             _P, _P, _I64, _P]),
    "ccmpc_sample_unicycle_ex": (ctypes.c_int, [_P, _P, _I64, _P, _I32, _P, _P, _I64, _I64, _I64,
                                                _D, _U64, _P, _I64, _P, _P, _I64, _P]),
    "ccmpc_bucket_workspace_bytes": (_SZ, [_I64, _I64, _I64, _I64]),
    "ccmpc_bucket": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _I64, _P,
                                    _P, _P, _SZ, _P, _I64, _P, _P, _P, _P, _P]),
    "ccmpc_compact_records": (ctypes.c_int, [_P, ctypes.c_int, _I64, _P, _P]),
    "ccmpc_load_predictions": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _I64, _I64, _I64, _I64,
                                              _P, _I64, _I64, _P, _P, _P]),
    "ccmpc_bucket_predictions": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _I64, _I64, _I64,
                                                _I64, _P, _P, _P, _I64, _P, _P, _P, _SZ, _P,
                                                _I64, _P, _P, _P, _P, _P, _P]),
    "ccmpc_bucket_predictions_indirect": (ctypes.c_int, [_P, ctypes.c_int, _P, _I64, _I64, _I64,
                                                         _I64, _P, _P, _P, _I64, _P, _P, _P, _SZ,
                                                         _P, _I64, _P, _P, _P, _P, _P, _P]),
    "ccmpc_bucket_predictions_packed": (ctypes.c_int, [_P, _P, _SZ, _P, _P, ctypes.c_int, _P,
                                                       _I64, _I64, _I64, _I64, _P, _P, _P, _I64,
                                                       _P, _P, _P, _SZ, _P, _I64, _P, _P, _P, _P,
                                                       _P, _P]),
    "ccmpc_bucket_predictions_indirect_packed": (ctypes.c_int, [_P, _P, _SZ, _P, ctypes.c_int,
                                                                _P, _I64, _I64, _I64, _I64, _P,
                                                                _P, _P, _I64, _P, _P, _P, _SZ,
                                                                _P, _I64, _P, _P, _P, _P, _P,
                                                                _P]),
    "ccmpc_sample_bucket_packed": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _I64, _P, _I32, _P, _P,
                                                  _I64, _I64, _I64, _D, _U64, _P, _I64, _P, _P,
                                                  _P, _I64, _P, _P, _P, _SZ, _P, _P, _I64, _P,
                                                  _P, _P, _P, _P]),
    "ccmpc_sample_bucket_workspace_bytes": (_SZ, [_I64, _I64, _I64, _I64]),
    "ccmpc_sample_bucket": (ctypes.c_int, [_P, _P, _I64, _P, _I32, _P, _P, _I64, _I64, _I64, _D,
                                           _U64, _P, _I64, _P, _P, _P, _I64, _P, _P, _P, _SZ, _P,
                                           _P, _I64, _P, _P, _P, _P, _P]),
    "ccmpc_affine_scale": (ctypes.c_int, [_P, _P, _I64, _I64, _P, _P, _P, _D, _I32, _P, _P, _P,
                                          _P]),
    "ccmpc_ideal_rollout": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _P, _P, _U64,
                                           _P, _P, _I64, _P, _P]),
    "ccmpc_ideal_moments_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "ccmpc_l4": (ctypes.c_int, [_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _I64, _P, _P, _P, _P,
                                _P, _P, _P, _P, _P]),
    "ccmpc_l4_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "ccmpc_l4_split": (ctypes.c_int, [_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _I64, _I64, _P,
                                      _P, _P, _SZ, _P, _P, _P, _P, _P, _P, _P]),
    "ccmpc_ideal_moments": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _P, _U64, _P,
                                           _P, _SZ, _P, _P, _P, _P]),
    "ccmpc_mpc_ltv": (ctypes.c_int, [_P, _I64, _I64, _D, _D, _D, _P, _P, _P]),
    "ccmpc_mpc_qp_workspace_bytes": (_SZ, [_I64, _I64, _I64, ctypes.c_int]),
    "ccmpc_mpc_qp": (ctypes.c_int, [_I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _I64, _P,
                                    ctypes.c_int, _P, _I64, _P, ctypes.c_int, _I32, _D, _P, _SZ,
                                    _P, _P, _P, _P, _P, _P]),
    "ccmpc_mpc_qp_ltv": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _I64, _P,
                                        ctypes.c_int, _P, _I64, _P, ctypes.c_int, _I32, _D, _P,
                                        _SZ, _P, _P, _P, _P, _P, _P]),
    "ccmpc_selftest": (ctypes.c_int, [ctypes.c_int, _I64, _P, _P, _D, _I32, _P]),
    "ccmpc_poison_lds": (ctypes.c_int, [_D, _P]),
}

SELFTEST_MVOE, SELFTEST_TANGENT, SELFTEST_BOUND, SELFTEST_PAIR = 0, 1, 2, 3


class CycleArgs(ctypes.Structure):
    """ccmpc_cycle_args (include/ccmpc.h): ccmpc_minkowski_cycle's arguments in one struct."""
    _fields_ = [("positions", _P), ("dtype", ctypes.c_int32), ("maxiter", ctypes.c_int32),
                ("ld", ctypes.c_int64), ("T", ctypes.c_int64), ("origin", _P),
                ("cell_off", _P), ("cell_cnt", _P), ("n_cells", ctypes.c_int64),
                ("n_particles_bound", ctypes.c_int64), ("workspace", _P),
                ("workspace_bytes", ctypes.c_size_t), ("ref_traj", _P), ("cell_ref", _P),
                ("cell_risk", _P), ("R", ctypes.c_double), ("tol", ctypes.c_double),
                ("out_mean", _P), ("out_cov", _P), ("out_rec", _P), ("out_prob_lower", _P),
                ("stream", _P)]


class CcmpcError(RuntimeError):
    pass


_lib = None


def load():
    """Load libccmpc.so once; raise loudly if it is missing or has the wrong ABI."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CcmpcError(
            f"libccmpc.so not found at {LIB_PATH}: build it with `make -C cc-mpc_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ccmpc_abi_version() != ABI_VERSION:
        raise CcmpcError(f"libccmpc ABI {lib.ccmpc_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


class NonFiniteRecordError(ValueError, TypeError):
    """A record whose inputs or outputs are inf/NaN.  The reference fails at different places
    for these, with different exception types: N_k < 2 gives a NaN np.cov that
    scipy.linalg.solve rejects (ValueError, makeconstraint.py:21); ref_y == mean_y gives an
    infinite slope whose candidate distances are NaN, so choose_closest_tangent indexes its
    candidates with None (TypeError, makeconstraint.py:194-205).  Both types are caught."""


def record_error(status, where):
    """The exception the reference raises where a record carries `status` (CCMPC_REC_*):
    SINGULAR / NOT_PD -> np.linalg.LinAlgError (np.linalg.inv, scipy.linalg.solve,
    np.linalg.cholesky); NO_TANGENT -> ValueError (v8ideal/__init__.py:925 unpacks
    choose_closest_tangent's 4-tuple of None into 3 names); NONFINITE / NOT_PSD ->
    NonFiniteRecordError."""
    msg = f"{where}: {STATUS.get(int(status), status)}"
    status = int(status)
    if status in (REC_SINGULAR, REC_NOT_PD):
        return np.linalg.LinAlgError(msg)
    if status == REC_NO_TANGENT:
        return ValueError(msg + " (too many values to unpack: the reference's None tuple)")
    return NonFiniteRecordError(msg)


def check(rc, what):
    if rc != CCMPC_OK:
        msg = load().ccmpc_last_error().decode(errors="replace")
        raise CcmpcError(f"{what} failed ({STATUS.get(rc, rc)}): {msg}")
