"""ctypes binding of libmpct.so (include/mpct.h).  The product path has NO CPU fallback: if the
HIP library is missing, importing the engine raises."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_CANDIDATES = ([os.environ["MPCT_LIB"]] if os.environ.get("MPCT_LIB") else []) + [
    os.path.join(_PKG, "csrc", "libmpct.so"),
    os.path.join(_HERE, "libmpct.so"),
]

c_int32_p = C.POINTER(C.c_int32)
c_double_p = C.POINTER(C.c_double)
c_int64_p = C.POINTER(C.c_int64)


class MpctDtf(C.Structure):
    _fields_ = [("len", C.c_int32), ("num", c_double_p), ("den", c_double_p), ("delay", C.c_int32)]


class MpctScenarioDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("my", C.c_int32), ("nu", C.c_int32), ("nd", C.c_int32),
        ("nit", C.c_int32),
        ("n2_max", C.c_int32), ("nu_max", C.c_int32),
        ("weights_squared", C.c_int32),
        ("vns_ink", C.c_int32),
        ("n1", c_int32_p),
        ("plant", C.POINTER(MpctDtf)),
        ("model", C.POINTER(MpctDtf)),
        ("na", c_int32_p),
        ("carima_A", c_double_p),
        ("nb", c_int32_p),
        ("carima_B", c_double_p),
        ("dp", c_int32_p),
        ("du_min", c_double_p), ("du_max", c_double_p),
        ("u_min", c_double_p), ("u_max", c_double_p),
        ("yref", c_double_p),
        ("dtc", C.c_int32),
        ("filter", C.POINTER(MpctDtf)),
        ("nq", C.c_int32),
        ("dist", C.POINTER(MpctDtf)),
        ("nplant", C.c_int32),
        ("plant_var", C.POINTER(MpctDtf)),
        ("mdband", C.c_int32),
        ("y_min", c_double_p), ("y_max", c_double_p),
        ("ecr_min", c_double_p), ("ecr_max", c_double_p),
        ("y_scale", c_double_p), ("u_scale", c_double_p),
        ("rho_ecr", C.c_double),
    ]


class MpctNmpcDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("model", C.c_int32),
        ("nx", C.c_int32), ("ny", C.c_int32), ("nu", C.c_int32),
        ("params", c_double_p), ("xc", c_int32_p),
        ("ts", C.c_double), ("nsub", C.c_int32),
        ("x0", c_double_p), ("u0", c_double_p),
        ("u_min", c_double_p), ("u_max", c_double_p),
        ("x_min", c_double_p), ("x_max", c_double_p),
        ("y_scale", c_double_p), ("u_scale", c_double_p),
        ("n_max", C.c_int32), ("nu_max", C.c_int32),
        ("nit", C.c_int32), ("yref", c_double_p), ("vns_ink", C.c_int32),
        ("sqp_max", C.c_int32), ("sqp_tol", C.c_double),
    ]


class MpctOpts(C.Structure):
    _fields_ = [("open_loop", C.c_int32), ("want_traj", C.c_int32), ("max_qp_iter", C.c_int32),
                ("device", C.c_int32), ("feas_tol", C.c_double)]


class MpctResult(C.Structure):
    _fields_ = [("J1", c_double_p), ("j21", c_double_p), ("j22", c_double_p), ("Jnu", c_double_p),
                ("status", c_int32_p), ("qp_iters", c_int64_p),
                ("y", c_double_p), ("u", c_double_p), ("ys", c_double_p), ("uopt", c_double_p)]


EXPORTS = [
    "mpct_abi_version", "mpct_last_error", "mpct_scenario_create", "mpct_scenario_destroy",
    "mpct_scenario_table", "mpct_eval_batch", "mpct_eval_batch_device", "mpct_lds_bytes", "mpct_lds_bytes_opts",
    "mpct_nmpc_scenario_create", "mpct_eval_batch_multi", "mpct_shard_candidates", "mpct_kernel_instance",
    "mpct_rank_device",
]

ABI_VERSION = 7
ST_QP_MAXITER, ST_QP_INFEAS, ST_NONFINITE, ST_SKIPPED, ST_BADHORIZON = 1, 2, 4, 8, 16
ST_SQP_MAXITER, ST_BOUNDS, ST_NOT_RUN = 32, 64, 128
NMPC_VANDEVUSSE = 1

_lib = None


def lib_path() -> str:
    override = os.environ.get("MPCT_LIB")  # e.g. the -DMPCT_PROFILE diagnostic build
    if override:
        return override
    for p in _CANDIDATES:
        if os.path.exists(p):
            return p
    raise ImportError(
        "libmpct.so not found (looked in %s). Build it with `python -c 'import __graft_entry__ as g; "
        "g.build()'` — the engine has no CPU fallback." % ", ".join(_CANDIDATES))


def load():
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64
    # (ROCm 7.0) and a second copy (/opt/rocm, 7.2) cannot open the device beside it.  Loading
    # torch first makes libmpct's NEEDED libamdhip64.so.7 bind to torch's copy by soname (libmpct
    # only uses hip_4.2-versioned symbols).  Without torch, the system runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(lib_path())
    lib.mpct_abi_version.restype = C.c_int32
    lib.mpct_last_error.restype = C.c_char_p
    lib.mpct_scenario_create.argtypes = [C.POINTER(MpctScenarioDesc), C.POINTER(C.c_void_p)]
    lib.mpct_scenario_create.restype = C.c_int32
    lib.mpct_nmpc_scenario_create.argtypes = [C.POINTER(MpctNmpcDesc), C.POINTER(C.c_void_p)]
    lib.mpct_nmpc_scenario_create.restype = C.c_int32
    lib.mpct_scenario_destroy.argtypes = [C.c_void_p]
    lib.mpct_scenario_destroy.restype = None
    lib.mpct_scenario_table.argtypes = [C.c_void_p, C.c_int32, c_double_p, C.c_int64]
    lib.mpct_scenario_table.restype = C.c_int64
    batch_args = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                  C.c_void_p, C.c_void_p, C.POINTER(MpctOpts), C.POINTER(MpctResult)]
    lib.mpct_eval_batch.argtypes = batch_args
    lib.mpct_eval_batch.restype = C.c_int32
    lib.mpct_eval_batch_device.argtypes = batch_args + [C.c_void_p]
    lib.mpct_eval_batch_device.restype = C.c_int32
    lib.mpct_lds_bytes.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    lib.mpct_lds_bytes.restype = C.c_int64
    lib.mpct_lds_bytes_opts.argtypes = [C.c_void_p, C.POINTER(MpctOpts), C.c_int32, C.c_int32]
    lib.mpct_lds_bytes_opts.restype = C.c_int64
    lib.mpct_eval_batch_multi.argtypes = [C.c_void_p, C.c_int32, c_int32_p] + batch_args[1:]
    lib.mpct_eval_batch_multi.restype = C.c_int32
    lib.mpct_shard_candidates.argtypes = [C.c_int64, C.c_int32, C.c_int32, c_int64_p, C.c_int64]
    lib.mpct_shard_candidates.restype = C.c_int64
    lib.mpct_kernel_instance.argtypes = [C.c_void_p, C.POINTER(MpctOpts), C.c_char_p, C.c_int32]
    lib.mpct_kernel_instance.restype = C.c_int32
    lib.mpct_rank_device.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.mpct_rank_device.restype = C.c_int32
    if lib.mpct_abi_version() != ABI_VERSION:
        raise ImportError("libmpct ABI version mismatch")
    _lib = lib
    return lib


def last_error() -> str:
    return load().mpct_last_error().decode(errors="replace")
