"""ctypes binding of libsemops.so (include/sem_ops.h).

This is the only place Python touches the C ABI.  The library is built in-tree
(sem_amd/lib/libsemops.so, see sem_amd/build.py) and loaded from there; if it is
missing or fails to load, every entry point raises -- there is no CPU fallback.
Status codes are mapped the way the reference reports errors: SEM_EINVAL ->
ValueError (Solvers/SEM.py:18-19,108-109,158-159), anything else -> RuntimeError.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.environ.get("SEM_LIBDIR") or os.path.join(_HERE, "lib"), "libsemops.so")

ABI_VERSION = 15
SEM_OK, SEM_EINVAL, SEM_EHIP, SEM_ENOMEM, SEM_EUNSUPPORTED = 0, 1, 2, 3, 4
# kernel-selection knobs (include/sem_ops.h enum sem_tune; process-global, not thread-safe); the values between
# them are retired knobs (round 6), refused by sem_set_tuning
TUNE_BAND_TILE, TUNE_BAND_KP, TUNE_MFMA_TILE, TUNE_NS_APPLY, TUNE_EDGE_THOMAS = 0, 2, 4, 6, 7
TUNE_RETIRED = (1, 3, 5, 8, 9, 10, 11, 12)
SIDE_W, SIDE_E, SIDE_S, SIDE_N = 1, 2, 4, 8
DIR_NONE, DIR_IDENTITY, DIR_REPLACE = 0, 1, 2
ALGO_AUTO, ALGO_VALU, ALGO_MFMA, ALGO_COLUMN, ALGO_BAND = 0, 1, 2, 3, 4

_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)


class SemInfo(C.Structure):
    _fields_ = [("P", C.c_int), ("nex", C.c_int), ("ney", C.c_int), ("ex_begin", C.c_int), ("ex_end", C.c_int),
                ("device", C.c_int), ("dx", C.c_double), ("dy", C.c_double), ("NX", C.c_int64), ("NY", C.c_int64),
                ("N", C.c_int64), ("line_begin", C.c_int64), ("line_end", C.c_int64), ("n_local", C.c_int64),
                ("dof_begin", C.c_int64)]


class SemApplyDesc(C.Structure):
    _fields_ = [("c_mass", C.c_double), ("c_stiff", C.c_double), ("c_gradx", C.c_double), ("c_grady", C.c_double),
                ("cu", C.c_void_p), ("cv", C.c_void_p), ("c_extra", C.c_double), ("ea", C.c_void_p),
                ("eb", C.c_void_p), ("ec", C.c_void_p), ("ed", C.c_void_p), ("c_acc", C.c_double),
                ("dir_mode", C.c_int), ("dir_mask", C.c_void_p), ("dir_val", C.c_void_p), ("dir_sides", C.c_uint),
                ("algo", C.c_int), ("pos_begin", C.c_int), ("pos_end", C.c_int)]


class SemVelocityDesc(C.Structure):
    _fields_ = [("c_mass", C.c_double), ("c_stiff", C.c_double), ("c_gradx", C.c_double), ("c_grady", C.c_double),
                ("cu", C.c_void_p), ("cv", C.c_void_p), ("juu", C.c_void_p), ("juv", C.c_void_p), ("jvu", C.c_void_p),
                ("jvv", C.c_void_p), ("dir_mask", C.c_void_p), ("dir_sides", C.c_uint), ("ncomp", C.c_int),
                ("col_begin", C.c_int), ("col_end", C.c_int)]


class SemNestedDesc(C.Structure):
    _fields_ = [("P", C.c_int), ("nex", C.c_int), ("ney", C.c_int), ("nc", C.c_int), ("NY", C.c_int64),
                ("Xi", C.c_void_p), ("Aei", C.c_void_p), ("Yie", C.c_void_p), ("Se", C.c_void_p),
                ("pi", C.c_void_p), ("pe", C.c_void_p), ("T", C.c_void_p), ("C", C.c_void_p), ("Ye", C.c_void_p),
                ("Ed", C.c_void_p), ("El", C.c_void_p), ("Eu", C.c_void_p), ("XiB", C.c_void_p), ("AXB", C.c_void_p),
                ("ABY", C.c_void_p), ("Pw", C.c_void_p)]


class SemNsDesc(C.Structure):
    _fields_ = [("c_mass", C.c_double), ("c_stiff", C.c_double), ("c_gradx", C.c_double), ("c_grady", C.c_double),
                ("cu", C.c_void_p), ("cv", C.c_void_p), ("juu", C.c_void_p), ("juv", C.c_void_p), ("jvu", C.c_void_p),
                ("jvv", C.c_void_p), ("c_T", C.c_double), ("T", C.c_void_p), ("c_div", C.c_double),
                ("dval_u", C.c_void_p), ("dval_v", C.c_void_p), ("dir_mask", C.c_void_p), ("dir_sides", C.c_uint),
                ("pin_first", C.c_int), ("pin", C.c_int64), ("pin_val", C.c_double), ("uv_pitch", C.c_int64)]


class SemFrontLaunch(C.Structure):
    _fields_ = [("ntiles", C.c_int), ("rows", C.c_int), ("lanes", C.c_int), ("kmax", C.c_int), ("back", C.c_int),
                ("form", C.c_int), ("op", C.c_void_p),
                ("dims", C.c_void_p), ("xoff", C.c_void_p), ("yoff", C.c_void_p), ("tiles", C.c_void_p),
                ("xidx", C.c_void_p), ("yidx", C.c_void_p), ("W", C.c_void_p), ("stage", C.c_void_p)]


class SemLeafLaunch(C.Structure):
    _fields_ = [("nelem", C.c_int), ("n", C.c_int), ("ld", C.c_int), ("nb", C.c_int), ("nnz", C.c_int),
                ("stride", C.c_int64), ("blob", C.c_void_p), ("iidx", C.c_void_p), ("pat", C.c_void_p),
                ("W", C.c_void_p), ("stage", C.c_void_p), ("sstride", C.c_int64), ("soff", C.c_int64)]


# name -> (restype, argtypes); mirrors include/sem_ops.h one-for-one
_SIGS = {
    "sem_abi_version": (C.c_int, []),
    "sem_last_error": (C.c_char_p, []),
    "sem_max_order": (C.c_int, []),
    "sem_build_id": (C.c_char_p, []),
    "sem_set_tuning": (C.c_int, [C.c_int, C.c_int]),
    "sem_get_tuning": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "sem_gll_nodes": (C.c_int, [C.c_int, _dp, _dp, _dp]),
    "sem_gll_differentiation": (C.c_int, [C.c_int, _dp]),
    "sem_gll_gradient": (C.c_int, [C.c_int, _dp]),
    "sem_gll_stiffness": (C.c_int, [C.c_int, _dp]),
    "sem_gll_evaluation": (C.c_int, [C.c_int, _dp, C.c_int64, _dp]),
    "sem_global_index": (C.c_int, [C.c_int, C.c_int, C.c_int, _i64p, _i64p, _i64p, _i64p, C.c_int64, _i64p]),
    "sem_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int,
                             C.POINTER(C.c_void_p)]),
    "sem_destroy": (C.c_int, [C.c_void_p]),
    "sem_get_info": (C.c_int, [C.c_void_p, C.POINTER(SemInfo)]),
    "sem_apply": (C.c_int, [C.c_void_p, C.POINTER(SemApplyDesc), C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_kernel_name": (C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_int]),
    "sem_gather_elements": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_dss": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_eval_interpolation": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_interface_pack": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_int, C.c_void_p, C.c_void_p]),
    "sem_interface_unpack": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_int, C.c_void_p,
                                       C.c_void_p]),
    "sem_basis_dot2_work_size": (C.c_int64, [C.c_int, C.c_int64]),
    "sem_basis_dot2": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p]),
    "sem_basis_update": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_velocity_block_sizes": (C.c_int, [C.c_void_p, _i64p]),
    "sem_line_block_sizes": (C.c_int, [C.c_void_p, C.c_int, _i64p]),
    "sem_velocity_blocks": (C.c_int, [C.c_void_p, C.POINTER(SemVelocityDesc)] + [C.c_void_p] * 7),
    "sem_condensed_block_sizes": (C.c_int, [C.c_void_p, C.c_int, _i64p]),
    "sem_condensed_blocks": (C.c_int, [C.c_void_p, C.POINTER(SemVelocityDesc)] + [C.c_void_p] * 12),
    "sem_ns_apply": (C.c_int, [C.c_void_p, C.POINTER(SemNsDesc)] + [C.c_void_p] * 7),
    "sem_nested_solve": (C.c_int, [C.POINTER(SemNestedDesc), C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_int64, C.c_void_p]),
    "sem_nested_back_solve": (C.c_int, [C.POINTER(SemNestedDesc), C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_int64, C.c_void_p]),
    "sem_nested_iface_rhs": (C.c_int, [C.POINTER(SemNestedDesc), C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                       C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
    "sem_interface_rhs": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_int64, C.c_void_p, C.c_void_p]),
    "sem_block_gemv": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p), _i64p, C.c_void_p,
                                 C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]),
    "sem_dense_inverse_small": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]),
    "sem_givens_column": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "sem_gemv_rows2": (C.c_int, [C.c_int, C.c_double, C.c_double, C.c_int, C.c_void_p, C.c_int64, C.c_void_p,
                                 C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sem_front_gemv": (C.c_int, [C.POINTER(SemFrontLaunch), C.c_void_p]),
    "sem_leaf_forward": (C.c_int, [C.POINTER(SemLeafLaunch), C.c_void_p]),
    "sem_front_sparse_rows": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                        C.c_int64, C.c_void_p]),
    "sem_front_scatter": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p]),
    "sem_gemv_rows": (C.c_int, [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_int64, C.c_void_p, C.c_double,
                                C.c_void_p, C.c_void_p]),
}

_lib = None


def load():
    """Load libsemops.so (building it first if sources are newer).  Raises if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    # Build only when the library is absent (or SEM_AUTOBUILD=1 asks for a staleness check):
    # snapshot copies reset mtimes, and concurrent ranks must not race a rebuild.
    if not os.path.exists(LIB_PATH) or os.environ.get("SEM_AUTOBUILD", "0") == "1":
        try:
            from . import build as _build
            _build.build()
        except Exception as e:  # noqa: BLE001 - surface the real reason below
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libsemops.so is missing and could not be built: {e}") from e
    lib = C.CDLL(LIB_PATH)
    if not hasattr(lib, "sem_build_id") or lib.sem_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH} was built for another ABI version; rebuild: python -m sem_amd.build")
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _check_build_id(lib)
    _lib = lib
    return lib


def _check_build_id(lib):
    """The library must be built from the sources in this tree (a stale .so would make the GPU
    tests validate old kernels), and must not be a diagnostic build unless asked for."""
    bid = lib.sem_build_id().decode()
    base, diag = bid.split("+")[0], bid.endswith("+diag")
    if diag and os.environ.get("SEM_ALLOW_DIAG", "0") != "1":
        raise RuntimeError(f"{LIB_PATH} is a diagnostic build (SEM_DIAGNOSTICS=1); set SEM_ALLOW_DIAG=1 to use it")
    try:
        from .build import source_hash
        want = source_hash()
    except OSError:  # sources not shipped with this tree: nothing to compare against
        return
    if base != want:
        raise RuntimeError(f"{LIB_PATH} (build id {bid}) was not built from the sources in this tree "
                           f"(hash {want}); rebuild: python -m sem_amd.build")


def check(status):
    if status == SEM_OK:
        return
    msg = load().sem_last_error().decode(errors="replace")
    if status == SEM_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(f"libsemops error {status}: {msg}")


def exported_symbols():
    return list(_SIGS)
