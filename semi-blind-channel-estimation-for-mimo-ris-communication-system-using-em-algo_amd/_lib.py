"""ctypes binding of libsbce.so (C-ABI declared in include/sbce.h).

This is the ONLY way the package reaches its compute path.  There is no CPU
fallback: if the shared library is missing, or no HIP device is visible, the
calls raise ``SbceUnavailable``.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsbce.so")
# the A/B build (csrc/sbce_internal.h SBCE_AB): the same C-ABI plus the SBCE_* switches; loaded
# only by debug_env() (tests' cross-checks, tools), never by the product path
AB_LIB_PATH = os.path.join(_HERE, "libsbce_ab.so")

SBCE_ABI_VERSION = 6
SBCE_ESTEP_SOFT = 0
SBCE_ESTEP_HARD = 1
SBCE_ESTEP_PM = 2
SBCE_ESTEP_PM_SOFT = 3
SBCE_ESTEP_ZF = 4
SBCE_ESTEP_MMSE = 5
SBCE_ESTEP_GAUSS = 6
SBCE_SOLVE_CHOL = 0
SBCE_SOLVE_CHOL_DROP = 1
SBCE_SOLVE_MINNORM = 2
SBCE_STATUS_NONHPD = 1
SBCE_STATUS_PILOT = 2
SBCE_STATUS_DETECTOR = 4
SBCE_STATUS_DEBUG = 8
SBCE_STATUS_RANK = 16

EXPORTED = ("sbce_abi_version", "sbce_strerror", "sbce_workspace_bytes",
            "sbce_workspace_bytes_solve", "sbce_em",
            "sbce_estep", "sbce_mstep", "sbce_ser", "sbce_gauss_expand", "sbce_nmse")


class SbceUnavailable(RuntimeError):
    """libsbce.so is not built or no GPU is available (the product never falls back)."""


class SbceError(RuntimeError):
    pass


class Dims(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("n_tx", ctypes.c_int32), ("n_rx", ctypes.c_int32),
                ("n_psi", ctypes.c_int32), ("t_p", ctypes.c_int32), ("t_d", ctypes.c_int32),
                ("m", ctypes.c_int32), ("partition_r", ctypes.c_int32), ("varn", ctypes.c_double),
                ("varx", ctypes.c_double)]


class Ptrs(ctypes.Structure):
    _fields_ = [("y_d", ctypes.c_void_p), ("y_p", ctypes.c_void_p), ("psi_d", ctypes.c_void_p),
                ("u_p", ctypes.c_void_p), ("cons", ctypes.c_void_p), ("theta", ctypes.c_void_p),
                ("x_d_true", ctypes.c_void_p), ("llf", ctypes.c_void_p),
                ("h_true", ctypes.c_void_p), ("iters_done", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("workspace", ctypes.c_void_p),
                ("workspace_bytes", ctypes.c_size_t), ("x_dest", ctypes.c_void_p),
                ("x_sup", ctypes.c_void_p), ("varn_t", ctypes.c_void_p)]


_lib = None
_ab = None
_ab_active = 0


def load(path=None):
    """Load libsbce.so (CPU-safe: loading does not touch the GPU).

    PyTorch is imported FIRST: its ROCm wheel ships its own HIP runtime (torch/lib/libamdhip64.so,
    SONAME libamdhip64.so.7), and the device buffers and streams this library receives come from
    that runtime.  Loaded after it, libsbce.so's NEEDED libamdhip64.so.7 resolves to the same
    already-loaded runtime; loaded before it, the system /opt/rocm runtime would come in as well
    and the process would run two HIP runtimes (the second to initialise finds no device:
    hipErrorNoDevice on every launch)."""
    global _lib
    if path is None and _ab_active:
        return load_ab()
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise SbceUnavailable(f"{p} not built: run __graft_entry__.build()")
    import torch  # noqa: F401  (the HIP runtime this library must share; no GPU is touched)
    lib = ctypes.CDLL(p)
    lib.sbce_abi_version.restype = ctypes.c_int
    lib.sbce_abi_version.argtypes = []
    lib.sbce_strerror.restype = ctypes.c_char_p
    lib.sbce_strerror.argtypes = [ctypes.c_int]
    lib.sbce_workspace_bytes.restype = ctypes.c_int
    lib.sbce_workspace_bytes.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(ctypes.c_size_t)]
    lib.sbce_workspace_bytes_solve.restype = ctypes.c_int
    lib.sbce_workspace_bytes_solve.argtypes = [ctypes.POINTER(Dims), ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_size_t)]
    lib.sbce_em.restype = ctypes.c_int
    lib.sbce_em.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Ptrs), ctypes.c_int,
                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.sbce_estep.restype = ctypes.c_int
    lib.sbce_estep.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Ptrs), ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
    lib.sbce_mstep.restype = ctypes.c_int
    lib.sbce_mstep.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Ptrs), ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.sbce_ser.restype = ctypes.c_int
    lib.sbce_ser.argtypes = [ctypes.POINTER(Dims), ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p]
    lib.sbce_gauss_expand.restype = ctypes.c_int
    lib.sbce_gauss_expand.argtypes = [ctypes.POINTER(Dims), ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
    lib.sbce_nmse.restype = ctypes.c_int
    lib.sbce_nmse.argtypes = [ctypes.POINTER(Dims), ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p]
    if lib.sbce_abi_version() != SBCE_ABI_VERSION:
        raise SbceUnavailable("libsbce ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def load_ab():
    """The A/B build libsbce_ab.so (same C-ABI; the SBCE_* switches live only there)."""
    global _ab
    if _ab is None:
        _ab = load(AB_LIB_PATH)
    return _ab


def use_ab():
    """Route every later load() to the A/B build for the rest of the process (development
    tools only: A/B arms, counters, clocks)."""
    global _ab_active
    _ab_active += 1
    return load_ab()


def reload_debug_env():
    """Re-read the SBCE_* A/B switches (include/sbce.h SBCE_STATUS_DEBUG) into the A/B library;
    they are otherwise read once, when libsbce_ab.so is loaded.  Returns True when a
    result-affecting switch is active."""
    lib = load_ab()
    lib.sbce_debug_reload_env.restype = ctypes.c_int
    return lib.sbce_debug_reload_env() == 1


@contextlib.contextmanager
def debug_env(**env):
    """Run a block on the A/B library with SBCE_* debug switches set (diagnostics and A/B tests
    only): ``with debug_env(SBCE_ESTEP_IMPL="valu"): ...``.  Inside the block load() -- and so
    every package call and engine made there -- returns libsbce_ab.so; the environment is
    restored after.  The product library libsbce.so has no switches."""
    global _ab_active
    old = {k: os.environ.get(k) for k in env}
    _ab_active += 1
    try:
        for k, v in env.items():
            os.environ[k] = str(v)
        reload_debug_env()
        yield load_ab()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        reload_debug_env()
        _ab_active -= 1


def check(rc, what):
    if rc != 0:
        msg = load().sbce_strerror(rc).decode()
        raise SbceError(f"{what} failed: {msg} ({rc})")


def workspace_bytes(dims, solve=None):
    """Workspace of sbce_em / sbce_mstep for `dims`: for every solve mode (solve=None) or for
    one SBCE_SOLVE_* mode (sbce_workspace_bytes_solve)."""
    n = ctypes.c_size_t(0)
    if solve is None:
        check(load().sbce_workspace_bytes(ctypes.byref(dims), ctypes.byref(n)),
              "sbce_workspace_bytes")
    else:
        check(load().sbce_workspace_bytes_solve(ctypes.byref(dims), int(solve), ctypes.byref(n)),
              "sbce_workspace_bytes_solve")
    return n.value
