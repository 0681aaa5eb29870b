"""ctypes binding of libolpe.so (include/olpe.h).

There is no fallback: if the library is missing or cannot be loaded, importing the
sampler raises.  Build it with ``python -m olpefit_amd.build`` (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OLPE_LIB", os.path.join(HERE, "libolpe.so"))

OK, EINVAL, EHIP, ENOMEM, ESTATE, ECOMM, EIO = 0, -1, -2, -3, -4, -5, -6
DTYPE_F32, DTYPE_F64 = 0, 1
EVAL_EXACT, EVAL_FAST = 0, 1


class OlpeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"olpe error {code}: {msg}")
        self.code = code


_P = C.c_void_p
_i = C.c_int
_ll = C.c_longlong
_d = C.c_double
_pd = C.POINTER(C.c_double)
_pu32 = C.POINTER(C.c_uint32)
_pu8 = C.POINTER(C.c_uint8)
_pll = C.POINTER(C.c_longlong)

#: name -> (restype, argtypes); mirrors include/olpe.h and the test hooks of
#: include/olpe_test.h one-to-one
SIGNATURES = {
    "olpe_version": (_i, []),
    "olpe_device_count": (_i, [C.POINTER(_i)]),
    "olpe_device_mem": (_i, [_i, _pll, _pll]),
    "olpe_device_pci_id": (_i, [_i, C.c_char_p, _i]),
    "olpe_last_error": (C.c_char_p, []),
    "olpe_create": (_i, [_P, _i, _P, _d, _pu8, _i, _i, _i, _i, _i, C.POINTER(_P)]),
    "olpe_destroy": (None, [_P]),
    "olpe_set_eval_mode": (_i, [_P, _i]),
    "olpe_model": (_i, [_P, _pd, _pd]),
    "olpe_chi2_batch": (_i, [_P, _pd, _i, _pd]),
    "olpe_seed": (_i, [_P, _pu32, _i]),
    "olpe_state_set": (_i, [_P, _pd, _pd, _pd]),
    "olpe_state_get": (_i, [_P, _pd, _pd, _pd]),
    "olpe_run": (_i, [_P, _ll, _ll, _i, _ll, _pll]),
    "olpe_chain_read": (_i, [_P, _pd]),
    "olpe_count": (_i, [_P, _pll]),
    "olpe_count_reset": (_i, [_P, _ll]),
    "olpe_done_at": (_i, [_P, _pll]),
    "olpe_run_gibbs": (_i, [_P, _pd, _pd, _pd, _i, _ll, _ll, _i, _pd]),
    "olpe_rng_get": (_i, [_P, _pu32, _pd]),
    "olpe_rng_set": (_i, [_P, _pu32, _pd]),
    "olpe_rng_stream": (_i, [_P, _i, _i, _P]),
    "olpe_trace_enable": (_i, [_P, _i]),
    "olpe_trace_read": (_i, [_P, _pd]),
    "olpe_sync": (_i, [_P]),
    "olpe_last_kernel_ms": (_i, [_P, _pd]),
    "olpe_kernel_times": (_i, [_P, _i, _pd]),
    "olpe_last_units": (_i, [_P, C.POINTER(C.c_int)]),
    "olpe_unit_stats": (_i, [_P, _pll]),
    "olpe_csv_format": (_i, [_pd, _ll, _i, _i, C.c_char_p, C.c_size_t,
                             C.POINTER(C.c_size_t)]),
    "olpe_csv_write_chains": (_i, [C.POINTER(C.c_char_p), _pd, _i, _ll, _i, _i, _i]),
    "olpe_csv_append_chains": (_i, [C.POINTER(C.c_char_p), _pd, _i, _ll, _ll, _i, _i, _pll]),
    "olpe_csv_shape": (_i, [C.c_char_p, _pll, C.POINTER(_i)]),
    "olpe_csv_read_chains": (_i, [C.POINTER(C.c_char_p), _i, _ll, _i, _ll, _pd, _i]),
    "olpe_acceptance_format": (_i, [_pd, _i, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "olpe_acceptance_write": (_i, [C.POINTER(C.c_char_p), _pd, _pd, _i, _i, _i, _pu8]),
    "olpe_moments_accumulate": (_i, [_P]),
    "olpe_moments_reset": (_i, [_P]),
    "olpe_moments_get": (_i, [_P, _pll, _pd, _pd]),
    "olpe_moments_set": (_i, [_P, _ll, _pd, _pd]),
    "olpe_moments_summary": (_i, [_P, _pd, _pd]),
    "olpe_comm_unique_id": (_i, [_pu8]),
    "olpe_comm_init": (_i, [_P, _pu8, _i, _i]),
    "olpe_comm_timeout": (_i, [_P, _d]),
    "olpe_comm_info": (_i, [_P, C.POINTER(_i), C.POINTER(_i)]),
    "olpe_comm_allgather_state": (_i, [_P, _pd]),
    "olpe_comm_allgather_chain": (_i, [_P, _ll, _ll, _pd, _pll]),
    "olpe_comm_gather_limit": (_i, [_P, _ll]),
    "olpe_comm_allreduce_moments": (_i, [_P, _pd]),
    "olpe_moments_fault": (_i, [_P, _i]),
    "olpe_test_hold_handoff": (_i, [_P, _i]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load libolpe.so and attach the signatures.  Raises OSError if missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"libolpe.so not found at {path}: build it with "
                      "`python -m olpefit_amd.build` (hipcc, gfx950)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != OK:
        msg = load().olpe_last_error().decode(errors="replace")
        raise OlpeError(rc, msg)
