"""ctypes binding of libcsa_legacy.so (C ABI declared in include/csa_legacy.h).

The library is built in-tree by :func:`build` (``hipcc --offload-arch=gfx950``).
There is no fallback: if the library is missing or a call fails, the error is
raised to the caller.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.environ.get("CSA_LIB") or os.path.join(HERE, "libcsa_legacy.so")  # CSA_LIB: A/B builds
SRC = os.path.join(HERE, "csrc", "csa_legacy.hip")
SRC_MT = os.path.join(HERE, "csrc", "legacy_mt.cpp")   # host-only MT19937 mode
HEADER = os.path.join(REPO, "include", "csa_legacy.h")

CSA_OK = 0
CSA_E_INVALID = 1
CSA_E_BAD_QUOTAS = 2
CSA_E_NO_CANDIDATE = 3
CSA_E_ATTEMPT_LIMIT = 4
CSA_E_UNSUPPORTED = 5
CSA_E_HIP = 6
CSA_E_SELECTION = 7

CSA_WANT_PANELS = 0x1
CSA_WANT_COUNTS = 0x2
CSA_WANT_PAIRS = 0x4
CSA_WANT_UNIQUE = 0x8

CSA_PAIR_FP4 = 0
CSA_PAIR_I8 = 1
CSA_PAIR_OVERWRITE = 0x100  # engine flag: store this batch's pair counts instead of adding
CSA_PAIR_SHARED = 0x200     # engine hint: the launch overlaps concurrent draws
CSA_PAIR_ALONE = 0x400      # engine hint: nothing runs beside the launch (the kernel fastest alone)
CSA_DRAW_RESET_STATUS = 0x1  # csa_draw_xt_async flags: zero the status words, and the draw statistics,
CSA_DRAW_RESET_STATS = 0x2   # on the stream before the draw

# every symbol include/csa_legacy.h declares, with its ctypes signature
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
SIGNATURES = {
    "csa_version": (ctypes.c_int, []),
    "csa_last_error": (ctypes.c_char_p, []),
    "csa_device_count": (ctypes.c_int, [_P]),
    "csa_current_device": (ctypes.c_int, [_P]),
    "csa_instance_create": (ctypes.c_int, [_I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "csa_instance_destroy": (None, [_P]),
    "csa_instance_info": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "csa_instance_set_state": (ctypes.c_int, [_P, _P, _P, _P]),
    "csa_legacy_sample": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _U32, _P, _P, _P, _P, _P]),
    "csa_legacy_sample_devices": (ctypes.c_int, [_P, _P, _I32, _I32, _U64, _U64, _U64, _U32, _U32, _P, _P, _P,
                                                 _P, _P]),
    "csa_legacy_find": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _P]),
    "csa_legacy_attempt": (ctypes.c_int, [_P, _I32, _U64, _U64, _U32, _P, _P, _P, _P, _P]),
    "csa_first_panel_not_in": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _U64, _U64, _P, _P]),
    "csa_draw_round_panels": (ctypes.c_int, [_P, _I32, _P]),
    "csa_draw_async": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _P, _P, _P, _P, _P]),
    "csa_redraw_async": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _P, _P]),
    "csa_picks_stride": (_I32, [_I32]),
    "csa_draw_picks_supported": (ctypes.c_int, [_P, _I32]),
    "csa_draw_picks_async": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _P, _P, _P]),
    "csa_picks_pack_async": (ctypes.c_int, [_P, _U64, _I32, _I32, _P, _P, _P]),
    "csa_panel_hash_async": (ctypes.c_int, [_P, _U64, _I32, _P, _P]),
    "csa_draw_kernel_name": (ctypes.c_int, [_P, _I32, ctypes.c_char_p, _U64]),
    "csa_xt_pad": (_I32, [_I32]),
    "csa_transpose_count_async": (ctypes.c_int, [_P, _U64, _I32, _P, _P, _P]),
    "csa_pair_scratch_bytes": (_U64, [_I32, _U64, _U32]),
    "csa_pair_counts_ex_async": (ctypes.c_int, [_P, _U64, _I32, _P, _U32, _P, _U64, _P]),
    "csa_pair_counts_async": (ctypes.c_int, [_P, _U64, _I32, _P, _P]),
    "csa_unique_async": (ctypes.c_int, [_P, _P, _U64, _I32, _P, _U64, _P, _P, _P]),
    "csa_pair_histogram_async": (ctypes.c_int, [_P, _I32, _P, _U64, _P, _P]),
    "csa_unique_segments_async": (ctypes.c_int, [_P, _P, _U32, _U64, _P, _I32, _P, _U64, _P, _P, _P]),
    "csa_exchange_scratch_bytes": (_U64, [_U64]),
    "csa_exchange_pack_async": (ctypes.c_int, [_P, _P, _U64, _I32, _U32, _U64, _P, _U64, _P, _P, _P, _P, _P]),
    "csa_pairs_pack_async": (ctypes.c_int, [_P, _I32, _P, _P]),
    "csa_pairs_unpack_async": (ctypes.c_int, [_P, _I32, _P, _P]),
    "csa_pairs_upper_async": (ctypes.c_int, [_P, _I32, ctypes.c_double, _P, _P]),
    "csa_pairs_diag_async": (ctypes.c_int, [_P, _I32, _P, _P]),
    "csa_draw_xt_async": (ctypes.c_int, [_P, _I32, _U64, _U64, _U64, _U32, _P, _P, _P, _P, _P, _P, _U32, _P]),
    "csa_status_decode": (ctypes.c_int, [_P]),
    "csa_legacy_draw_mt": (ctypes.c_int, [_I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _U64, _U32,
                                          _I32, _P, _P, _P, _P, _P, _P, _P]),
    "csa_instance_set_address": (ctypes.c_int, [_P, _P]),
    "csa_instance_draw_stats": (ctypes.c_int, [_P, _I32, _P]),
    "csa_instance_draw_stats_reset": (ctypes.c_int, [_P, _P]),
    "csa_instance_draw_stats_async": (ctypes.c_int, [_P, _P, _P]),
    "csa_exchange_keys_async": (ctypes.c_int, [_P, _P, _U64, _I32, _U64, _U32, _U64, _P, _U64, _P, _P, _P, _P]),
    "csa_unique_keys_scratch_bytes": (_U64, [_U64, _I32]),
    "csa_unique_keys_async": (ctypes.c_int, [_P, _I32, _U64, _U32, _P, _U32, _U64, _P, _P, _U64, _P, _P, _P]),
}

_lib = None


class NativeLibraryError(RuntimeError):
    """libcsa_legacy.so is missing or failed to load (no CPU fallback exists)."""


class CsaError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("csa error %d: %s" % (code, message))
        self.code = code


def build(verbose=False):
    """Compile csrc/csa_legacy.hip for gfx950 into LIB_PATH (in-tree)."""
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", LIB_PATH, SRC, SRC_MT]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return LIB_PATH


def lib():
    """Load (once) and return the ctypes library; raises NativeLibraryError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            "%s not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); the LEGACY path has no CPU fallback" % LIB_PATH)
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError("failed to load %s: %s" % (LIB_PATH, e)) from e
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("CSA_LIB") and not hasattr(L, name):
            continue  # an older A/B build (CSA_LIB) may predate newer entry points
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    msg = lib().csa_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc):
    if rc != CSA_OK:
        raise CsaError(rc, last_error())
    return rc


def ptr(a):
    """Address of a numpy array / torch tensor (or None)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)
