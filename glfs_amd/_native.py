"""ctypes binding of glfs_amd/libglfsx.so (the C-ABI in include/glfsx.h).

The native library is the product: every hash / encrypt call below runs in
the gfx950 HIP kernels.  There is no Python or CPU fallback -- if the library
is missing this module raises at import, and if no GPU is visible every
compute call raises DeviceError (GLFSX_E_DEVICE).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# GLFSX_LIB: an alternative build of the same library (A/B tuning runs only)
LIB_PATH = os.environ.get("GLFSX_LIB") or os.path.join(_HERE, "libglfsx.so")

GLFSX_OK = 0
GLFSX_E_BLOCKSIZE_GT_MAX = -1
GLFSX_E_BLOCKSIZE_LT_MIN = -2
GLFSX_E_STORE = -3
GLFSX_E_DEVICE = -4
GLFSX_E_ARG = -5
GLFSX_E_UNSUPPORTED = -6
GLFSX_E_NOMEM = -7
GLFSX_E_IO = -8
GLFSX_STORE_TRUST = 0
GLFSX_STORE_HASH = 1


class GlfsxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"glfsx error {code}: {msg}")
        self.code = code


class Panic(GlfsxError):
    """Where the reference panics (blob.go:91, blob.go:94)."""


class StoreError(GlfsxError):
    """A store.Post failure (blob.go:153-156, 175-178)."""


class DeviceError(GlfsxError):
    """No usable HIP device / HIP runtime failure."""


class glfsx_root(ctypes.Structure):
    _fields_ = [("ref", ctypes.c_uint8 * 64), ("size", ctypes.c_uint64),
                ("block_size", ctypes.c_uint64)]


POST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_uint8), ctypes.c_void_p,
                           ctypes.c_uint64)
# glfsx_read_at_fn: io.ReaderAt.ReadAt(ctx, buf, len, off) -> count / 0 / < 0
READ_AT_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_uint64, ctypes.c_uint64)

# Every entry point declared in include/glfsx.h (tests/test_abi.py checks the
# header and the .so against this list).
_VP, _U64, _SZ, _INT, _CP = (ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t,
                             ctypes.c_int, ctypes.c_char_p)
SIGNATURES = {
    "glfsx_last_error": (_CP, []),
    "glfsx_device_count": (_INT, []),
    "glfsx_set_device": (_INT, [_INT]),
    "glfsx_version": (_CP, []),
    "glfsx_set_split_target": (ctypes.c_uint32, [ctypes.c_uint32]),
    "glfsx_set_latency_wgs": (ctypes.c_uint32, [ctypes.c_uint32]),
    "glfsx_debug_fused": (_U64, [ctypes.c_uint32, _U64]),
    "glfsx_fused_failures": (_U64, []),
    "glfsx_debug_one_drop": (None, [ctypes.c_uint32]),
    "glfsx_clock_probe": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    "glfsx_one_stats": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    "glfsx_derive_key": (_INT, [_VP, _SZ, _CP, _VP, _SZ]),
    "glfsx_post": (_INT, [_CP, _VP, _U64, _VP, _VP, _CP]),
    "glfsx_post_batch": (_INT, [_CP, _VP, _U64, _U64, _VP, _VP, _CP]),
    "glfsx_post_batch_device": (_INT, [_CP, _VP, _U64, _U64, _VP, _VP, _CP, _VP]),
    "glfsx_dek_batch_device": (_INT, [_CP, _VP, _U64, _U64, _VP, _VP]),
    "glfsx_cid_batch_device": (_INT, [_VP, _U64, _U64, _VP, _VP, _CP, _VP]),
    "glfsx_writer_new": (_VP, [_U64, _U64, _CP, _CP, POST_FN, _VP,
                               ctypes.POINTER(ctypes.c_int)]),
    "glfsx_writer_write": (_INT, [_VP, _VP, _SZ]),
    "glfsx_writer_flush": (_INT, [_VP]),
    "glfsx_writer_copy": (_INT, [_VP, _VP, _U64, _U64]),
    "glfsx_writer_reserve": (_INT, [_VP, ctypes.POINTER(ctypes.c_void_p),
                                    ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_writer_commit": (_INT, [_VP, _U64]),
    "glfsx_writer_read_at": (_INT, [_VP, READ_AT_FN, _VP, _U64, _U64,
                                    ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_writer_read_fd": (_INT, [_VP, _INT, _U64, _U64, ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_writer_write_device": (_INT, [_VP, _VP, _SZ, _VP]),
    "glfsx_writer_write_ctext": (_INT, [_VP, _VP, _U64, _U64, _VP]),
    "glfsx_writer_write_ctext_blocks": (_INT, [_VP, _VP, _U64, _U64, _U64, _VP]),
    "glfsx_writer_set_strict": (_INT, [_VP, _INT]),
    "glfsx_writer_set_devices": (_INT, [_VP, _VP, _INT]),
    "glfsx_writer_error": (_CP, [_VP]),
    "glfsx_writer_finish": (_INT, [_VP, ctypes.POINTER(glfsx_root)]),
    "glfsx_writer_free": (None, [_VP]),
    "glfsx_create": (_INT, [_U64, _U64, _CP, _CP, _VP, _U64, POST_FN, _VP,
                            ctypes.POINTER(glfsx_root)]),
    "glfsx_create_device": (_INT, [_U64, _CP, _CP, _VP, _U64, _VP,
                                   ctypes.POINTER(glfsx_root),
                                   ctypes.POINTER(ctypes.c_uint64), _VP]),
    "glfsx_create_devices": (_INT, [_U64, _CP, _CP, _INT, _VP, _VP, _VP, _VP, _VP,
                                    ctypes.POINTER(glfsx_root),
                                    ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_create_devices_ms": (_INT, [ctypes.POINTER(ctypes.c_float), _INT]),
    "glfsx_shard_device": (_INT, [_U64, _CP, _CP, _VP, _U64, _U64, _U64, _VP,
                                  _VP, _VP]),
    "glfsx_root_from_level1": (_INT, [_U64, _CP, _CP, _CP, _U64, _U64,
                                      ctypes.POINTER(glfsx_root)]),
    "glfsx_post_blobs": (_INT, [_U64, _U64, _CP, _CP, _VP, _VP, _VP, _U64, POST_FN, _VP,
                                _VP]),
    "glfsx_post_blobs_device": (_INT, [_U64, _CP, _CP, _VP, _VP, _VP, _U64, _U64, _VP,
                                       _VP, _VP]),
    "glfsx_chacha20_xor": (_INT, [_CP, _VP, _VP, _U64]),
    "glfsx_fill_splitmix_device": (_INT, [_VP, _U64, _U64, _U64, _VP]),
    "glfsx_decrypt_batch_device": (_INT, [_VP, _U64, _U64, _VP, _VP, _VP]),
    "glfsx_decrypt_batch": (_INT, [_VP, _U64, _U64, _VP, _VP]),
    "glfsx_sink_count": (_INT, [_VP, _INT, _VP, _VP, _U64]),
    "glfsx_tree_encode": (_INT, [_U64, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _U64,
                                 ctypes.POINTER(ctypes.c_uint64), _VP]),
    "glfsx_tree_encode_device": (_INT, [_U64, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                        _U64, _VP, ctypes.POINTER(ctypes.c_uint64), _VP]),
    "glfsx_fill_splitmix_blobs_device": (_INT, [_VP, _U64, _U64, _U64, _VP]),
    "glfsx_post_tree_device": (_INT, [_U64, _U64, _CP, _CP, _CP, _VP, _VP, _VP, _U64, _VP,
                                      _VP, _VP, _VP, _VP, _VP, _VP, _VP, _U64, _VP, _U64,
                                      _VP, ctypes.POINTER(glfsx_root),
                                      ctypes.POINTER(ctypes.c_uint64), _VP]),
    "glfsx_store_new": (_VP, [_U64, _INT, _U64, _INT, _CP]),
    "glfsx_store_free": (None, [_VP]),
    "glfsx_store_post": (_INT, [_VP, _INT, _VP, _VP, _U64]),
    "glfsx_store_exists": (_INT, [_VP, _CP]),
    "glfsx_store_get": (_INT, [_VP, _CP, ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_store_stats": (_U64, [_VP, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64)]),
    "glfsx_store_error": (_CP, [_VP]),
    "glfsx_depth": (_INT, [_U64, _U64]),
    "glfsx_branching_factor": (_U64, [_U64]),
}

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"glfs_amd native library not built ({LIB_PATH}); run "
        "`python -c 'import __graft_entry__ as g; g.build()'` -- there is no "
        "CPU fallback for the glfsx path")

# PyTorch-ROCm bundles its own libamdhip64.so.7 / libhsa-runtime64.so.  If
# libglfsx.so were loaded first, /opt/rocm's runtime would be mapped and torch
# would then bring up a second HIP runtime that sees no GPU.  Importing torch
# first makes the dynamic linker satisfy our NEEDED libamdhip64.so.7 with the
# already-loaded runtime, so torch tensors and glfsx share one HIP runtime.
try:
    import torch  # noqa: F401
except ImportError:  # a plain C consumer (e.g. a cgo binding) needs no torch
    pass

lib = ctypes.CDLL(LIB_PATH)
for _name, (_res, _args) in SIGNATURES.items():
    if os.environ.get("GLFSX_LIB") and not hasattr(lib, _name):
        continue  # an older build under A/B comparison
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def last_error() -> str:
    return (lib.glfsx_last_error() or b"").decode(errors="replace")


def check(rc: int, msg: str | None = None) -> None:
    if rc == GLFSX_OK:
        return
    if msg is None:
        msg = last_error()
    if rc in (GLFSX_E_BLOCKSIZE_GT_MAX, GLFSX_E_BLOCKSIZE_LT_MIN):
        raise Panic(rc, msg)
    if rc == GLFSX_E_STORE:
        raise StoreError(rc, msg)
    if rc == GLFSX_E_DEVICE:
        raise DeviceError(rc, msg)
    raise GlfsxError(rc, msg)


def device_count() -> int:
    return lib.glfsx_device_count()


def set_device(dev: int) -> None:
    check(lib.glfsx_set_device(dev))


def set_latency_wgs(wgs: int) -> int:
    """Tuning knob (include/glfsx.h): launches of at most `wgs` workgroups
    use the latency-mode kernels.  Returns the previous value."""
    return lib.glfsx_set_latency_wgs(wgs)


def set_split_target(wgs: int) -> int:
    """Tuning knob (include/glfsx.h): launches of fewer than `wgs` workgroups
    spread each block over several workgroups.  0 disables.  Returns the
    previous value."""
    return lib.glfsx_set_split_target(wgs)
