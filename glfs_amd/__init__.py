"""glfs_amd -- MI355X-native GLFS bigblob write path.

The product is libglfsx.so (C-ABI: include/glfsx.h) built from glfs_amd/csrc:
gfx950 HIP kernels for the per-block DEK (keyed BLAKE3), ChaCha20 encryption
and CID (BLAKE3-256 of the ciphertext), plus the C++ host runtime that mirrors
bigblob's Writer.  This package is a thin ctypes mirror of the reference's
bigblob/glfs write API for tests and benchmarks.
"""
from . import _native  # noqa: F401  (raises ImportError if not built)
from . import bigblob, glfs  # noqa: F401

__all__ = ["bigblob", "glfs"]
