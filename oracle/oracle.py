"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package glfs_amd/.
See oracle.h for what is restated (reference file:line) and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_uint8),
                           ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64)

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_u8p = ctypes.c_char_p
        L.oracle_blake3.argtypes = [c_u8p, ctypes.c_size_t, c_u8p, c_u8p, ctypes.c_size_t]
        L.oracle_chacha20_xor.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, c_u8p, c_u8p,
                                          ctypes.c_uint32]
        L.oracle_derive_key.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_size_t]
        L.oracle_post.argtypes = [c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_size_t, c_u8p]
        L.oracle_writer_new.restype = ctypes.c_void_p
        L.oracle_writer_new.argtypes = [ctypes.c_uint64, ctypes.c_uint64, c_u8p, c_u8p,
                                        SINK_FN, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_int)]
        L.oracle_writer_write.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_size_t]
        L.oracle_writer_finish.argtypes = [ctypes.c_void_p, c_u8p,
                                           ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_writer_free.argtypes = [ctypes.c_void_p]
        L.oracle_create_closed.restype = ctypes.c_int64
        L.oracle_create_closed.argtypes = [ctypes.c_uint64, c_u8p, c_u8p, c_u8p,
                                           ctypes.c_uint64, c_u8p, SINK_FN, ctypes.c_void_p]
        L.oracle_depth.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_post_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, c_u8p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                        c_u8p, ctypes.c_int]
        L.oracle_post_batch_simd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, c_u8p,
                                             ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_uint64, c_u8p, ctypes.c_int]
        L.oracle_post_batch_gomix.argtypes = L.oracle_post_batch_simd.argtypes
        L.oracle_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_fill_splitmix_blobs.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_uint64]
        _lib = L
    return _lib


def blake3(data: bytes, key: bytes | None = None, out_len: int = 32) -> bytes:
    out = ctypes.create_string_buffer(out_len)
    lib().oracle_blake3(out, out_len, key, data, len(data))
    return out.raw


def chacha20_xor(data: bytes, key: bytes, nonce: bytes = bytes(12), counter: int = 0) -> bytes:
    out = ctypes.create_string_buffer(max(len(data), 1))
    lib().oracle_chacha20_xor(out, data, len(data), key, nonce, counter)
    return out.raw[:len(data)]


def derive_key(salt: bytes, data: bytes) -> bytes:
    """ref.go:152 DeriveKey(out[:32], salt, input)."""
    out = ctypes.create_string_buffer(32)
    lib().oracle_derive_key(out, salt, data, len(data))
    return out.raw


def post(salt: bytes, ptext: bytes, cid_key: bytes | None = None) -> tuple[bytes, bytes]:
    """ref.go:98 post(): returns (ref64 = CID||DEK, ctext)."""
    ref = ctypes.create_string_buffer(64)
    ct = ctypes.create_string_buffer(max(len(ptext), 1))
    lib().oracle_post(ref, ct, salt, ptext, len(ptext), cid_key)
    return ref.raw, ct.raw[:len(ptext)]


class WriterPanic(Exception):
    """Raised where the reference panics (blob.go:91, blob.go:94)."""


def create(data: bytes, block_size: int, salt: bytes | None = None,
           store_max: int | None = None, cid_key: bytes | None = None,
           chunks: list[int] | None = None, closed_form: bool = False):
    """Streaming writer (blob.go:85-206) over `data`, written in pieces of the
    sizes in `chunks` (io.Copy granularity).  Returns (root_ref, size, bs, posts)
    where posts = [(kind, ref, len, ctext)] in Post order."""
    posts = []

    def sink(_ctx, kind, ref, ct, n):
        posts.append((kind, ctypes.string_at(ref, 64), n,
                      ctypes.string_at(ct, n) if n else b""))
        return 0

    cb = SINK_FN(sink)
    root = ctypes.create_string_buffer(64)
    if closed_form:
        lib().oracle_create_closed(block_size, salt, cid_key, data, len(data), root, cb, None)
        return root.raw, len(data), block_size, posts
    err = ctypes.c_int(0)
    smax = store_max if store_max is not None else block_size
    w = lib().oracle_writer_new(block_size, smax, salt, cid_key, cb, None, ctypes.byref(err))
    if not w:
        raise WriterPanic({-1: f"blockSize {block_size} > maxSize {smax}",
                           -2: "blockSize cannot be < 128"}[err.value])
    try:
        if chunks is None:
            chunks = [len(data)]
        off = 0
        for c in chunks:
            piece = data[off:off + c]
            if lib().oracle_writer_write(w, piece, len(piece)) != 0:
                raise RuntimeError("sink error")
            off += c
        if off < len(data):
            rest = data[off:]
            lib().oracle_writer_write(w, rest, len(rest))
        size = ctypes.c_uint64()
        bs = ctypes.c_uint64()
        if lib().oracle_writer_finish(w, root, ctypes.byref(size), ctypes.byref(bs)) != 0:
            raise RuntimeError("finish failed")
        return root.raw, size.value, bs.value, posts
    finally:
        lib().oracle_writer_free(w)


def depth(size: int, block_size: int) -> int:
    return lib().oracle_depth(size, block_size)


def fill_splitmix(n: int, seed: int, offset: int = 0) -> bytes:
    buf = ctypes.create_string_buffer(max(n, 1))
    lib().oracle_fill_splitmix(buf, offset, n, seed)
    return buf.raw[:n]


def mod251(n: int) -> bytes:
    return bytes(i % 251 for i in range(n))
