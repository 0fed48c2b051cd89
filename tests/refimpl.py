"""Independent primitive implementations present in this image, used to pin the
oracle (test infrastructure only).

  * BLAKE3: upstream C BLAKE3 1.8.2 compiled into LLVM, exported from
    /opt/rocm/lib/llvm/lib/libclang-cpp.so as llvm_blake3_* (no header
    shipped; the hasher struct is < 2 KiB, we allocate 4 KiB).
  * ChaCha20: OpenSSL libcrypto EVP_chacha20 (16-byte IV = LE32 counter ||
    12-byte nonce), and libsodium crypto_stream_chacha20_ietf_xor_ic.

Both are loaded from the image's own libraries, never from /root/reference.
Callers skip when a library is absent.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os

_LLVM = "/opt/rocm/lib/llvm/lib/libclang-cpp.so"
_b3 = None
_ssl = None
_sodium = None


def blake3_lib():
    global _b3
    if _b3 is None:
        if not os.path.exists(_LLVM):
            return None
        L = ctypes.CDLL(_LLVM)
        L.llvm_blake3_hasher_init.argtypes = [ctypes.c_void_p]
        L.llvm_blake3_hasher_init_keyed.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.llvm_blake3_hasher_update.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                                ctypes.c_size_t]
        L.llvm_blake3_hasher_finalize.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                                  ctypes.c_size_t]
        L.llvm_blake3_version.restype = ctypes.c_char_p
        _b3 = L
    return _b3


def blake3(data: bytes, key: bytes | None = None, out_len: int = 32) -> bytes:
    L = blake3_lib()
    h = ctypes.create_string_buffer(4096)
    if key is None:
        L.llvm_blake3_hasher_init(h)
    else:
        L.llvm_blake3_hasher_init_keyed(h, key)
    L.llvm_blake3_hasher_update(h, data, len(data))
    out = ctypes.create_string_buffer(out_len)
    L.llvm_blake3_hasher_finalize(h, out, out_len)
    return out.raw


def openssl_lib():
    global _ssl
    if _ssl is None:
        name = ctypes.util.find_library("crypto")
        if not name:
            return None
        L = ctypes.CDLL(name)
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_chacha20.restype = ctypes.c_void_p
        L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                        ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                        ctypes.c_int]
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        _ssl = L
    return _ssl


def chacha20_xor(data: bytes, key: bytes, nonce: bytes = bytes(12), counter: int = 0) -> bytes:
    L = openssl_lib()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        iv = counter.to_bytes(4, "little") + nonce
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_chacha20(), None, key, iv) == 1
        out = ctypes.create_string_buffer(len(data) + 64)
        outl = ctypes.c_int(0)
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), data, len(data)) == 1
        return out.raw[:outl.value]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def sodium_lib():
    global _sodium
    if _sodium is None:
        for p in ("/opt/conda/lib/libsodium.so", ctypes.util.find_library("sodium")):
            if p and os.path.exists(p):
                L = ctypes.CDLL(p)
                L.crypto_stream_chacha20_ietf_xor_ic.argtypes = [
                    ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulonglong, ctypes.c_char_p,
                    ctypes.c_uint32, ctypes.c_char_p]
                _sodium = L
                break
    return _sodium


def sodium_chacha20_xor(data: bytes, key: bytes, nonce: bytes = bytes(12),
                        counter: int = 0) -> bytes:
    L = sodium_lib()
    out = ctypes.create_string_buffer(max(len(data), 1))
    assert L.crypto_stream_chacha20_ietf_xor_ic(out, data, len(data), nonce, counter, key) == 0
    return out.raw[:len(data)]
