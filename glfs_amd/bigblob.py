"""Python mirror of the reference's bigblob write-path interface.

Reference: bigblob/machine.go, bigblob/blob.go, bigblob/ref.go, bigblob/index.go
(blobcache/glfs, Go).  Same names (snake_case), same argument meaning, same
error behaviour (Panic where Go panics, StoreError where Go returns the store
error).  Everything below is a thin ctypes call into libglfsx.so; the hashing
and encryption run in the gfx950 kernels.
"""
from __future__ import annotations

import ctypes
import io
import os
import stat
import time
from collections import OrderedDict
from dataclasses import dataclass
from typing import BinaryIO, Optional, Protocol, Union

from . import _native as N
from ._native import Panic, StoreError  # noqa: F401  (re-exported)

DEK_SIZE = 32          # ref.go:16
CID_SIZE = 32          # blobcache.CIDSize [ext]
REF_SIZE = CID_SIZE + DEK_SIZE  # ref.go:52
MAX_REF_SIZE = REF_SIZE         # index.go:6
KIND_DATA, KIND_INDEX = 0, 1
KIND_COPY = 2  # a blob copied by Sync (its kind is not known to the copier)


@dataclass(frozen=True)
class Ref:
    """ref.go:54-57: Ref{CID, DEK}; binary form CID || DEK (ref.go:77-82)."""
    cid: bytes
    dek: bytes

    def marshal_binary(self) -> bytes:
        return self.cid + self.dek

    @staticmethod
    def from_bytes(x: bytes) -> "Ref":
        """ref.go:59-75 RefFromBytes."""
        if len(x) < REF_SIZE:
            raise ValueError(f"too small to be ref len={len(x)}")
        return Ref(bytes(x[:CID_SIZE]), bytes(x[CID_SIZE:REF_SIZE]))

    def to_json(self) -> dict:
        return {"cid": self.cid.hex(), "dek": self.dek.hex()}


@dataclass(frozen=True)
class Root:
    """blob.go:17-21 Root{Ref, Size, BlockSize}."""
    ref: Ref
    size: int
    block_size: int

    def equals(self, other: "Root") -> bool:  # blob.go:27-29
        return (self.size == other.size and self.block_size == other.block_size
                and self.ref == other.ref)


class WO(Protocol):
    """The write-only store boundary (bcsdk.WO, [ext]): MaxSize + Post.
    post() receives the ctext and the GPU-computed ref (CID || DEK)."""

    def max_size(self) -> int: ...

    def post(self, ctext: bytes, ref: bytes, kind: int) -> None: ...


def _salt_arg(salt: Optional[bytes]) -> Optional[bytes]:
    if salt is None:
        return None
    if len(salt) != 32:
        raise ValueError("salt must be 32 bytes")
    return bytes(salt)


def derive_key(salt: bytes, data: bytes, out_len: int = 32) -> bytes:
    """ref.go:152-161 DeriveKey(out, salt, input): BLAKE3 keyed with salt,
    first out_len XOF bytes (GPU)."""
    out = ctypes.create_string_buffer(max(out_len, 1))
    data = data if isinstance(data, (bytes, memoryview)) else bytes(data)
    N.check(N.lib.glfsx_derive_key(out, out_len, _salt_arg(salt), data, len(data)))
    return out.raw[:out_len]


def depth(size: int, block_size: int) -> int:
    """blob.go:256-264."""
    return N.lib.glfsx_depth(size, block_size)


def branching_factor(block_size: int) -> int:
    """blob.go:266-268."""
    return N.lib.glfsx_branching_factor(block_size)


def _make_post_cb(store: Optional[WO]):
    """(post function, error list, post_ctx) for the C-ABI.  A NativeStore
    is passed as its C function (no Python per Post)."""
    if store is None:
        return N.POST_FN(0), None, None
    native = getattr(store, "native_post", None)
    if native is not None:
        return native[0], [], native[1]
    errors: list = []

    def cb(_ctx, kind, ref, ctext, n):
        try:
            ct = ctypes.string_at(ctext, n) if n else b""
            store.post(ct, ctypes.string_at(ref, REF_SIZE), kind)
            return 0
        except Exception as e:  # surfaced as StoreError
            errors.append(e)
            return 1

    return N.POST_FN(cb), errors, None


class Writer:
    """blob.go:71-83 Writer (NewWriter/Write/Finish)."""

    def __init__(self, machine: "Machine", store: WO, salt: Optional[bytes],
                 cid_key: Optional[bytes] = None, strict: bool = False):
        self._cb, self._errors, ctx = _make_post_cb(store)
        err = ctypes.c_int(0)
        self._w = N.lib.glfsx_writer_new(machine.block_size, store.max_size(),
                                         _salt_arg(salt), cid_key, self._cb, ctx,
                                         ctypes.byref(err))
        if not self._w:
            N.check(err.value)
        self._strict = bool(strict)
        if strict:
            # blob.go:120-133 error timing: every Write returns after the
            # Posts of the blocks it completed were delivered
            N.check(N.lib.glfsx_writer_set_strict(self._w, 1))

    def _raise(self, rc: int):
        if rc == N.GLFSX_E_STORE and self._errors:
            raise StoreError(rc, repr(self._errors[0])) from self._errors[0]
        N.check(rc, (N.lib.glfsx_writer_error(self._w) or b"").decode(errors="replace"))

    def write_device(self, d_ptr: int, n: int, stream=None) -> int:
        """Write n bytes already in HBM (device pointer), ordered after the
        work on `stream` (a hipStream_t handle or None)."""
        rc = N.lib.glfsx_writer_write_device(self._w, d_ptr, n, stream)
        if rc:
            self._raise(rc)
        return n

    def write_ctext(self, ctext, refs: bytes, block_size: int) -> int:
        """Write the plaintext of data blocks given as ciphertext (decrypted
        on the GPU with each ref's DEK; the plaintext never leaves the
        device).  ctext: block j at j*block_size, the last block short."""
        if hasattr(ctext, "ctypes"):   # a numpy array: pass its memory as is
            buf, n = ctext.ctypes.data, ctext.nbytes
        elif isinstance(ctext, bytes):
            buf, n = ctext, len(ctext)
        else:
            mv = memoryview(ctext).cast("B")
            n = len(mv)
            buf = (ctypes.c_char * n).from_buffer(mv) if not mv.readonly else bytes(mv)
        rc = N.lib.glfsx_writer_write_ctext(self._w, buf, n, block_size, bytes(refs))
        if rc:
            self._raise(rc)
        return n

    def write_ctext_blocks(self, addrs, total: int, refs: bytes, block_size: int) -> int:
        """write_ctext with ciphertext block j at address addrs[j] (memory
        the caller keeps alive for the call, e.g. a NativeStore's blobs)."""
        arr = (ctypes.c_void_p * max(len(addrs), 1))(*addrs)
        rc = N.lib.glfsx_writer_write_ctext_blocks(self._w, arr, len(addrs), total, block_size,
                                                   bytes(refs))
        if rc:
            self._raise(rc)
        return total

    def flush(self) -> None:
        """Deliver the Posts of every complete block written so far."""
        rc = N.lib.glfsx_writer_flush(self._w)
        if rc:
            self._raise(rc)

    def write(self, data) -> int:
        """blob.go:120-133 (any bytes-like object; not copied on the way)."""
        if isinstance(data, bytes):
            buf, n = data, len(data)
        else:
            mv = memoryview(data).cast("B")
            n = len(mv)
            buf = (ctypes.c_char * n).from_buffer(mv) if not mv.readonly else bytes(mv)
        rc = N.lib.glfsx_writer_write(self._w, buf, n)
        if rc:
            self._raise(rc)
        return n

    def read_from(self, r) -> int:
        """io.ReaderFrom (io.Copy in Create/Concat, blob.go:213,341, uses it).
        A regular file (an *os.File, an io.ReaderAt) is read from its current
        position to its end by several threads at once straight into the
        writer's pinned staging (glfsx_writer_read_fd), then positioned after
        what was read; any other stream goes r.readinto() straight into the
        staging (glfsx_writer_reserve / glfsx_writer_commit), no second copy.
        Strict writer (the Go binding's default, integration/go/gpu.go
        ReadFrom): the call's batches are pipelined and their Posts delivered
        before it returns, so a store error comes back from this call -- where
        the reference's io.Copy returns it -- after the same Posts."""
        if not self._strict:
            return self._read_from(r)
        N.check(N.lib.glfsx_writer_set_strict(self._w, 0))
        try:
            got = self._read_from(r)
        finally:
            N.check(N.lib.glfsx_writer_set_strict(self._w, 1))
            rc = N.lib.glfsx_writer_flush(self._w)
            if rc:
                self._raise(rc)   # a store error before the reader's own
        return got

    def _read_from(self, r) -> int:
        fd = _regular_fd(r)
        if fd is not None:
            pos = r.tell()
            got = self.read_fd(fd, pos)
            r.seek(pos + got)
            return got
        total = 0
        buf, cap = ctypes.c_void_p(), ctypes.c_uint64()
        while True:
            rc = N.lib.glfsx_writer_reserve(self._w, ctypes.byref(buf), ctypes.byref(cap))
            if rc:
                self._raise(rc)
            view = (ctypes.c_char * cap.value).from_address(buf.value)
            n = r.readinto(memoryview(view).cast("B"))
            rc = N.lib.glfsx_writer_commit(self._w, n or 0)
            if rc:
                self._raise(rc)
            if n is None:
                # a non-blocking stream with nothing ready yet: not the end
                # of the input (io.Copy goes on after a (0, nil) Read)
                time.sleep(0.0005)
                continue
            total += n
            if n == 0:
                return total

    def read_fd(self, fd: int, offset: int = 0, n: int = (1 << 64) - 1) -> int:
        """n bytes (default: to the end) of file descriptor fd from `offset`
        into the writer, pread by several threads at once
        (glfsx_writer_read_fd; the descriptor's own offset is not used).
        Returns the bytes taken."""
        got = ctypes.c_uint64()
        rc = N.lib.glfsx_writer_read_fd(self._w, fd, offset, n, ctypes.byref(got))
        if rc:
            self._raise(rc)
        return got.value

    def read_at(self, read_at, offset: int = 0, n: int = (1 << 64) - 1) -> int:
        """io.ReaderAt route (glfsx_writer_read_at): read_at(buf: memoryview,
        off: int) -> bytes read (0 at the end), called from several threads
        at once on disjoint ranges.  Returns the bytes taken."""
        def cb(_ctx, buf, ln, off):
            try:
                return int(read_at(memoryview((ctypes.c_char * ln).from_address(buf)).cast("B"),
                                   off))
            except Exception:
                return -5   # EIO
        fn = N.READ_AT_FN(cb)
        got = ctypes.c_uint64()
        rc = N.lib.glfsx_writer_read_at(self._w, fn, None, offset, n, ctypes.byref(got))
        if rc:
            self._raise(rc)
        return got.value

    def finish(self) -> Root:
        """blob.go:135-150."""
        r = N.glfsx_root()
        rc = N.lib.glfsx_writer_finish(self._w, ctypes.byref(r))
        if rc:
            self._raise(rc)
        return Root(Ref.from_bytes(bytes(r.ref)), r.size, r.block_size)

    def close(self) -> None:
        if self._w:
            N.lib.glfsx_writer_free(self._w)
            self._w = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _regular_fd(r) -> Optional[int]:
    """The descriptor of a seekable regular file behind r, or None.

    Only a plain file object qualifies: an io.FileIO, or a buffered reader
    whose raw stream is one (what open(p, "rb") returns), so that tell() is
    a byte offset into the descriptor's file.  A wrapper that transforms
    the bytes (gzip / bz2 / lzma files, whose fileno() is the compressed
    file's and whose tell() is a decompressed position) reads through
    readinto instead."""
    raw = r
    if isinstance(r, (io.BufferedReader, io.BufferedRandom)):
        raw = r.raw
    if type(raw) is not io.FileIO:
        return None
    try:
        if not r.seekable():
            return None
        fd = r.fileno()
        return fd if stat.S_ISREG(os.fstat(fd).st_mode) else None
    except (OSError, ValueError, io.UnsupportedOperation):
        return None


def _copy(w, r: Union[bytes, bytearray, memoryview, BinaryIO]) -> None:
    """io.Copy: a bytes-like source is one Write (bytes.Reader is a WriterTo);
    a stream with readinto goes through the Writer's ReadFrom (read straight
    into the staging), any other stream in 32 KiB pieces."""
    if isinstance(r, (bytes, bytearray, memoryview)):
        w.write(r)
        return
    if hasattr(r, "readinto"):
        w.read_from(r)
        return
    while True:
        piece = r.read(32 * 1024)
        if not piece:
            return
        w.write(piece)


class Machine:
    """bigblob/machine.go:32-55.  block_size 0 = the store's MaxSize."""

    def __init__(self, block_size: int = 0, cache_size: int = 64):
        if block_size < 0:  # machine.go:24 WithBlockSize panics
            raise Panic(N.GLFSX_E_ARG, str(block_size))
        self.block_size = block_size
        self.cache_size = cache_size
        # machine.go:36 getF LRU, keyed by Ref.Key() (= BLAKE3(CID||DEK) in
        # the reference; the 64-B ref itself identifies the same entry)
        self._cache: "OrderedDict[bytes, bytes]" = OrderedDict()

    # ------------------------------------------------------------ read side
    def get_f(self, store, ref: Ref) -> bytes:
        """ref.go:113-126 getF: fetch the ctext by CID, decrypt with the DEK
        (ChaCha20 on the GPU), cache the plaintext."""
        key = ref.marshal_binary()
        hit = self._cache.get(key)
        if hit is not None:
            self._cache.move_to_end(key)
            return hit
        data = crypto_xor(ref.dek, store.get(ref.cid))
        if self.cache_size > 0:
            self._cache[key] = data
            if len(self._cache) > self.cache_size:
                self._cache.popitem(last=False)
        return data

    def get_piece(self, store, root: Ref, bf: int, level: int, block_index: int) -> Ref:
        """blob.go:53-69 getPiece: walk index nodes down to the block's ref.
        Index nodes must be exactly bf*64 bytes (newIndexUsing)."""
        while level > 0:
            data = self.get_f(store, root)
            if len(data) != bf * MAX_REF_SIZE:
                raise ValueError("data is not correct size for index")
            span = bf ** (level - 1)
            i = block_index // span
            root = Ref.from_bytes(data[i * MAX_REF_SIZE:(i + 1) * MAX_REF_SIZE])
            block_index %= span
            level -= 1
        return root

    def read_at(self, store, x: Root, offset: int, n: int) -> tuple:
        """blob.go:31-51 ReadAt: at most ONE block per call (quirk kept).
        Returns (data, eof) where eof mirrors the io.EOF the reference
        returns when the read ends exactly at Size."""
        level = depth(x.size, x.block_size)
        bf = branching_factor(x.block_size)
        block_index, rel = divmod(offset, x.block_size)
        ref = self.get_piece(store, x.ref, bf, level, block_index)
        data = self.get_f(store, ref)
        if rel > len(data):  # Go slices data[relOffset:] and panics
            raise Panic(N.GLFSX_E_ARG, "slice bounds out of range")
        out = data[rel:rel + n]
        return out, offset + len(out) == x.size

    def new_reader(self, store, root: Root) -> "Reader":
        """io.go:23-30."""
        return Reader(self, store, root)

    def traverse(self, store, root: Root, enter, exit) -> None:
        """traverse.go:18-52: pre-order Enter(cid) -> bool (False skips the
        subtree), post-order Exit(level, ref).  Children stop at the first
        all-zero CID."""
        if root.block_size == 0:
            raise ValueError("block size cannot be zero")
        self._traverse(store, root.block_size, depth(root.size, root.block_size),
                       root.ref, enter, exit)

    def _traverse(self, store, bs, level, x: Ref, enter, exit) -> None:
        if not enter(x.cid):
            return
        if level > 0:
            data = self.get_f(store, x)
            if len(data) != bs:
                raise ValueError("data is not correct size for index")
            for i in range(bs // MAX_REF_SIZE):
                r2 = Ref.from_bytes(data[i * MAX_REF_SIZE:(i + 1) * MAX_REF_SIZE])
                if r2.cid == bytes(CID_SIZE):
                    break
                self._traverse(store, bs, level - 1, r2, enter, exit)
        exit(level, x)

    def sync(self, dst, src, x: Root, fn=None) -> None:
        """blob.go:270-315 Sync: nothing to do if dst has the root CID;
        otherwise call fn(reader), then copy every reachable blob, children
        before their index node (the reference's post-order).  The index
        levels are read one batched GPU decrypt per level."""
        if exists_unit(dst, x.ref.cid):
            return
        if fn is not None:
            fn(self.new_reader(src, x))
        levels = _tree_levels(src.get, x)
        bf = branching_factor(x.block_size)

        def emit(k: int, j: int) -> None:
            if k + 1 < len(levels):
                for c in range(j * bf, min((j + 1) * bf, len(levels[k + 1]))):
                    emit(k + 1, c)
            copy_blob(dst, src, levels[k][j])

        if x.size == 0:
            copy_blob(dst, src, x.ref)
        else:
            emit(0, 0)

    def populate(self, store, root: Root, dst) -> None:
        """blob.go:317-331 Populate: add every reachable CID that dst lacks
        (Enter skips subtrees dst already has; Exit adds)."""
        self.traverse(store, root, lambda cid: not exists_unit(dst, cid),
                      lambda level, ref: dst.add(ref.cid))

    def post(self, store: WO, salt: Optional[bytes], data: bytes,
             cid_key: Optional[bytes] = None) -> Ref:
        """ref.go:98-111 post: DEK = DeriveKey(salt, ptext), ctext =
        ChaCha20(DEK) ^ ptext, CID = the store's hash of ctext -- all on the
        GPU -- then store.Post(ctext).  A store error propagates."""
        data = bytes(data)
        ref = ctypes.create_string_buffer(REF_SIZE)
        ct = ctypes.create_string_buffer(max(len(data), 1))
        N.check(N.lib.glfsx_post(_salt_arg(salt) or bytes(32), data, len(data), ct, ref,
                                 cid_key))
        store.post(ct.raw[:len(data)], ref.raw, KIND_DATA)
        return Ref.from_bytes(ref.raw)

    def new_writer(self, store: WO, salt: Optional[bytes] = None,
                   cid_key: Optional[bytes] = None, strict: bool = False) -> Writer:
        """blob.go:85-114 (strict: the reference's per-Write error timing)."""
        return Writer(self, store, salt, cid_key, strict)

    def concat(self, store, block_size: int, salt: Optional[bytes], *roots: Root) -> Root:
        """blob.go:333-345."""
        return _concat(self, store, block_size, salt, roots)

    def create(self, store: WO, salt: Optional[bytes], r,
               cid_key: Optional[bytes] = None) -> Root:
        """blob.go:209-217."""
        w = self.new_writer(store, salt, cid_key)
        try:
            _copy(w, r)
            return w.finish()
        finally:
            w.close()


def _gather(store, refs, size: int):
    """The blobs of `refs`, concatenated into one uninitialised buffer of
    `size` bytes (straight from a NativeStore's memory when possible)."""
    import numpy as np
    out = np.empty(size, dtype=np.uint8)
    base, off = out.ctypes.data, 0
    direct = hasattr(store, "get_into")
    for ref in refs:
        if direct:
            off += store.get_into(ref.cid, base + off, size - off)
        else:
            c = store.get(ref.cid)
            if off + len(c) > size:
                raise ValueError("blob larger than its root says")
            out[off:off + len(c)] = np.frombuffer(c, dtype=np.uint8)
            off += len(c)
    if off != size:
        raise ValueError(f"blob read {off} bytes, root says {size}")
    return out


def _concat(machine: "Machine", store, block_size: int, salt, roots, cid_key=None) -> Root:
    """blob.go:333-345 Concat: every root's bytes, in order, through a new
    Writer.  The index levels are read with one batched decrypt per level;
    the data blocks go to the Writer as ciphertext and are decrypted on the
    GPU right into its staging (glfsx_writer_write_ctext), so the plaintext
    never crosses PCIe.  Like the reference, the `block_size` argument is
    ignored: the writer uses the machine's block size (quirk recorded in
    SURVEY's appendix)."""
    w = machine.new_writer(store, salt, cid_key)
    try:
        for r in roots:
            if r.size == 0:
                continue
            data_refs = _tree_levels(store.get, r)[-1]
            if r.block_size % 64:
                w.write(read_all(store, r))
                continue
            refs = b"".join(x.marshal_binary() for x in data_refs)
            if hasattr(store, "addr"):   # blocks straight from the store's memory
                addrs, got = [], 0
                for i, x in enumerate(data_refs):
                    a, n = store.addr(x.cid)
                    want = r.block_size if i + 1 < len(data_refs) else \
                        r.size - r.block_size * (len(data_refs) - 1)
                    if n != want:
                        raise ValueError(f"block {i} has {n} bytes, the root says {want}")
                    addrs.append(a)
                    got += n
                w.write_ctext_blocks(addrs, got, refs, r.block_size)
                continue
            ct = _gather(store, data_refs, r.size)
            w.write_ctext(ct, refs, r.block_size)
        return w.finish()
    finally:
        w.close()


class Reader:
    """io.go:15-54 Reader: Read / ReadAt / Seek over a Root (each call reads
    from at most one block, as the reference's ReadAt does)."""
    SEEK_SET, SEEK_CUR, SEEK_END = 0, 1, 2

    def __init__(self, machine: Machine, store, root: Root):
        self.o, self.store, self.root, self.offset = machine, store, root, 0

    def read_at(self, n: int, at: int) -> tuple:
        return self.o.read_at(self.store, self.root, at, n)

    def read(self, n: int = -1) -> bytes:
        """Python io semantics on top of ReadAt: returns b"" at EOF; n < 0
        reads to the end (block by block)."""
        if self.offset >= self.root.size:
            return b""
        if n < 0:
            parts = []
            while self.offset < self.root.size:
                parts.append(self.read(self.root.size - self.offset))
            return b"".join(parts)
        data, _ = self.o.read_at(self.store, self.root, self.offset, n)
        self.offset += len(data)
        return data

    def seek(self, offset: int, whence: int = 0) -> int:
        if whence == self.SEEK_SET:
            self.offset = offset
        elif whence == self.SEEK_CUR:
            self.offset += offset
        elif whence == self.SEEK_END:
            self.offset = self.root.size + offset
        else:
            raise Panic(N.GLFSX_E_ARG, "invalid whence")
        return self.offset


def exists_unit(store, cid: bytes) -> bool:
    """machine.go:86-92 ExistsUnit."""
    return bool(store.exists(cid))


def copy_blob(dst, src, ref: Ref) -> None:
    """blob.go:306-315 copyBlob: Get the ctext from src, Post it to dst.
    The destination is a pre-hashed store (its Post takes the CID with the
    bytes), so the copy keeps the CID the source holds."""
    ct = src.get(ref.cid)
    dst.post(ct, ref.cid + bytes(DEK_SIZE), KIND_COPY)


class CIDSet:
    """A minimal AddExister (machine.go:81-84): Exists + Add over CIDs."""

    def __init__(self):
        self.cids: set = set()

    def exists(self, cid: bytes) -> bool:
        return cid in self.cids

    def add(self, cid: bytes) -> None:
        self.cids.add(cid)


class ErrNotFound(KeyError):
    """blobcache.ErrNotFound{CID} [ext]: Get of a CID the store lacks."""

    def __init__(self, cid: bytes):
        super().__init__(f"blob not found: {cid.hex()}")
        self.cid = cid


class NativeStore:
    """The native store of the C-ABI (glfsx_store_*, include/glfsx.h): an
    in-memory content-addressed store whose Post takes the GPU-computed CID
    (mode "trust": a pre-hashed Post; verify_every=k re-hashes every k-th
    Post on the host) or re-hashes every ctext on the host as blobcache's
    MemStore.Post does behind ref.go:103 (mode "hash").  The Writer hands it
    its Posts as a C function pointer: no Python per Post."""

    def __init__(self, max_size: int, mode: str = "trust", verify_every: int = 0,
                 keep_data: bool = True, cid_key: Optional[bytes] = None):
        m = {"trust": N.GLFSX_STORE_TRUST, "hash": N.GLFSX_STORE_HASH}[mode]
        self._max = max_size
        self._s = N.lib.glfsx_store_new(max_size, m, verify_every, int(keep_data), cid_key)
        if not self._s:
            raise N.GlfsxError(N.GLFSX_E_UNSUPPORTED,
                               "host BLAKE3 (libclang-cpp.so) unavailable for a hashing store")
        self.native_post = (ctypes.cast(N.lib.glfsx_store_post, N.POST_FN),
                            ctypes.c_void_p(self._s))

    def max_size(self) -> int:
        return self._max

    def post(self, ctext: bytes, ref: bytes, kind: int = KIND_DATA) -> None:
        rc = N.lib.glfsx_store_post(self._s, kind, ref, ctext, len(ctext))
        if rc:
            raise StoreError(rc, (N.lib.glfsx_store_error(self._s) or b"").decode())

    def exists(self, cid: bytes) -> bool:
        return bool(N.lib.glfsx_store_exists(self._s, bytes(cid)))

    def get(self, cid: bytes) -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        if N.lib.glfsx_store_get(self._s, bytes(cid), ctypes.byref(p), ctypes.byref(n)):
            raise ErrNotFound(bytes(cid))
        return ctypes.string_at(p, n.value) if n.value else b""

    def addr(self, cid: bytes):
        """(address, length) of the blob in the store's own memory, valid
        until the store is freed (glfsx_store_get)."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        if N.lib.glfsx_store_get(self._s, bytes(cid), ctypes.byref(p), ctypes.byref(n)):
            raise ErrNotFound(bytes(cid))
        return p.value or 0, n.value

    def get_into(self, cid: bytes, dst_addr: int, cap: int) -> int:
        """Copy the blob straight from the store's memory to dst_addr (at
        most cap bytes); returns its length."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        if N.lib.glfsx_store_get(self._s, bytes(cid), ctypes.byref(p), ctypes.byref(n)):
            raise ErrNotFound(bytes(cid))
        if n.value > cap:
            raise ValueError("blob larger than the destination")
        if n.value:
            ctypes.memmove(dst_addr, p, n.value)
        return n.value

    def stats(self) -> dict:
        posts, nbytes, hashed = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        blobs = N.lib.glfsx_store_stats(self._s, ctypes.byref(posts), ctypes.byref(nbytes),
                                        ctypes.byref(hashed))
        return {"blobs": blobs, "posts": posts.value, "bytes": nbytes.value,
                "rehashed": hashed.value}

    def __len__(self) -> int:
        return self.stats()["blobs"]

    def close(self) -> None:
        if self._s:
            N.lib.glfsx_store_free(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MemStore:
    """In-memory stand-in for blobcache's schema.MemStore [ext].  It keeps
    (CID -> ctext) as posted by the GPU path (a pre-hashed Post: the CID was
    computed on the device).  Tests re-verify every CID with the oracle."""

    def __init__(self, max_size: int):
        self._max = max_size
        self.blobs: dict[bytes, bytes] = {}
        self.log: list[tuple[int, bytes, int]] = []  # (kind, ref, len)

    def max_size(self) -> int:
        return self._max

    def post(self, ctext: bytes, ref: bytes, kind: int = KIND_DATA) -> None:
        if len(ctext) > self._max:
            raise ValueError(f"blob too large {len(ctext)} > {self._max}")
        self.blobs[ref[:CID_SIZE]] = ctext
        self.log.append((kind, ref, len(ctext)))

    def __len__(self) -> int:
        return len(self.blobs)

    def exists(self, cid: bytes) -> bool:
        return cid in self.blobs

    def get(self, cid: bytes) -> bytes:
        try:
            return self.blobs[cid]
        except KeyError:
            raise ErrNotFound(cid) from None

    def delete(self, cids) -> None:
        for cid in cids:
            self.blobs.pop(cid, None)


def crypto_xor(dek: bytes, data: bytes) -> bytes:
    """ref.go:137-144 cryptoXOR (ChaCha20, zero nonce, counter 0) on the GPU;
    self-inverse, so it is also getF's decrypt (ref.go:122)."""
    data = bytes(data)
    out = ctypes.create_string_buffer(max(len(data), 1))
    N.check(N.lib.glfsx_chacha20_xor(bytes(dek), data, out, len(data)))
    return out.raw[:len(data)]


def decrypt_level(ctexts, refs, block_size: int) -> list:
    """getF (ref.go:113-126) for the blobs of one tree level at once: every
    ctext but the last is exactly block_size bytes (index nodes; a blob's
    data blocks), decrypted with its ref's DEK in ONE batched GPU call
    (glfsx_decrypt_batch).  Returns the plaintexts in order."""
    n = len(ctexts)
    if n == 0:
        return []
    if any(len(c) != block_size for c in ctexts[:-1]) or len(ctexts[-1]) > block_size \
            or block_size % 64:
        return [crypto_xor(r.dek, c) for r, c in zip(refs, ctexts)]
    data = b"".join(ctexts)
    rb = b"".join(r.marshal_binary() for r in refs)
    out = ctypes.create_string_buffer(max(len(data), 1))
    N.check(N.lib.glfsx_decrypt_batch(data, len(data), block_size, rb, out))
    raw = out.raw
    return [raw[i * block_size:i * block_size + len(c)] for i, c in enumerate(ctexts)]


def _tree_levels(get, root: Root) -> list:
    """The refs of every level of root's tree, top (the root) first, data
    blocks last: each index level is fetched with get(cid) and decrypted in
    one batch (blob.go:53-69 getPiece's walk, level by level)."""
    bs = root.block_size
    bf = branching_factor(bs)
    lvl = depth(root.size, bs)
    n0 = -(-root.size // bs)
    levels = [[root.ref]]
    for k in range(lvl, 0, -1):
        refs = levels[-1]
        nodes = decrypt_level([get(r.cid) for r in refs], refs, bs)
        want = -(-n0 // bf ** (k - 1))          # refs at level k-1
        child = []
        for node in nodes:
            if len(node) != bf * MAX_REF_SIZE:
                raise ValueError("data is not correct size for index")
            take = min(bf, want - len(child))
            child += [Ref.from_bytes(node[i * 64:(i + 1) * 64]) for i in range(take)]
        levels.append(child)
    return levels


def read_all(store, root: Root) -> bytes:
    """Read side (blob.go:31-69 ReadAt/getPiece, ref.go:113-126 getF) of a
    whole blob: the index levels and then all data blocks, each level one
    batched GPU decrypt (the data level straight into the output buffer)."""
    if root.size == 0:
        return b""
    bs = root.block_size
    data_refs = _tree_levels(store.get, root)[-1]
    if bs % 64:
        return b"".join(crypto_xor(r.dek, store.get(r.cid)) for r in data_refs)
    ct = _gather(store, data_refs, root.size)
    out = bytearray(root.size)
    rb = b"".join(r.marshal_binary() for r in data_refs)
    obuf = (ctypes.c_char * len(out)).from_buffer(out)
    N.check(N.lib.glfsx_decrypt_batch(ct.ctypes.data, len(ct), bs, rb, obuf))
    del obuf
    return bytes(out)
