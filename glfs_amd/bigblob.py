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
    out = ctypes.create_string_buffer(32)
    data = bytes(data)
    N.check(N.lib.glfsx_derive_key(out, out_len, _salt_arg(salt), data, len(data)))
    return out.raw[:out_len]


def depth(size: int, block_size: int) -> int:
    """blob.go:256-264."""
    return N.lib.glfsx_depth(size, block_size)


def branching_factor(block_size: int) -> int:
    """blob.go:266-268."""
    return N.lib.glfsx_branching_factor(block_size)


def _make_post_cb(store: Optional[WO]):
    if store is None:
        return N.POST_FN(0), None
    errors: list = []

    def cb(_ctx, kind, ref, ctext, n):
        try:
            ct = ctypes.string_at(ctext, n) if n else b""
            store.post(ct, ctypes.string_at(ref, REF_SIZE), kind)
            return 0
        except Exception as e:  # surfaced as StoreError
            errors.append(e)
            return 1

    return N.POST_FN(cb), errors


class Writer:
    """blob.go:71-83 Writer (NewWriter/Write/Finish)."""

    def __init__(self, machine: "Machine", store: WO, salt: Optional[bytes],
                 cid_key: Optional[bytes] = None, strict: bool = False):
        self._cb, self._errors = _make_post_cb(store)
        err = ctypes.c_int(0)
        self._w = N.lib.glfsx_writer_new(machine.block_size, store.max_size(),
                                         _salt_arg(salt), cid_key, self._cb, None,
                                         ctypes.byref(err))
        if not self._w:
            N.check(err.value)
        if strict:
            # blob.go:120-133 error timing: every Write returns after the
            # Posts of the blocks it completed were delivered
            N.check(N.lib.glfsx_writer_set_strict(self._w, 1))

    def _raise(self, rc: int):
        if rc == N.GLFSX_E_STORE and self._errors:
            raise StoreError(rc, repr(self._errors[0])) from self._errors[0]
        N.check(rc, (N.lib.glfsx_writer_error(self._w) or b"").decode(errors="replace"))

    def flush(self) -> None:
        """Deliver the Posts of every complete block written so far."""
        rc = N.lib.glfsx_writer_flush(self._w)
        if rc:
            self._raise(rc)

    def write(self, data: bytes) -> int:
        """blob.go:120-133."""
        data = bytes(data)
        rc = N.lib.glfsx_writer_write(self._w, data, len(data))
        if rc:
            self._raise(rc)
        return len(data)

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


def _copy(w, r: Union[bytes, bytearray, memoryview, BinaryIO]) -> None:
    """io.Copy: a bytes-like source is one Write (bytes.Reader is a WriterTo);
    a stream is copied in 32 KiB pieces."""
    if isinstance(r, (bytes, bytearray, memoryview)):
        w.write(r)
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
        otherwise call fn(reader), then copy every reachable blob (children
        before their index node)."""
        if exists_unit(dst, x.ref.cid):
            return
        if fn is not None:
            fn(self.new_reader(src, x))
        self._sync(dst, src, x.block_size, x.ref, depth(x.size, x.block_size))

    def _sync(self, dst, src, bs, ref: Ref, level: int) -> None:
        if level > 0:
            data = self.get_f(src, ref)
            if len(data) != bs:
                raise ValueError("data is not correct size for index")
            for i in range(bs // MAX_REF_SIZE):
                r2 = Ref.from_bytes(data[i * MAX_REF_SIZE:(i + 1) * MAX_REF_SIZE])
                if r2.cid == bytes(CID_SIZE):
                    break
                self._sync(dst, src, bs, r2, level - 1)
        copy_blob(dst, src, ref)

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


def _concat(machine: "Machine", store, block_size: int, salt, roots, cid_key=None) -> Root:
    """blob.go:333-345 Concat: read every root (GPU decrypt of each blob via
    the read side), stream the bytes through a new Writer.  Like the
    reference, the `block_size` argument is ignored: the writer uses the
    machine's block size (quirk recorded in SURVEY's appendix)."""
    w = machine.new_writer(store, salt, cid_key)
    try:
        for r in roots:
            w.write(read_all(store, r))
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


def read_all(store: MemStore, root: Root) -> bytes:
    """Read side (blob.go:31-69 ReadAt/getPiece, ref.go:113-126 getF) for
    round-trip verification: walk the index tree, decrypt each blob."""
    bs = root.block_size
    bf = branching_factor(bs)
    lvl = depth(root.size, bs)

    def get_f(ref: Ref) -> bytes:
        return crypto_xor(ref.dek, store.get(ref.cid))

    out = io.BytesIO()

    def walk(ref: Ref, level: int, remaining: int) -> int:
        data = get_f(ref)
        if level == 0:
            out.write(data)
            return len(data)
        if len(data) != bf * MAX_REF_SIZE:
            raise ValueError("data is not correct size for index")
        got = 0
        for i in range(bf):
            if got >= remaining:
                break
            child = Ref.from_bytes(data[i * 64:(i + 1) * 64])
            got += walk(child, level - 1, remaining - got)
        return got

    if root.size:
        walk(root.ref, lvl, root.size)
    return out.getvalue()
