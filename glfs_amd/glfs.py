"""Python mirror of the reference's glfs typed-object write API.

Reference: glfs.go:12-97, machine.go:12-66, blob.go:15-39 (blobcache/glfs).
Quirk kept for parity: NewMachine ignores its options, so the machine salt is
always 0^32 (machine.go:41-48) and WithSalt has no effect.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from . import bigblob
from .bigblob import Root

DEFAULT_BLOCK_SIZE = 1 << 21  # glfs.go:12
TYPE_BLOB = "blob"            # glfs.go:18
TYPE_TREE = "tree"            # glfs.go:19


@dataclass(frozen=True)
class Ref:
    """glfs.go:35-38 Ref{Type, bigblob.Root} (Root embedded/flattened)."""
    type: str
    root: Root

    def equals(self, other: "Ref") -> bool:
        return self.type == other.type and self.root.equals(other.root)

    def to_json(self) -> dict:
        d = {"type": self.type}
        d.update(self.root.ref.to_json())
        d["size"] = self.root.size
        d["blockSize"] = self.root.block_size
        return d


class ErrRefType(TypeError):
    """errors.go:20-26."""

    def __init__(self, have: str, want: str):
        super().__init__(f"wrong type HAVE: {have} WANT: {want}")
        self.have, self.want = have, want


def with_salt(salt: bytes):
    """machine.go:15-19 WithSalt -- dead: NewMachine never applies options."""
    def opt(m: "Machine") -> None:
        m.salt = salt
    return opt


class TypedWriter:
    """glfs.go:68-92."""

    def __init__(self, ty: str, bw: bigblob.Writer):
        self.ty = ty
        self.bw = bw

    def write(self, data: bytes) -> int:
        return self.bw.write(data)

    def finish(self) -> Ref:
        root = self.bw.finish()
        self.bw.close()
        return Ref(self.ty, root)


class Machine:
    """machine.go:27-48."""

    def __init__(self, *opts):
        self.salt = bytes(32)  # opts are ignored (machine.go:41-48)
        self.block_size = DEFAULT_BLOCK_SIZE
        self.bbag = bigblob.Machine(block_size=self.block_size)

    def make_salt(self, ty: str) -> bytes:
        """machine.go:50-54."""
        return bigblob.derive_key(self.salt, ty.encode())

    def new_typed_writer(self, store, ty: str, strict: bool = False) -> TypedWriter:
        """glfs.go:74-76 (strict: the reference's per-Write error timing)."""
        return TypedWriter(ty, self.bbag.new_writer(store, self.make_salt(ty), strict=strict))

    def post_typed(self, store, ty: str, r) -> Ref:
        """glfs.go:50-57."""
        tw = self.new_typed_writer(store, ty)
        try:
            bigblob._copy(tw, r)
            return tw.finish()
        finally:
            tw.bw.close()

    def post_blob(self, store, r) -> Ref:
        """blob.go:15-17."""
        return self.post_typed(store, TYPE_BLOB, r)

    def post_blobs(self, store, blobs) -> list:
        """n sequential PostBlob calls (machine.go:64-66), batched: blobs of
        at most 16 KiB share one GPU launch pair (one lane per blob), larger
        ones go through the Writer.  The store sees the same Posts in the
        same order."""
        import ctypes
        from . import _native as N
        blobs = [bytes(b) for b in blobs]
        n = len(blobs)
        if n == 0:
            return []
        offs, lens, pos = [], [], 0
        for b in blobs:
            offs.append(pos)
            lens.append(len(b))
            pos += len(b)
        data = b"".join(blobs)
        O = (ctypes.c_uint64 * n)(*offs)
        L = (ctypes.c_uint64 * n)(*lens)
        roots = ctypes.create_string_buffer(64 * n)
        cb, errors, ctx = bigblob._make_post_cb(store)
        rc = N.lib.glfsx_post_blobs(self.block_size, store.max_size(),
                                    self.make_salt(TYPE_BLOB), None, data or b"\0",
                                    O, L, n, cb, ctx, roots)
        if rc == N.GLFSX_E_STORE and errors:
            raise bigblob.StoreError(rc, repr(errors[0])) from errors[0]
        N.check(rc)
        rr = roots.raw   # (.raw copies the whole buffer on every access)
        return [Ref(TYPE_BLOB, Root(bigblob.Ref(rr[64 * i:64 * i + 32], rr[64 * i + 32:64 * i + 64]),
                                    lens[i], self.block_size)) for i in range(n)]

    def new_blob_writer(self, store) -> TypedWriter:
        """blob.go:37-39."""
        return self.new_typed_writer(store, TYPE_BLOB)

    # ------------------------------------------------------------ read side
    def get_typed(self, store, ty: str, x: Ref) -> bigblob.Reader:
        """glfs.go:59-66 GetTyped (ty "" accepts any type)."""
        if ty and x.type != ty:
            raise ErrRefType(x.type, ty)
        return self.bbag.new_reader(store, x.root)

    def get_blob(self, store, x: Ref) -> bigblob.Reader:
        """blob.go:20-22, 33-35."""
        return self.get_typed(store, TYPE_BLOB, x)

    def get_blob_bytes(self, store, x: Ref, max_size: int) -> bytes:
        """blob.go:25-31 (readAtMost: more than max_size bytes is an error)."""
        r = self.get_blob(store, x)
        if x.root.size > max_size:
            raise ValueError(f"blob exceeds max size {max_size}")
        return r.read()

    def sync(self, dst, src, x: Ref) -> None:
        """sync.go:14-39 Sync: copy everything x references from src into dst;
        a tree's entries are synced (from the tree bytes bigblob's Sync hands
        over) before the tree blob itself; nothing happens when dst already
        has the root."""
        if x.type == TYPE_BLOB:
            self.bbag.sync(dst, src, x.root, lambda r: None)
        elif x.type == TYPE_TREE:
            from .tree import read_tree_bytes

            def sync_entries(r):
                for ent in read_tree_bytes(r.read()):
                    self.sync(dst, src, ent.ref)

            self.bbag.sync(dst, src, x.root, sync_entries)
        else:
            raise ValueError(f"can't sync unrecognized type {x.type}")

    def get_at_path(self, store, ref: Ref, subpath: str) -> Ref:
        """tree.go:91-99 GetAtPath (ErrNoEnt when nothing is at subpath)."""
        from .tree import get_at_path
        return get_at_path(store, ref, subpath)

    # ---------------------------------------------------------------- trees
    def new_tree_writer(self, store, **kw):
        """tree.go:290-298."""
        from .tree import TreeWriter
        return TreeWriter(self, store, **kw)

    def post_tree(self, store, ents, **kw) -> Ref:
        """tree.go:195-238."""
        from .tree import post_tree
        return post_tree(self, store, ents, **kw)

    def post_tree_slice(self, store, ents, **kw) -> Ref:
        """tree.go:240-247."""
        return self.post_tree(store, list(ents), **kw)

    def post_tree_map(self, store, m: dict, **kw) -> Ref:
        """tree.go:249-260."""
        from .tree import post_tree_map
        return post_tree_map(self, store, m, **kw)

    def get_tree_slice(self, store, ref: Ref, max_ents: int = 10 ** 6, **kw) -> list:
        """tree.go:137-143."""
        from .tree import get_tree_slice
        return get_tree_slice(store, ref, max_ents, **kw)


_default: Optional[Machine] = None


def _default_machine() -> Machine:
    global _default
    if _default is None:
        _default = Machine()
    return _default


def post_typed(store, ty: str, r) -> Ref:
    """machine.go:59-61."""
    return _default_machine().post_typed(store, ty, r)


def post_blob(store, r) -> Ref:
    """machine.go:64-66."""
    return _default_machine().post_blob(store, r)


def post_blobs(store, blobs) -> list:
    """Batched PostBlob on the default machine (see Machine.post_blobs)."""
    return _default_machine().post_blobs(store, blobs)


def sync(dst, src, x: Ref) -> None:
    """sync.go:14 on the default machine."""
    _default_machine().sync(dst, src, x)


def get_at_path(store, ref: Ref, subpath: str) -> Ref:
    """tree.go:91 on the default machine."""
    return _default_machine().get_at_path(store, ref, subpath)


def post_tree(store, ents) -> Ref:
    """tree.go:195 PostTree on the default machine."""
    return _default_machine().post_tree(store, ents)


def post_tree_slice(store, ents) -> Ref:
    """tree.go:240 PostTreeSlice on the default machine."""
    return _default_machine().post_tree_slice(store, ents)


def post_tree_map(store, m: dict) -> Ref:
    """tree.go:250 PostTreeMap on the default machine."""
    return _default_machine().post_tree_map(store, m)


def get_tree_slice(store, ref: Ref, max_ents: int = 10 ** 6) -> list:
    """tree.go:137 GetTreeSlice on the default machine."""
    return _default_machine().get_tree_slice(store, ref, max_ents)


def new_blob_writer(store) -> TypedWriter:
    """blob.go:37-39 NewBlobWriter on the default machine."""
    return _default_machine().new_blob_writer(store)


def get_blob(store, x: Ref) -> bigblob.Reader:
    """blob.go:20-22 GetBlob on the default machine."""
    return _default_machine().get_blob(store, x)
