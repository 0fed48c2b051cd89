"""Trees: the glfs directory object over the GPU write path.

Reference: tree.go (blobcache/glfs, Go).  A tree is a typed blob (type
"tree", typeSalt = DeriveKey(0^32, "tree")) whose bytes are JSON lines, one
TreeEntry per line, sorted by name (tree.go:284-320 TreeWriter, 195-238
PostTree).  The bytes go through the same bigblob Writer (GPU DEK + ChaCha20 +
CID) as every blob.

The line format is Go's ``json.Encoder.Encode(TreeEntry)`` (go 1.25, go.mod:3):
``{"name":N,"mode":M,"ref":{"type":T,"cid":C,"dek":"<hex>","size":S,"blockSize":B}}\\n``
with field order from the struct tags (tree.go:74-78, glfs.go:35-38,
bigblob/blob.go:17-21, bigblob/ref.go:54-57) and Go's string escaping (HTML
characters as \\u003c/\\u003e/\\u0026, U+2028/2029 escaped, \\b \\f \\n \\r \\t,
other control bytes as \\u00XX, invalid UTF-8 as U+FFFD).

PARITY UNPINNED at one field: ``cid`` is blobcache.CID's JSON form, which
lives in the blobcache module (go.mod:16) and is absent here.  The encoder is
a parameter (``cid_json``); the default writes the lower-case hex string.
Everything else in the line is fixed by the reference.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Callable, Iterable, Optional

from . import bigblob
from . import glfs
from .bigblob import Root

MODE_DIR = 1 << 31          # os.ModeDir
MODE_FILE = 0o644           # tree.go:262-267 getFileMode
MODE_TREE = 0o755 | MODE_DIR


class TreeError(ValueError):
    """The errors tree.go returns with fmt.Errorf / errors.New."""


class ErrNoEnt(KeyError):
    """errors.go:8-14 ErrNoEnt{Name}."""

    def __init__(self, name: str):
        super().__init__(f"no entry at {name}")
        self.name = name


def is_err_no_ent(err: BaseException) -> bool:
    """errors.go:16-18."""
    return isinstance(err, ErrNoEnt)


@dataclass(frozen=True)
class TreeEntry:
    """tree.go:74-78 TreeEntry{Name, FileMode, Ref}."""
    name: str
    file_mode: int
    ref: glfs.Ref

    def validate(self) -> None:
        """tree.go:80-89."""
        if clean_path(self.name) != self.name:
            raise TreeError(f"name ({self.name}) is not properly cleaned")
        if self.name == "":
            raise TreeError("TreeEntry name cannot be empty")


def get_file_mode(ref: glfs.Ref) -> int:
    """tree.go:262-267."""
    return MODE_TREE if ref.type == glfs.TYPE_TREE else MODE_FILE


def _go_path_clean(p: str) -> str:
    """Go path.Clean (lexical): collapse //, drop ., resolve .. where it can."""
    if p == "":
        return "."
    rooted = p.startswith("/")
    out: list[str] = []
    for part in p.split("/"):
        if part in ("", "."):
            continue
        if part == "..":
            if out and out[-1] != "..":
                out.pop()
            elif not rooted:
                out.append("..")
            continue
        out.append(part)
    s = "/".join(out)
    if rooted:
        return "/" + s
    return s or "."


def clean_path(x: str) -> str:
    """tree.go:269-277 CleanPath."""
    x = _go_path_clean(x).strip("/")
    return "" if x == "." else x


def is_valid_name(x: str) -> bool:
    """tree.go:279-282."""
    return x != "" and "/" not in x


def _name_key(name: str) -> bytes:
    # strings.Compare is byte-wise on the Go string's bytes
    return go_bytes(name)


def sort_tree_entries(ents: list) -> None:
    """tree.go:32-34 (slices.SortFunc by name)."""
    ents.sort(key=lambda e: _name_key(e.name))


def validate_tree_entries(ents: list) -> None:
    """tree.go:36-50."""
    keys = [_name_key(e.name) for e in ents]
    if keys != sorted(keys):
        raise TreeError("tree entries are not sorted")
    for a, b in zip(ents, ents[1:]):
        if a.name == b.name:
            raise TreeError(f"duplicate tree entry {a} {b}")
    for e in ents:
        e.validate()


def lookup(ents: list, name: str) -> Optional[TreeEntry]:
    """tree.go:22-30 (binary search over sorted entries)."""
    lo, hi, k = 0, len(ents), _name_key(name)
    while lo < hi:
        mid = (lo + hi) // 2
        if _name_key(ents[mid].name) < k:
            lo = mid + 1
        else:
            hi = mid
    if lo < len(ents) and ents[lo].name == name:
        return ents[lo]
    return None


# ------------------------------------------------------------------- JSON
_ESC = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t",
        "\b": "\\b", "\f": "\\f", "<": "\\u003c", ">": "\\u003e", "&": "\\u0026",
        "\u2028": "\\u2028", "\u2029": "\\u2029"}


def go_bytes(s: str) -> bytes:
    """A Go string's bytes from its Python mirror: undecodable bytes ride in
    a str as surrogate escapes (U+DC80..U+DCFF); other lone surrogates are
    kept as their (invalid) 3-byte encodings."""
    try:
        return s.encode("utf-8", "surrogateescape")
    except UnicodeEncodeError:
        return s.encode("utf-8", "surrogatepass")


def go_json_string(s: str) -> str:
    """encoding/json appendString with escapeHTML (the Encoder default):
    invalid UTF-8 becomes the 6-byte escape \\ufffd, one per bad byte."""
    out = ['"']
    for ch in go_bytes(s).decode("utf-8", "surrogateescape"):
        e = _ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ch < " ":
            out.append("\\u%04x" % ord(ch))
        elif 0xD800 <= ord(ch) <= 0xDFFF:  # an undecodable byte
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def cid_json_hex(cid: bytes) -> str:
    """Default CID JSON form (parity unpinned, see module docstring)."""
    return '"' + cid.hex() + '"'


def ref_json(ref: glfs.Ref, cid_json: Callable[[bytes], str] = cid_json_hex) -> str:
    """glfs.Ref as encoding/json writes it: Type, then the promoted fields of
    the embedded bigblob.Root (cid, dek, size, blockSize)."""
    r = ref.root
    return ('{"type":' + go_json_string(ref.type) + ',"cid":' + cid_json(r.ref.cid)
            + ',"dek":"' + r.ref.dek.hex() + '","size":' + str(r.size)
            + ',"blockSize":' + str(r.block_size) + "}")


def entry_json_line(te: TreeEntry, cid_json: Callable[[bytes], str] = cid_json_hex) -> bytes:
    """json.Encoder.Encode(te): one line, trailing newline."""
    s = ('{"name":' + go_json_string(te.name) + ',"mode":' + str(te.file_mode)
         + ',"ref":' + ref_json(te.ref, cid_json) + "}\n")
    return s.encode("utf-8")


def encode_lines(ents, cid_json: Callable[[bytes], str] = cid_json_hex):
    """The JSON lines of `ents` in order, and each line's end offset.  The
    default cid form is encoded natively (glfsx_tree_encode: host C++,
    multi-threaded, byte-identical to entry_json_line); a custom cid_json
    goes through entry_json_line."""
    import ctypes
    from . import _native as N
    n = len(ents)
    if cid_json is not cid_json_hex or n == 0:
        lines = [entry_json_line(e, cid_json) for e in ents]
        ends, acc = [], 0
        for ln in lines:
            acc += len(ln)
            ends.append(acc)
        return b"".join(lines), ends
    names = [go_bytes(e.name) for e in ents]
    types = [go_bytes(e.ref.type) for e in ents]
    U64 = ctypes.c_uint64 * (n + 1)

    def offs(parts):
        o, acc = [0], 0
        for p in parts:
            acc += len(p)
            o.append(acc)
        return U64(*o)

    modes = (ctypes.c_uint32 * n)(*[e.file_mode for e in ents])
    roots = b"".join(e.ref.root.ref.cid + e.ref.root.ref.dek for e in ents)
    sizes = (ctypes.c_uint64 * n)(*[e.ref.root.size for e in ents])
    bss = (ctypes.c_uint64 * n)(*[e.ref.root.block_size for e in ents])
    nb, tb = b"".join(names), b"".join(types)
    no, to = offs(names), offs(types)
    total = ctypes.c_uint64()
    ends = (ctypes.c_uint64 * n)()
    N.check(N.lib.glfsx_tree_encode(n, nb, no, modes, tb, to, roots, sizes, bss, None, 0,
                                    ctypes.byref(total), ends))
    out = ctypes.create_string_buffer(max(total.value, 1))
    N.check(N.lib.glfsx_tree_encode(n, nb, no, modes, tb, to, roots, sizes, bss, out,
                                    total.value, ctypes.byref(total), ends))
    return out.raw[:total.value], list(ends)


def _cid_from_json(v) -> bytes:
    if isinstance(v, str):
        return bytes.fromhex(v)
    raise TreeError(f"cannot decode cid {v!r}")


def entry_from_json(obj: dict, cid_from_json=_cid_from_json) -> TreeEntry:
    r = obj["ref"]
    root = Root(bigblob.Ref(cid_from_json(r["cid"]), bytes.fromhex(r["dek"])),
                int(r["size"]), int(r["blockSize"]))
    return TreeEntry(obj["name"], int(obj["mode"]), glfs.Ref(r["type"], root))


# ------------------------------------------------------------------ writer
class TreeWriter:
    """tree.go:284-320.  Put checks order and referential integrity, then
    json-encodes the entry into a TypedWriter("tree").  The typed writer runs
    in strict mode, so a store error surfaces at the same Put as in the
    reference (the Put whose line completes the failing block)."""

    def __init__(self, machine: "glfs.Machine", store,
                 cid_json: Callable[[bytes], str] = cid_json_hex):
        self.dst = store
        self.tw = machine.new_typed_writer(store, glfs.TYPE_TREE, strict=True)
        self.cid_json = cid_json
        self.last_name = ""

    def _check(self, te: TreeEntry, last: str) -> None:
        if _name_key(te.name) <= _name_key(last):
            raise TreeError(f"cannot write tree entries out of order "
                            f"{te.name!r} <= {last!r}")
        if not exists_unit(self.dst, te.ref.root.ref.cid):
            raise TreeError(f"adding tree ent {te} would violate referential integrity")

    def put(self, te: TreeEntry) -> None:
        """tree.go:295-312."""
        self._check(te, self.last_name)
        self.tw.write(entry_json_line(te, self.cid_json))
        self.last_name = te.name

    def put_many(self, ents) -> None:
        """Put each entry in order (tree.go:295-312), batched: the entries
        before the first failing check are encoded at once (natively) and
        written, then that check's error is raised -- the same bytes reach
        the Writer as with one Put per entry."""
        ents = list(ents)
        err, k, last = None, len(ents), self.last_name
        for i, te in enumerate(ents):
            try:
                self._check(te, last)
            except TreeError as e:
                err, k = e, i
                break
            last = te.name
        if k:
            data, _ = encode_lines(ents[:k], self.cid_json)
            self.tw.write(data)
            self.last_name = ents[k - 1].name
        if err is not None:
            raise err

    def finish(self) -> glfs.Ref:
        """tree.go:315-317."""
        try:
            return self.tw.finish()
        finally:
            self.tw.bw.close()


def exists_unit(store, cid: bytes) -> bool:
    """bigblob.ExistsUnit [ext store]: the store's Exists for one CID."""
    return bool(store.exists(cid))


def post_tree(machine: "glfs.Machine", store, ents: Iterable[TreeEntry],
              cid_json: Callable[[bytes], str] = cid_json_hex) -> glfs.Ref:
    """tree.go:195-238 PostTree: entries may carry paths; subdirectories are
    posted first (recursively), then this level's sorted entries."""
    root_ents: list = []
    subents: dict = {}
    for ent in ents:
        p = clean_path(ent.name)
        if p == "":
            return ent.ref
        parts = p.split("/", 1)
        if len(parts) == 1:
            root_ents.append(TreeEntry(parts[0], ent.file_mode, ent.ref))
        else:
            subents.setdefault(parts[0], []).append(
                TreeEntry(parts[1], ent.file_mode, ent.ref))
    for k, ents2 in subents.items():
        ref = post_tree(machine, store, ents2, cid_json)
        root_ents.append(TreeEntry(k, get_file_mode(ref), ref))
    sort_tree_entries(root_ents)
    tw = TreeWriter(machine, store, cid_json)
    try:
        tw.put_many(root_ents)
    except BaseException:
        tw.tw.bw.close()
        raise
    return tw.finish()


def post_tree_map(machine: "glfs.Machine", store, m: dict,
                  cid_json: Callable[[bytes], str] = cid_json_hex) -> glfs.Ref:
    """tree.go:249-260 PostTreeMap."""
    return post_tree(machine, store,
                     [TreeEntry(k, get_file_mode(v), v) for k, v in m.items()], cid_json)


# ------------------------------------------------------------------ reader
def read_tree_bytes(data: bytes, cid_from_json=_cid_from_json) -> list:
    """TreeReader.Next over the decoded bytes (tree.go:340-372): a stream of
    JSON values, each a TreeEntry, strictly increasing names, each valid."""
    dec = json.JSONDecoder()
    s = data.decode("utf-8", "replace")
    i, n, out, last = 0, len(s), [], ""
    while True:
        while i < n and s[i] in " \t\r\n":
            i += 1
        if i >= n:
            return out
        obj, i = dec.raw_decode(s, i)
        te = entry_from_json(obj, cid_from_json)
        if _name_key(te.name) <= _name_key(last):
            raise TreeError(f"tree entries are out of order: {te.name} <= {last}")
        te.validate()
        last = te.name
        out.append(te)


def get_tree_slice(store, ref: glfs.Ref, max_ents: int = 10 ** 6,
                   cid_from_json=_cid_from_json) -> list:
    """tree.go:137-143 GetTreeSlice (the read side decrypts on the GPU)."""
    if ref.type != glfs.TYPE_TREE:
        raise TreeError(f"wrong ref type: have {ref.type} want {glfs.TYPE_TREE}")
    ents = read_tree_bytes(bigblob.read_all(store, ref.root), cid_from_json)
    return ents[:max_ents]


def lookup_path(store, ent: TreeEntry, subpath: str,
                cid_from_json=_cid_from_json) -> TreeEntry:
    """tree.go:101-133 Lookup: walk subpath one name at a time through the
    (GPU-decrypted) tree blobs; entries are sorted, so a scan stops at the
    first name past the wanted one."""
    subpath = subpath.strip("/")
    if subpath == "":
        return ent
    if ent.ref.type != glfs.TYPE_TREE:
        raise TreeError("can only take subpath of type tree")
    head, _, rest = subpath.partition("/")
    for e in get_tree_slice(store, ent.ref, 1 << 62, cid_from_json):
        if e.name == head:
            return lookup_path(store, e, rest, cid_from_json)
        if _name_key(e.name) > _name_key(head):
            break
    raise ErrNoEnt(head)


def get_at_path(store, ref: glfs.Ref, subpath: str, cid_from_json=_cid_from_json) -> glfs.Ref:
    """tree.go:91-99 GetAtPath."""
    return lookup_path(store, TreeEntry("", 0, ref), subpath, cid_from_json).ref
