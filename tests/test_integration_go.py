"""The reference-side binding (integration/go/) is real: the patch applies to
the reference's bigblob/blob.go, the cgo preamble compiles against
include/glfsx.h, and every C symbol and Go hook it uses exists.

There is no Go toolchain in this image, so the Go files are
checked structurally; the C half of the cgo binding is compiled with gcc.
`git apply --check` only reads /root/reference (nothing is written there).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "integration", "go")
REF = "/root/reference"


def _read(name):
    with open(os.path.join(GO, name)) as f:
        return f.read()


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bigblob")) or not shutil.which("git"),
                    reason="the reference checkout is only in the build container")
def test_patch_applies_to_reference():
    p = subprocess.run(["git", "apply", "--check", "-v", os.path.join(GO, "bigblob_gpu.patch")],
                       cwd=REF, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    assert "Checking patch bigblob/blob.go" in p.stderr


def test_patch_hooks_exist_in_both_builds():
    """What the patched blob.go calls (newGPUWriter, gpu.ctx, gpu.Write,
    gpu.Finish, the gpu field's type) is defined with and without the
    glfsgpu tag, with the reference's types (bcsdk.WO, blob.go:85)."""
    patch = _read("bigblob_gpu.patch")
    added = "\n".join(ln[1:] for ln in patch.splitlines()
                      if ln.startswith("+") and not ln.startswith("+++"))
    assert "w.gpu = ag.newGPUWriter(s, salt, blockSize)" in added
    assert "w.gpu.write(&w.buf, data)" in added and "w.gpu.Finish(ctx)" in added
    assert "w.gpu.ctx = ctx" in added and "gpu *gpuWriter" in added
    assert "return w.gpu.readFrom(&w.buf, r)" in added and "io.Copy(writerOnly{w}, r)" in added
    # round 6: a writer that never reached the GPU finishes on the Go path
    assert "if w.gpu.started() {" in added and "w.gpu = nil" in added
    # context lines are the reference's own (blob.go:85-86)
    assert " func (ag *Machine) NewWriter(s bcsdk.WO, salt *[32]byte) *Writer {" in patch
    assert "-\treturn &Writer{" in patch and "+\tw := &Writer{" in patch
    for name, tag in (("gpu.go", "//go:build glfsgpu"), ("gpu_stub.go", "//go:build !glfsgpu")):
        src = _read(name)
        assert src.startswith(tag + "\n"), name
        assert re.search(r"^package bigblob$", src, re.M), name
        assert re.search(r"type gpuWriter struct\s*\{[^}]*\bctx\s+context\.Context", src, re.S), name
        assert re.search(r"func \(ag \*Machine\) newGPUWriter\((s )?bcsdk\.WO, (salt )?\*\[32\]byte, "
                         r"(blockSize )?int\) \*gpuWriter", src), name
        assert re.search(r"func \(gw \*gpuWriter\) started\(\) bool", src), name
        assert re.search(r"func \(gw \*gpuWriter\) write\((buf )?\*\[\]byte, (data )?\[\]byte\) "
                         r"\(int, error\)", src), name
        assert re.search(r"func \(gw \*gpuWriter\) readFrom\((buf )?\*\[\]byte, (r )?io\.Reader\) "
                         r"\(int64, error\)", src), name
        assert re.search(r"func \(gw \*gpuWriter\) Write\((data )?\[\]byte\) \(int, error\)", src), name
        assert re.search(r"func \(gw \*gpuWriter\) Finish\((ctx )?context\.Context\) "
                         r"\(\*Root, error\)", src), name
        assert re.search(r"func \(gw \*gpuWriter\) ReadFrom\((r )?io\.Reader\) "
                         r"\(int64, error\)", src), name
        assert "schema.WO" not in src, name
        assert src.count("{") == src.count("}"), name
        assert src.count("(") == src.count(")"), name


def test_cgo_symbols_are_in_the_header():
    hdr = open(os.path.join(ROOT, "include", "glfsx.h")).read()
    src = _read("gpu.go")
    used = set(re.findall(r"\b(glfsx_\w+)", src))
    assert used, "no C symbols?"
    for sym in sorted(used):
        assert re.search(r"\b" + sym + r"\b", hdr), sym
    for const in set(re.findall(r"C\.(GLFSX_\w+)", src)):
        assert re.search(r"\b" + const + r"\b", hdr), const


@pytest.mark.skipif(not shutil.which("gcc"), reason="no gcc")
def test_cgo_preamble_compiles(tmp_path):
    """The cgo preamble of gpu.go is plain C over glfsx.h: compile it with
    gcc -Werror (goPost, which cgo generates from the //export, is stubbed)."""
    src = _read("gpu.go")
    m = re.search(r"/\*\n(.*?)\*/\nimport \"C\"", src, re.S)
    assert m, "no cgo preamble"
    pre = "\n".join(ln for ln in m.group(1).splitlines() if not ln.startswith("#cgo"))
    c = tmp_path / "preamble.c"
    c.write_text(pre + """
int goPost(uintptr_t ctx, int kind, uint8_t *ref, void *ctext, uint64_t len) {
  (void)ctx; (void)kind; (void)ref; (void)ctext; (void)len; return 0;
}
int64_t goReadAt(uintptr_t ctx, void *buf, uint64_t len, uint64_t off) {
  (void)ctx; (void)buf; (void)len; (void)off; return 0;
}
void *touch(void) {
  static void *fns[7];
  fns[0] = (void *)writer_new; fns[1] = (void *)writer_devices;
  fns[2] = (void *)derive_key; fns[3] = (void *)post_tramp;
  fns[4] = (void *)writer_read_fd; fns[5] = (void *)writer_read_at;
  fns[6] = (void *)read_at_tramp;
  return fns;
}
""")
    p = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-c",
                        "-I", os.path.join(ROOT, "include"), str(c), "-o",
                        str(tmp_path / "preamble.o")], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_integration_md_embeds_the_shipped_files():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "embed_integration", os.path.join(ROOT, "scripts", "embed_integration.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert text.count("<!-- embed: integration/go/") == 6
    assert mod.render(text) == text, "run scripts/embed_integration.py"


@pytest.mark.skipif(not shutil.which("gcc"), reason="no gcc")
def test_glfs_cgo_preamble_compiles(tmp_path):
    """glfs_gpu.go's preamble (PostBlobs / PostTreeMapGPU) compiles with gcc
    -Werror against glfsx.h (goPostBlobs stubbed)."""
    src = _read("glfs_gpu.go")
    m = re.search(r"/\*\n(.*?)\*/\nimport \"C\"", src, re.S)
    assert m, "no cgo preamble"
    pre = "\n".join(ln for ln in m.group(1).splitlines() if not ln.startswith("#cgo"))
    c = tmp_path / "glfs_preamble.c"
    c.write_text(pre + """
int goPostBlobs(uintptr_t ctx, int kind, uint8_t *ref, void *ctext, uint64_t len) {
  (void)ctx; (void)kind; (void)ref; (void)ctext; (void)len; return 0;
}
void *touch(void) {
  static void *fns[2];
  fns[0] = (void *)post_blobs; fns[1] = (void *)tree_encode;
  return fns;
}
""")
    p = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-c",
                        "-I", os.path.join(ROOT, "include"), str(c), "-o",
                        str(tmp_path / "glfs_preamble.o")], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_cgo_handles_never_become_go_pointers():
    """a cgo.Handle (small integers from 1) converted to
    unsafe.Pointer in Go trips checkptr; it must travel as C.uintptr_t and
    the exported callbacks must take uintptr_t."""
    for name in ("gpu.go", "glfs_gpu.go"):
        src = _read(name)
        assert not re.search(r"unsafe\.Pointer\(uintptr\(", src), name
        for fn in re.findall(r"//export (\w+)\nfunc \w+\(([^)]*)\)", src):
            assert fn[1].startswith("ctx C.uintptr_t"), (name, fn)
        for ext in re.findall(r"extern \w+ (go\w+)\(([^)]*)\)", src):
            assert ext[1].startswith("uintptr_t ctx"), (name, ext)


def test_glfs_batch_entry_points_in_both_builds():
    """PostBlobs / PostTreeMapGPU exist with and without the glfsgpu tag,
    with the same signatures, in package glfs; the shared helper has no
    build tag; the reference names they call exist in the reference."""
    sig_pb = r"func \(ag \*Machine\) PostBlobs\(ctx context\.Context, s schema\.WO, " \
             r"blobs \[\]\[\]byte\) \(\[\]Ref, error\)"
    sig_tm = r"func \(ag \*Machine\) PostTreeMapGPU\(ctx context\.Context, s schema\.WO, " \
             r"m map\[string\]Ref\) \(\*Ref, error\)"
    for name, tag in (("glfs_gpu.go", "//go:build glfsgpu"),
                      ("glfs_gpu_stub.go", "//go:build !glfsgpu")):
        src = _read(name)
        assert src.startswith(tag + "\n"), name
        assert re.search(r"^package glfs$", src, re.M), name
        assert re.search(sig_pb, src) and re.search(sig_tm, src), name
        assert src.count("{") == src.count("}") and src.count("(") == src.count(")"), name
    shared = _read("glfs_batch.go")
    assert "//go:build" not in shared and re.search(r"^package glfs$", shared, re.M)
    assert "func postBlobsSeq(" in shared
    if os.path.isdir(REF):
        ref = "".join(open(os.path.join(REF, f)).read()
                      for f in ("machine.go", "tree.go", "glfs.go", "blob.go"))
        for name in ("func (ag *Machine) PostTreeMap(", "func (ag *Machine) PostBlob(",
                     "func (ag *Machine) PostTyped(", "func (ag *Machine) makeSalt(",
                     "func SortTreeEntries(", "func CleanPath(", "func getFileMode(",
                     "TypeBlob = ", "TypeTree = "):
            assert name in ref, name


def test_read_from_matches_io_copy_file_wrapper():
    """since Go 1.22 io.Copy(w, *os.File) reaches ReadFrom
    with f.WriteTo's fileWithoutWriteTo wrapper, so the pread route takes an
    *os.File or exactly that wrapper type (plainFile, by dynamic type name);
    a user type embedding *os.File that overrides Read has the same methods
    and must NOT match, so nothing is matched by method set.  gpu_test.go
    (glfsgpu tag) checks both through io.Copy."""
    src = _read("gpu.go")
    body = src[src.index("func (gw *gpuWriter) readFromRoutes("):]
    body = body[:body.index("\n}\n")]
    assert "r.(osFile)" not in body and "plainFile(r)" in body
    assert "positionedReader(r)" in body and "io.ReaderAt\n" not in body
    assert "atomic.AddUint64(&fdRouteReads, 1)" in body
    pf = src[src.index("func plainFile("):]
    pf = pf[:pf.index("\n}\n")]
    assert 'r.(*os.File)' in pf and '"os.fileWithoutWriteTo"' in pf
    pr = src[src.index("func positionedReader("):]
    pr = pr[:pr.index("\n}\n")]
    assert "case *io.SectionReader:" in pr and "case *bytes.Reader:" in pr
    iface = re.search(r"type osFile interface \{([^}]*)\}", src)
    assert iface and "Fd() uintptr" in iface.group(1) and "io.Seeker" in iface.group(1) \
        and "Stat() (os.FileInfo, error)" in iface.group(1)
    test = _read("gpu_test.go")
    assert test.startswith("//go:build glfsgpu\n") and re.search(r"^package bigblob$", test, re.M)
    assert "fdRouteReads" in test and "ag.Create(ctx" in test and 'import "C"' not in test
    assert "type upperFile struct{ *os.File }" in test
    assert "TestCreateFromFileWrapperUsesItsRead" in test
    assert test.count("{") == test.count("}") and test.count("(") == test.count(")")


def test_strict_error_timing_is_the_default():
    """the drop-in returns a store error where the
    reference does by default (GLFSX_STRICT=1): Write with blob.go:120-133's
    timing; ReadFrom pipelines its own batches with the writer's strict flag
    off and flushes before it returns, so io.Copy still gets the error
    (tests/test_gpu_writer.py::test_strict_read_from_returns_the_io_copy_error
    runs the same sequence through the C-ABI)."""
    src = _read("gpu.go")
    assert 'strict      = envInt("GLFSX_STRICT", 1)' in src
    body = src[src.index("func (gw *gpuWriter) ReadFrom("):]
    body = body[:body.index("\n}\n")]
    assert "C.glfsx_writer_set_strict(gw.w, 0)" in body
    assert body.index("C.glfsx_writer_set_strict(gw.w, 0)") < body.index("n, err := gw.readFromRoutes(r)") \
        < body.index("C.glfsx_writer_set_strict(gw.w, 1)") < body.index("C.glfsx_writer_flush(gw.w)")
    assert "func (gw *gpuWriter) readFromRoutes(r io.Reader) (int64, error) {" in src
    assert src.count("{") == src.count("}") and src.count("(") == src.count(")")
