"""The library's remaining tunables, each at a
non-default value once, against the oracle.

The library reads five GLFSX_* variables, all tuning, none selecting a
different algorithm: GLFSX_BATCH_MIB and GLFSX_SLOTS (read by every
glfsx_writer_new: the Writer's batch size and pinned slots per lane),
GLFSX_SPIN_US (the poll bound of a wait), GLFSX_NUMA (copy-pool threads on
the GPU's NUMA node) and GLFSX_READ_THREADS (reader threads per batch of
glfsx_writer_read_fd / _read_at) -- the last three are read once per
process, so they run in a child process.  The Python binding reads GLFSX_LIB
(a build variant, tests/test_gpu_variants.py).
"""
import ctypes
import os
import subprocess
import sys

import pytest

from test_gpu_multi import _gpu_post_log, _oracle_post_log

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20

@pytest.mark.parametrize("env", [{"GLFSX_SLOTS": "2"}, {"GLFSX_SLOTS": "4"},
                                 {"GLFSX_BATCH_MIB": "3"}])
def test_writer_knobs_vs_oracle(gpu, O, env):
    """A 70 MiB + 5 B host stream at 1 MiB blocks in 4 MiB writes, with 2 or
    4 batch slots per lane, or 3-block batches: the whole Post log and root
    equal the oracle writer's."""
    data = O.fill_splitmix(70 * MIB + 5, 17)
    want_root, want_log = _oracle_post_log(O, data, MIB)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        root, log = _gpu_post_log(gpu, data, MIB, None, 4 * MIB)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    assert root == want_root
    assert log == want_log


_CHILD = r"""
import ctypes, os, sys, tempfile
sys.path.insert(0, {root!r})
from glfs_amd import _native as N
from oracle import oracle as O
N.set_device(0)
data = O.fill_splitmix(70 * (1 << 20) + 3, 23)
want = O.create(data, 1 << 20)[0]
# glfsx_create: host Writer, one-shot posts and waits (GLFSX_SPIN_US)
root = N.glfsx_root()
N.check(N.lib.glfsx_create(1 << 20, 1 << 20, None, None, data, len(data), N.POST_FN(0), None,
                           ctypes.byref(root)))
assert bytes(root.ref) == want, "create"
# a file through the pread feeder (GLFSX_READ_THREADS, the copy pool: GLFSX_NUMA)
fd, path = tempfile.mkstemp(prefix="glfsx_knob_")
try:
    os.write(fd, data)
    err, got = ctypes.c_int(), ctypes.c_uint64()
    w = N.lib.glfsx_writer_new(1 << 20, 1 << 20, None, None, N.POST_FN(0), None, ctypes.byref(err))
    assert w
    try:
        N.check(N.lib.glfsx_writer_read_fd(w, fd, 0, len(data), ctypes.byref(got)))
        N.check(N.lib.glfsx_writer_finish(w, ctypes.byref(root)))
    finally:
        N.lib.glfsx_writer_free(w)
    assert got.value == len(data) and bytes(root.ref) == want, "read_fd"
finally:
    os.close(fd)
    os.unlink(path)
print("knobs ok")
"""


@pytest.mark.parametrize("env", [{"GLFSX_SPIN_US": "0"}, {"GLFSX_NUMA": "0"},
                                 {"GLFSX_READ_THREADS": "2"}])
def test_process_knobs_vs_oracle(gpu, env):
    """The once-per-process knobs, each in a child process: a 70 MiB Create
    from host memory and the same bytes through the file feeder, both roots
    equal to the oracle's."""
    e = dict(os.environ)
    e.update(env)
    p = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT)], capture_output=True,
                       text=True, timeout=300, env=e, cwd=ROOT)
    assert p.returncode == 0 and "knobs ok" in p.stdout, (p.returncode, p.stderr[-3000:])
