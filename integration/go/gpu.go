//go:build glfsgpu

// The bigblob write path on MI355X: with -tags glfsgpu, every
// bigblob.Writer (and so glfs.PostBlob / PostTyped / TypedWriter / PostTree
// and bigblob.Create / Concat) hashes through libglfsx (include/glfsx.h).
// Goes to bigblob/gpu.go of blobcache/glfs; bigblob_gpu.patch adds the
// delegation to blob.go.  Build: CGO_CFLAGS=-I<glfsx>/include
// CGO_LDFLAGS="-L<glfsx>/lib -lglfsx" go build -tags glfsgpu ./...
//
// Environment:
//   GLFSX_STRICT=1   (the default) blob.go:120-133 error timing: a store
//                    error comes back from the Write that completed the
//                    failing block, and from the ReadFrom (io.Copy) call
//                    that fed it -- ReadFrom pipelines its own batches and
//                    delivers their Posts before it returns.  0 pipelines
//                    Write too: the error comes from the Write or Finish
//                    whose 64 MiB batch held it (the Posts are the same
//                    prefix either way, and Create returns the same error).
//   GLFSX_DEVICES=0,1,...  hash each Writer's batches round-robin on these
//                    GPUs (one Writer fed by one io.Reader over several PCIe
//                    links; Posts still in block order).
//   GLFSX_PARITY=k   re-hash every k-th Post through the store's own Post
//                    and compare CIDs (parity mode).

package bigblob

/*
#cgo LDFLAGS: -lglfsx
#include <stdlib.h>
#include <string.h>
#include "glfsx.h"

// C cannot call a Go func value: the writer's cgo.Handle travels through
// post_ctx as an integer (converted to void * on the C side only, so Go never
// turns a small handle value into an unsafe.Pointer -- checkptr rejects
// that) and goPost dispatches on it.
extern int goPost(uintptr_t ctx, int kind, uint8_t *ref, void *ctext, uint64_t len);
static int post_tramp(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                      uint64_t len) {
	return goPost((uintptr_t)ctx, kind, (uint8_t *)ref, (void *)ctext, len);
}
// io.ReaderAt.ReadAt for glfsx_writer_read_at, called from the library's
// reader threads (cgo runs the callback on an extra M).
extern int64_t goReadAt(uintptr_t ctx, void *buf, uint64_t len, uint64_t off);
static int64_t read_at_tramp(void *ctx, void *buf, uint64_t len, uint64_t off) {
	return goReadAt((uintptr_t)ctx, buf, len, off);
}

// glfsx_last_error() is thread-local and a goroutine may move to another OS
// thread between two cgo calls, so each wrapper copies the error text in the
// SAME C call that failed.
static void copy_err(char *err, size_t cap) {
	strncpy(err, glfsx_last_error(), cap - 1);
	err[cap - 1] = 0;
}
static glfsx_writer *writer_new(uint64_t bs, uint64_t max, const uint8_t *salt,
                                uintptr_t h, int *rc, char *err, size_t cap) {
	glfsx_writer *w = glfsx_writer_new(bs, max, salt, NULL, post_tramp, (void *)h, rc);
	if (!w) copy_err(err, cap);
	return w;
}
static int writer_read_fd(glfsx_writer *w, int fd, uint64_t off, uint64_t n, uint64_t *got) {
	return glfsx_writer_read_fd(w, fd, off, n, got);
}
static int writer_read_at(glfsx_writer *w, uintptr_t h, uint64_t off, uint64_t n,
                          uint64_t *got) {
	return glfsx_writer_read_at(w, read_at_tramp, (void *)h, off, n, got);
}
static int writer_devices(glfsx_writer *w, const int *devs, int n, char *err, size_t cap) {
	int rc = glfsx_writer_set_devices(w, devs, n);
	if (rc) copy_err(err, cap);
	return rc;
}
static int derive_key(uint8_t *out, size_t n, const uint8_t *salt, const void *in,
                      size_t len, char *err, size_t cap) {
	int rc = glfsx_derive_key(out, n, salt, in, len);
	if (rc) copy_err(err, cap);
	return rc;
}
*/
import "C"

import (
	"bytes"
	"context"
	"errors"
	"fmt"
	"io"
	"math"
	"os"
	"reflect"
	"runtime/cgo"
	"strconv"
	"strings"
	"sync"
	"sync/atomic"
	"unsafe"

	"blobcache.io/blobcache/src/bcsdk"
	"blobcache.io/blobcache/src/blobcache"
)

// PrehashedWO is implemented by stores that accept a CID the caller computed
// (the GPU already hashed every ctext): no second BLAKE3 pass on the host.
// glfsx_store (include/glfsx.h) is such a store; a blobcache client would add
// PostHashed next to Post.
type PrehashedWO interface {
	PostHashed(ctx context.Context, cid blobcache.CID, data []byte) error
}

var (
	parityEvery = envInt("GLFSX_PARITY", 0)
	strict      = envInt("GLFSX_STRICT", 1)
	devices     = envInts("GLFSX_DEVICES")
	// A blob shorter than this (and than one block) never reaches the GPU:
	// the reference's own Go path posts it.  One PostBlob per small file
	// (glfsposix, glfstar) is ~7x cheaper on a CPU core than a GPU call --
	// 4 KiB: 149 k blobs/s against 22 k calls/s from one thread, 2.39 M
	// against 0.23 M from 16 (bench cpu_baseline.small_blobs,
	// postblob_concurrency) -- and the crossover is ~32-48 KiB (DESIGN.md
	// section 11).  0 sends every blob to the GPU.
	gpuMinBytes = envInt("GLFSX_GPU_MIN_BYTES", 32<<10)
)

// gpuStarts counts writers that reached the GPU (gpu_test.go).
var gpuStarts uint64

// gpuWriter is the GPU half of a bigblob Writer.  It holds the bytes of a
// blob in the Writer's own buf until they reach minBytes; only then is the
// library's writer created (start) and the buffered bytes handed to it, so
// a blob that ends first is finished by blob.go's Go path with the same
// Posts (the GPU path's Posts are the reference's; tests/test_gpu_*).
type gpuWriter struct {
	w        *C.glfsx_writer // nil until start
	ag       *Machine
	s        bcsdk.WO
	salt     [32]byte
	minBytes int
	ctx      context.Context
	err      error // the store's error, returned by the Write/Finish that saw it
	h        cgo.Handle
	n        uint64
}

// newGPUWriter is called by NewWriter (blob.go:85-114) after the reference's
// checks: blockSize is the one it chose, salt the one it uses (never nil).
func (ag *Machine) newGPUWriter(s bcsdk.WO, salt *[32]byte, blockSize int) *gpuWriter {
	if C.glfsx_device_count() == 0 {
		return nil // no GPU: the Go path (the library has no CPU fallback)
	}
	gw := &gpuWriter{ag: ag, s: s, ctx: context.TODO(), minBytes: gpuMinBytes}
	if salt != nil {
		gw.salt = *salt
	}
	if blockSize < gw.minBytes {
		gw.minBytes = blockSize // the reference posts its first block there
	}
	return gw
}

func (gw *gpuWriter) started() bool { return gw.w != nil }

// start creates the library's writer and hands it the bytes buffered so
// far (*buf, emptied).  blob.go:85-114 (NewWriter): block size 0 means the
// store's MaxSize (bigblob machine.go:22-30).
func (gw *gpuWriter) start(buf *[]byte) error {
	if gw.w != nil {
		return nil
	}
	gw.h = cgo.NewHandle(gw)
	var rc C.int
	var cerr [512]C.char
	gw.w = C.writer_new(C.uint64_t(gw.ag.blockSize), C.uint64_t(gw.s.MaxSize()),
		(*C.uint8_t)(unsafe.Pointer(&gw.salt[0])), C.uintptr_t(gw.h), &rc, &cerr[0],
		C.size_t(len(cerr)))
	if gw.w == nil {
		gw.h.Delete()
		// (the block-size panics of blob.go:91,94 happened in NewWriter)
		return fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(&cerr[0]))
	}
	atomic.AddUint64(&gpuStarts, 1)
	C.glfsx_writer_set_strict(gw.w, C.int(strict))
	if len(devices) > 0 {
		cdevs := (*C.int)(C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0)))))
		defer C.free(unsafe.Pointer(cdevs))
		ds := unsafe.Slice(cdevs, len(devices))
		for i, d := range devices {
			ds[i] = C.int(d)
		}
		if rc := C.writer_devices(gw.w, cdevs, C.int(len(devices)), &cerr[0],
			C.size_t(len(cerr))); rc != 0 {
			gw.close()
			return fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(&cerr[0]))
		}
	}
	if len(*buf) > 0 {
		if _, err := gw.Write(*buf); err != nil {
			return err
		}
		*buf = (*buf)[:0]
	}
	return nil
}

// write is Writer.Write (blob.go:120-133) on this path: below minBytes the
// bytes wait in the Writer's buf, as the reference's do below a block.
func (gw *gpuWriter) write(buf *[]byte, data []byte) (int, error) {
	if gw.w == nil && len(*buf)+len(data) < gw.minBytes {
		*buf = append(*buf, data...)
		return len(data), nil
	}
	if err := gw.start(buf); err != nil {
		return 0, err
	}
	return gw.Write(data)
}

// readFrom is Writer.ReadFrom: the first minBytes are read into buf (a
// blob that ends there stays on the Go path), the rest by ReadFrom below.
func (gw *gpuWriter) readFrom(buf *[]byte, r io.Reader) (int64, error) {
	var n int64
	for gw.w == nil && len(*buf) < gw.minBytes {
		if cap(*buf) < gw.minBytes {
			b := make([]byte, len(*buf), gw.minBytes)
			copy(b, *buf)
			*buf = b
		}
		k, err := r.Read((*buf)[len(*buf):gw.minBytes])
		*buf = (*buf)[:len(*buf)+k]
		n += int64(k)
		if err == io.EOF {
			return n, nil
		}
		if err != nil {
			return n, err
		}
	}
	if err := gw.start(buf); err != nil {
		return n, err
	}
	m, err := gw.ReadFrom(r)
	return n + m, err
}

//export goPost
func goPost(ctx C.uintptr_t, kind C.int, ref *C.uint8_t, ctext unsafe.Pointer, n C.uint64_t) C.int {
	gw := cgo.Handle(ctx).Value().(*gpuWriter)
	// ctext is C memory, valid only during this call; the store copies it
	var data []byte
	if n > 0 {
		data = unsafe.Slice((*byte)(ctext), int(n))
	}
	var cid blobcache.CID
	copy(cid[:], unsafe.Slice((*byte)(unsafe.Pointer(ref)), 32))
	gw.n++
	if ps, ok := gw.s.(PrehashedWO); ok && (parityEvery == 0 || gw.n%uint64(parityEvery) != 0) {
		if err := ps.PostHashed(gw.ctx, cid, data); err != nil { // no host BLAKE3
			gw.err = err
			return 1
		}
		return 0
	}
	got, err := gw.s.Post(gw.ctx, data) // ref.go:103: the store hashes
	if err != nil {
		gw.err = err
		return 1
	}
	if got != cid { // parity: the store's CID must equal the GPU's
		gw.err = fmt.Errorf("glfsx: store CID %v != GPU CID %v", got, cid)
		return 2
	}
	return 0
}

func (gw *gpuWriter) fail(rc C.int) error {
	if rc == C.GLFSX_E_STORE && gw.err != nil {
		return gw.err
	}
	// the writer keeps its own error text: safe from any OS thread
	return fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(C.glfsx_writer_error(gw.w)))
}

// Write mirrors blob.go:120-133.  Go memory is passed for the duration of the
// call only (cgo pointer rules); the C side copies it into pinned staging.
func (gw *gpuWriter) Write(data []byte) (int, error) {
	if len(data) == 0 {
		return 0, nil
	}
	if rc := C.glfsx_writer_write(gw.w, unsafe.Pointer(&data[0]), C.size_t(len(data))); rc != 0 {
		return 0, gw.fail(rc)
	}
	return len(data), nil
}

// osFile is what ReadFrom needs of a file.
type osFile interface {
	Fd() uintptr
	Stat() (os.FileInfo, error)
	io.Seeker
}

// plainFile returns r as a file whose Read is the file's own read(2), or
// false: an *os.File, or io.Copy's own wrapper of one (since Go 1.22
// io.Copy(w, f) calls f.WriteTo, which for a writer that is not a socket
// calls io.Copy(w, fileWithoutWriteTo{f}), so ReadFrom never sees the
// *os.File itself -- ADVICE r4).  Matched by exact dynamic type, never by
// method set: a user type that embeds *os.File and overrides Read (to
// transform or limit the bytes) has every osFile method too, and the pread
// route would bypass its Read (ADVICE r5).
func plainFile(r io.Reader) (osFile, bool) {
	if f, ok := r.(*os.File); ok {
		return f, true
	}
	if reflect.TypeOf(r).String() == "os.fileWithoutWriteTo" {
		f, ok := r.(osFile)
		return f, ok
	}
	return nil, false
}

// positionedReader returns r as an io.ReaderAt + io.Seeker whose Read is
// ReadAt at the current offset, or false: the standard library's own types
// only, for the same reason as plainFile (an embedding type's Read may
// differ from the ReadAt it promotes).
func positionedReader(r io.Reader) (interface {
	io.ReaderAt
	io.Seeker
}, bool) {
	switch x := r.(type) {
	case *io.SectionReader:
		return x, true
	case *bytes.Reader:
		return x, true
	case *strings.Reader:
		return x, true
	}
	return nil, false
}

// fdRouteReads counts ReadFrom calls served by the pread route (gpu_test.go).
var fdRouteReads uint64

// gpuDeviceCount is glfsx_device_count for the tests (no cgo in _test.go).
func gpuDeviceCount() int { return int(C.glfsx_device_count()) }

// ReadFrom is io.Copy's fast path (Create, Concat: blob.go:213,341).  In
// strict mode (the default) the reference's io.Copy returns a store error
// from the Write that completed the failing block, i.e. from this call: the
// batches this call feeds are pipelined (the writer's strict flag is off
// meanwhile, so a generic reader's commits do not wait one block at a time)
// and glfsx_writer_flush delivers their Posts before it returns, so the
// error still comes back from this call, with the same Posts before it.
func (gw *gpuWriter) ReadFrom(r io.Reader) (int64, error) {
	if strict == 0 {
		return gw.readFromRoutes(r)
	}
	C.glfsx_writer_set_strict(gw.w, 0)
	n, err := gw.readFromRoutes(r)
	C.glfsx_writer_set_strict(gw.w, 1)
	if rc := C.glfsx_writer_flush(gw.w); rc != 0 {
		return n, gw.fail(rc) // a store error before the reader's own
	}
	return n, err
}

// readFromRoutes feeds the writer from r:
//   - A regular file (an *os.File, or io.Copy's fileWithoutWriteTo wrapper
//     of one; plainFile): read from its current offset to its end by the
//     library's reader threads with pread(2), straight into the writer's
//     pinned staging, while earlier batches hash (glfsx_writer_read_fd); the
//     file is left positioned after what was read, as io.Copy leaves it.
//   - An *io.SectionReader, *bytes.Reader or *strings.Reader
//     (positionedReader): the same through ReadAt from several threads
//     (glfsx_writer_read_at).
//   - Any other reader fills the staging directly, one Read at a time
//     (glfsx_writer_reserve / glfsx_writer_commit): every byte is copied
//     once, by r.Read, instead of into io.Copy's 32 KiB buffer and again by
//     Write.  C memory handed to Go as a slice is fine under the cgo rules;
//     it is not used after commit.
func (gw *gpuWriter) readFromRoutes(r io.Reader) (int64, error) {
	if f, ok := plainFile(r); ok {
		if st, err := f.Stat(); err == nil && st.Mode().IsRegular() {
			if pos, err := f.Seek(0, io.SeekCurrent); err == nil {
				var got C.uint64_t
				atomic.AddUint64(&fdRouteReads, 1)
				rc := C.writer_read_fd(gw.w, C.int(f.Fd()), C.uint64_t(pos), C.uint64_t(math.MaxUint64), &got)
				if _, err := f.Seek(pos+int64(got), io.SeekStart); err != nil && rc == 0 {
					return int64(got), err
				}
				if rc != 0 {
					return int64(got), gw.fail(rc)
				}
				return int64(got), nil
			}
		}
	}
	if ra, ok := positionedReader(r); ok {
		if pos, err := ra.Seek(0, io.SeekCurrent); err == nil {
			end, err := ra.Seek(0, io.SeekEnd)
			if err == nil && end >= pos {
				rd := &readerAt{r: ra}
				h := cgo.NewHandle(rd)
				var got C.uint64_t
				rc := C.writer_read_at(gw.w, C.uintptr_t(h), C.uint64_t(pos), C.uint64_t(end-pos), &got)
				h.Delete()
				if _, err := ra.Seek(pos+int64(got), io.SeekStart); err != nil && rc == 0 {
					return int64(got), err
				}
				if rc == C.GLFSX_E_IO && rd.err != nil {
					return int64(got), rd.err // io.Copy returns the reader's error
				}
				if rc != 0 {
					return int64(got), gw.fail(rc)
				}
				return int64(got), nil
			}
		}
	}
	var total int64
	for {
		var p unsafe.Pointer
		var room C.uint64_t
		if rc := C.glfsx_writer_reserve(gw.w, &p, &room); rc != 0 {
			return total, gw.fail(rc)
		}
		n, err := r.Read(unsafe.Slice((*byte)(p), int(room)))
		if rc := C.glfsx_writer_commit(gw.w, C.uint64_t(n)); rc != 0 {
			return total + int64(n), gw.fail(rc)
		}
		total += int64(n)
		if err == io.EOF {
			return total, nil
		}
		if err != nil {
			return total, err
		}
	}
}

// readerAt is the io.ReaderAt behind one glfsx_writer_read_at call.
type readerAt struct {
	r   io.ReaderAt
	err error
	mu  sync.Mutex
}

//export goReadAt
func goReadAt(ctx C.uintptr_t, buf unsafe.Pointer, n C.uint64_t, off C.uint64_t) C.int64_t {
	ra := cgo.Handle(ctx).Value().(*readerAt)
	k, err := ra.r.ReadAt(unsafe.Slice((*byte)(buf), int(n)), int64(off))
	if k > 0 {
		return C.int64_t(k) // a short count with io.EOF: the next call returns 0
	}
	if err == nil || err == io.EOF {
		return 0
	}
	ra.mu.Lock()
	ra.err = err
	ra.mu.Unlock()
	return -5 // EIO: glfsx_writer_read_at returns GLFSX_E_IO
}

// Finish mirrors blob.go:135-150.
func (gw *gpuWriter) Finish(ctx context.Context) (*Root, error) {
	gw.ctx = ctx
	defer gw.close()
	var r C.glfsx_root
	if rc := C.glfsx_writer_finish(gw.w, &r); rc != 0 {
		return nil, gw.fail(rc)
	}
	ref, err := RefFromBytes(C.GoBytes(unsafe.Pointer(&r.ref[0]), 64))
	if err != nil {
		return nil, err
	}
	return &Root{Ref: *ref, Size: uint64(r.size), BlockSize: uint64(r.block_size)}, nil
}

func (gw *gpuWriter) close() {
	if gw.w != nil {
		C.glfsx_writer_free(gw.w)
		gw.w = nil
		gw.h.Delete()
	}
}

// DeriveKeyGPU is DeriveKey (ref.go:152-161) on the GPU: any len(out), any
// input length.
func DeriveKeyGPU(out []byte, salt *[32]byte, input []byte) {
	if len(out) == 0 {
		return
	}
	var in unsafe.Pointer
	if len(input) > 0 {
		in = unsafe.Pointer(&input[0])
	}
	var cerr [512]C.char
	if rc := C.derive_key((*C.uint8_t)(unsafe.Pointer(&out[0])), C.size_t(len(out)),
		(*C.uint8_t)(unsafe.Pointer(&salt[0])), in, C.size_t(len(input)),
		&cerr[0], C.size_t(len(cerr))); rc != 0 {
		panic(errors.New(C.GoString(&cerr[0]))) // DeriveKey panics too (ref.go:155,159)
	}
}

func envInt(k string, def int) int {
	v, err := strconv.Atoi(os.Getenv(k))
	if err != nil {
		return def
	}
	return v
}

func envInts(k string) []int {
	var out []int
	for _, f := range strings.Split(os.Getenv(k), ",") {
		if v, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
			out = append(out, v)
		}
	}
	return out
}
