//go:build glfsgpu

// Tests of the GPU Writer's io.Copy fast paths.  Goes to bigblob/gpu_test.go
// of blobcache/glfs next to gpu.go; run with `go test -tags glfsgpu
// ./bigblob/` on a machine with a GPU and libglfsx.

package bigblob

import (
	"bytes"
	"context"
	"io"
	"math/rand"
	"os"
	"path/filepath"
	"sync/atomic"
	"testing"

	"blobcache.io/blobcache/src/blobcache"
	"blobcache.io/blobcache/src/schema"
	"github.com/stretchr/testify/require"
)

// io.Copy(w, f) with an *os.File source reaches gpuWriter.ReadFrom through
// f.WriteTo's fileWithoutWriteTo wrapper (Go >= 1.22): the pread route must
// still be taken, and the root must be the one the plain Write route gives.
func TestCreateFromFileTakesFdRoute(t *testing.T) {
	if gpuDeviceCount() == 0 {
		t.Skip("no GPU")
	}
	ctx := context.Background()
	const maxSize = 1 << 20
	data := make([]byte, 5*maxSize+333)
	rand.New(rand.NewSource(1)).Read(data)
	p := filepath.Join(t.TempDir(), "blob")
	require.NoError(t, os.WriteFile(p, data, 0o600))

	ag := NewMachine()
	want, err := ag.Create(ctx, schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize),
		nil, bytes.NewReader(data))
	require.NoError(t, err)

	f, err := os.Open(p)
	require.NoError(t, err)
	defer f.Close()
	_, err = f.Seek(0, io.SeekStart)
	require.NoError(t, err)
	before := atomic.LoadUint64(&fdRouteReads)
	got, err := ag.Create(ctx, schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize),
		nil, f)
	require.NoError(t, err)
	require.Equal(t, before+1, atomic.LoadUint64(&fdRouteReads), "pread route not taken")
	require.Equal(t, want.Ref, got.Ref)
	require.Equal(t, uint64(len(data)), got.Size)
	pos, err := f.Seek(0, io.SeekCurrent)
	require.NoError(t, err)
	require.Equal(t, int64(len(data)), pos) // io.Copy leaves the file at its end
}

// upperFile embeds *os.File and overrides Read: it has every method the
// pread route uses (Fd, Stat, Seek, ReadAt), but its bytes are the file's
// transformed by Read, so ReadFrom must take the generic Read route
// (ADVICE r5).
type upperFile struct{ *os.File }

func (u upperFile) Read(p []byte) (int, error) {
	n, err := u.File.Read(p)
	for i := range p[:n] {
		p[i] ^= 0x5a
	}
	return n, err
}

func TestCreateFromFileWrapperUsesItsRead(t *testing.T) {
	if gpuDeviceCount() == 0 {
		t.Skip("no GPU")
	}
	ctx := context.Background()
	const maxSize = 1 << 20
	data := make([]byte, 3*maxSize+77)
	rand.New(rand.NewSource(2)).Read(data)
	p := filepath.Join(t.TempDir(), "blob")
	require.NoError(t, os.WriteFile(p, data, 0o600))
	xored := make([]byte, len(data))
	for i, b := range data {
		xored[i] = b ^ 0x5a
	}

	ag := NewMachine()
	want, err := ag.Create(ctx, schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize),
		nil, bytes.NewReader(xored))
	require.NoError(t, err)

	f, err := os.Open(p)
	require.NoError(t, err)
	defer f.Close()
	before := atomic.LoadUint64(&fdRouteReads)
	got, err := ag.Create(ctx, schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize),
		nil, upperFile{f})
	require.NoError(t, err)
	require.Equal(t, before, atomic.LoadUint64(&fdRouteReads), "pread route bypassed Read")
	require.Equal(t, want.Ref, got.Ref)
}

// A blob below GLFSX_GPU_MIN_BYTES (and below one block) never reaches the
// GPU: the reference's Go path posts it, with the root the GPU path gives
// for the same bytes; a blob at the threshold starts the library's writer.
func TestSmallBlobStaysOnGoPath(t *testing.T) {
	if gpuDeviceCount() == 0 {
		t.Skip("no GPU")
	}
	ctx := context.Background()
	const maxSize = 1 << 20
	ag := NewMachine()
	for _, n := range []int{0, 1, 4096, gpuMinBytes - 1, gpuMinBytes, 3*maxSize + 5} {
		data := make([]byte, n)
		rand.New(rand.NewSource(int64(n))).Read(data)
		before := atomic.LoadUint64(&gpuStarts)
		got, err := ag.Create(ctx, schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize),
			nil, bytes.NewReader(data))
		require.NoError(t, err)
		started := atomic.LoadUint64(&gpuStarts) - before
		if n < gpuMinBytes {
			require.Equal(t, uint64(0), started, "blob of %d bytes reached the GPU", n)
		} else {
			require.Equal(t, uint64(1), started, "blob of %d bytes did not reach the GPU", n)
		}
		// the same bytes written in pieces: same root either way
		w := ag.NewWriter(schema.NewMem(blobcache.HashAlgo_BLAKE3_256.HashFunc(), maxSize), nil)
		for off := 0; off < n; off += 1000 {
			end := off + 1000
			if end > n {
				end = n
			}
			_, err := w.Write(data[off:end])
			require.NoError(t, err)
		}
		got2, err := w.Finish(ctx)
		require.NoError(t, err)
		require.Equal(t, got.Ref, got2.Ref)
		require.Equal(t, uint64(n), got.Size)
	}
}
