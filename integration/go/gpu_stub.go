//go:build !glfsgpu

// Without the glfsgpu build tag the bigblob write path is the reference's
// own Go code: newGPUWriter returns nil and blob.go's Writer runs unchanged.
// Goes to bigblob/gpu_stub.go of blobcache/glfs (see bigblob_gpu.patch).

package bigblob

import (
	"context"
	"io"

	"blobcache.io/blobcache/src/bcsdk"
)

type gpuWriter struct{ ctx context.Context }

func (gw *gpuWriter) started() bool                            { panic("unreachable") }
func (gw *gpuWriter) write(*[]byte, []byte) (int, error)       { panic("unreachable") }
func (gw *gpuWriter) readFrom(*[]byte, io.Reader) (int64, error) { panic("unreachable") }
func (gw *gpuWriter) Write([]byte) (int, error)                { panic("unreachable") }
func (gw *gpuWriter) ReadFrom(io.Reader) (int64, error)        { panic("unreachable") }
func (gw *gpuWriter) Finish(context.Context) (*Root, error)    { panic("unreachable") }

func (ag *Machine) newGPUWriter(bcsdk.WO, *[32]byte, int) *gpuWriter { return nil }
