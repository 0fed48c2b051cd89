// Shared by both builds of the batched glfs entry points (glfs_gpu.go with
// -tags glfsgpu, glfs_gpu_stub.go without).  Goes to package glfs.

package glfs

import (
	"bytes"
	"context"

	"blobcache.io/blobcache/src/schema"
)

// postBlobsSeq is len(blobs) sequential PostBlob calls (machine.go:64): the
// reference's path, used without a GPU.
func postBlobsSeq(ctx context.Context, ag *Machine, s schema.WO, blobs [][]byte) ([]Ref, error) {
	out := make([]Ref, len(blobs))
	for i, b := range blobs {
		r, err := ag.PostBlob(ctx, s, bytes.NewReader(b))
		if err != nil {
			return nil, err
		}
		out[i] = *r
	}
	return out, nil
}
