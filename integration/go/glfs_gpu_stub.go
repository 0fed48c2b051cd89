//go:build !glfsgpu

// Without the glfsgpu build tag the batched entry points of glfs_gpu.go run
// the reference's own per-blob path, so callers compile either way.  Goes to
// gpu_stub.go of package glfs in blobcache/glfs.

package glfs

import (
	"context"

	"blobcache.io/blobcache/src/schema"
)

// PostBlobs is len(blobs) sequential PostBlob calls (machine.go:64).
func (ag *Machine) PostBlobs(ctx context.Context, s schema.WO, blobs [][]byte) ([]Ref, error) {
	return postBlobsSeq(ctx, ag, s, blobs)
}

// PostTreeMapGPU is PostTreeMap (tree.go:250-260).
func (ag *Machine) PostTreeMapGPU(ctx context.Context, s schema.WO, m map[string]Ref) (*Ref, error) {
	return ag.PostTreeMap(ctx, s, m)
}
