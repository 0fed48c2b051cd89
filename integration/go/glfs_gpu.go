//go:build glfsgpu

// Batched glfs entry points on MI355X (BASELINE config 4: 1M x 4 KiB blobs
// under a wide tree).  Goes to gpu.go of package glfs in blobcache/glfs,
// beside bigblob/gpu.go.  Without the glfsgpu tag, glfs_gpu_stub.go gives
// the same functions over the reference's own per-blob path.
//
//   PostBlobs(ctx, s, blobs)       = len(blobs) sequential PostBlob calls
//                                    (machine.go:64), one glfsx_post_blobs call
//   PostTreeMapGPU(ctx, s, m)      = PostTreeMap (tree.go:250-260) for a flat
//                                    map, the JSON lines encoded by
//                                    glfsx_tree_encode on host cores

package glfs

/*
#cgo LDFLAGS: -lglfsx
#include <stdint.h>
#include <string.h>
#include "glfsx.h"

extern int goPostBlobs(uintptr_t ctx, int kind, uint8_t *ref, void *ctext, uint64_t len);
static int post_blobs_tramp(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                            uint64_t len) {
	return goPostBlobs((uintptr_t)ctx, kind, (uint8_t *)ref, (void *)ctext, len);
}
// The handle travels as an integer and becomes void * on the C side only.
static int post_blobs(uint64_t bs, uint64_t max, const uint8_t *salt, const void *data,
                      const uint64_t *offs, const uint64_t *lens, uint64_t n, uintptr_t h,
                      uint8_t *roots, char *err, size_t cap) {
	int rc = glfsx_post_blobs(bs, max, salt, NULL, data, offs, lens, n, post_blobs_tramp,
	                          (void *)h, roots);
	if (rc) {
		strncpy(err, glfsx_last_error(), cap - 1);
		err[cap - 1] = 0;
	}
	return rc;
}
static int tree_encode(uint64_t n, const uint8_t *names, const uint64_t *name_offs,
                       const uint32_t *modes, const uint8_t *types, const uint64_t *type_offs,
                       const uint8_t *roots, const uint64_t *sizes, const uint64_t *bss,
                       uint8_t *out, uint64_t cap, uint64_t *out_len, uint64_t *ends,
                       char *err, size_t ecap) {
	int rc = glfsx_tree_encode(n, names, name_offs, modes, types, type_offs, roots, sizes,
	                           bss, out, cap, out_len, ends);
	if (rc) {
		strncpy(err, glfsx_last_error(), ecap - 1);
		err[ecap - 1] = 0;
	}
	return rc;
}
*/
import "C"

import (
	"bytes"
	"context"
	"encoding/json"
	"fmt"
	"runtime/cgo"
	"strings"
	"unsafe"

	"blobcache.io/blobcache/src/blobcache"
	"blobcache.io/blobcache/src/schema"
	"blobcache.io/glfs/bigblob"
)

// blobsSink receives the Posts of one glfsx_post_blobs call, in call order.
type blobsSink struct {
	ctx context.Context
	s   schema.WO
	err error
}

//export goPostBlobs
func goPostBlobs(ctx C.uintptr_t, kind C.int, ref *C.uint8_t, ctext unsafe.Pointer, n C.uint64_t) C.int {
	bs := cgo.Handle(ctx).Value().(*blobsSink)
	var data []byte
	if n > 0 {
		data = unsafe.Slice((*byte)(ctext), int(n)) // C memory, valid during the call
	}
	var cid blobcache.CID
	copy(cid[:], unsafe.Slice((*byte)(unsafe.Pointer(ref)), 32))
	if ps, ok := bs.s.(bigblob.PrehashedWO); ok {
		if err := ps.PostHashed(bs.ctx, cid, data); err != nil {
			bs.err = err
			return 1
		}
		return 0
	}
	got, err := bs.s.Post(bs.ctx, data) // ref.go:103: the store hashes
	if err != nil {
		bs.err = err
		return 1
	}
	if got != cid {
		bs.err = fmt.Errorf("glfsx: store CID %v != GPU CID %v", got, cid)
		return 2
	}
	return 0
}

// PostBlobs is len(blobs) sequential PostBlob calls (machine.go:64) in one
// batched GPU call (glfsx_post_blobs): the Refs are PostBlob's, and the
// store receives every Post of blob 0, then blob 1, ... exactly as the
// sequential calls would deliver them (a single-block blob is one Post; a
// larger one its data blocks and index nodes).  The first failing Post
// stops the batch and its error is returned.  Blobs of up to 16 KiB (and
// one block) are hashed one GPU lane each -- config 4's 1M x 4 KiB is one
// launch pair -- instead of a Writer and a one-shot launch per blob.
func (ag *Machine) PostBlobs(ctx context.Context, s schema.WO, blobs [][]byte) ([]Ref, error) {
	n := len(blobs)
	if n == 0 {
		return nil, nil
	}
	if C.glfsx_device_count() == 0 { // no GPU: the reference's own path
		return postBlobsSeq(ctx, ag, s, blobs)
	}
	total := 0
	for _, b := range blobs {
		total += len(b)
	}
	// one contiguous Go buffer (no Go pointers inside), passed for the call only
	data := make([]byte, total+1)
	offs := make([]uint64, n)
	lens := make([]uint64, n)
	o := 0
	for i, b := range blobs {
		offs[i], lens[i] = uint64(o), uint64(len(b))
		o += copy(data[o:], b)
	}
	roots := make([]byte, 64*n)
	sink := &blobsSink{ctx: ctx, s: s}
	h := cgo.NewHandle(sink)
	defer h.Delete()
	salt := ag.makeSalt(TypeBlob)
	var cerr [512]C.char
	rc := C.post_blobs(C.uint64_t(ag.blockSize), C.uint64_t(s.MaxSize()),
		(*C.uint8_t)(unsafe.Pointer(&salt[0])), unsafe.Pointer(&data[0]),
		(*C.uint64_t)(unsafe.Pointer(&offs[0])), (*C.uint64_t)(unsafe.Pointer(&lens[0])),
		C.uint64_t(n), C.uintptr_t(h), (*C.uint8_t)(unsafe.Pointer(&roots[0])),
		&cerr[0], C.size_t(len(cerr)))
	switch {
	case rc == 0:
	case rc == C.GLFSX_E_STORE && sink.err != nil:
		return nil, sink.err
	case rc == C.GLFSX_E_BLOCKSIZE_GT_MAX || rc == C.GLFSX_E_BLOCKSIZE_LT_MIN:
		panic(C.GoString(&cerr[0])) // blob.go:91 / :94, as NewWriter panics
	default:
		return nil, fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(&cerr[0]))
	}
	out := make([]Ref, n)
	for i := range out {
		ref, err := bigblob.RefFromBytes(roots[64*i : 64*i+64])
		if err != nil {
			return nil, err
		}
		out[i] = Ref{Type: TypeBlob, Root: bigblob.Root{Ref: *ref, Size: lens[i],
			BlockSize: uint64(ag.blockSize)}}
	}
	return out, nil
}

// PostTreeMapGPU is PostTreeMap (tree.go:250-260) for a caller holding many
// roots.  For a flat map (every cleaned name non-empty, without "/") the
// entries are sorted (tree.go:238), checked for referential integrity in
// batched Exists calls (tree.go:304, ExistsUnit per entry), their JSON lines
// encoded by glfsx_tree_encode on host cores, and the lines posted as the
// tree blob (TypedWriter(tree) over them, the GPU writer).  The lines must
// be the bytes json.Encoder.Encode writes (tree.go:309): blobcache.CID's JSON
// form is not in the reference, so the first, middle and last lines are
// compared with encoding/json's and any difference falls back to
// PostTreeMap.  A nested map (names with "/") also takes PostTreeMap.
func (ag *Machine) PostTreeMapGPU(ctx context.Context, s schema.WO, m map[string]Ref) (*Ref, error) {
	ents := make([]TreeEntry, 0, len(m))
	for k, v := range m {
		p := CleanPath(k)
		if p == "" || strings.Contains(p, "/") || C.glfsx_device_count() == 0 {
			return ag.PostTreeMap(ctx, s, m)
		}
		ents = append(ents, TreeEntry{Name: p, FileMode: getFileMode(v), Ref: v})
	}
	SortTreeEntries(ents)
	if err := checkEntries(ctx, s, ents); err != nil {
		return nil, err
	}
	lines, ends, err := encodeTreeLines(ents)
	if err != nil {
		return nil, err
	}
	for _, i := range []int{0, len(ents) / 2, len(ents) - 1} {
		if i < 0 || i >= len(ents) {
			continue
		}
		want, err := json.Marshal(ents[i]) // json.Encoder.Encode = Marshal + "\n"
		if err != nil {
			return nil, err
		}
		lo := uint64(0)
		if i > 0 {
			lo = ends[i-1]
		}
		if !bytes.Equal(lines[lo:ends[i]], append(want, '\n')) {
			return ag.PostTreeMap(ctx, s, m) // the CID JSON form differs: the Go encoder
		}
	}
	return ag.PostTyped(ctx, s, TypeTree, bytes.NewReader(lines))
}

// checkEntries is TreeWriter.Put's two checks (tree.go:300-308) for every
// entry in sorted order, one entry at a time as Put makes them: the name
// order against the previous entry, then ExistsUnit.  Existence is asked in
// batches of the store's Exists, but the first failure by entry index is
// reported, whichever check it is, so the error is Put's (ADVICE r4).
func checkEntries(ctx context.Context, s schema.WO, ents []TreeEntry) error {
	const batch = 4096
	order := func(i int) error {
		if i > 0 && ents[i].Name <= ents[i-1].Name { // tree.go:301-303
			return fmt.Errorf("cannot write tree entries out of order %q <= %q",
				ents[i].Name, ents[i-1].Name)
		}
		return nil
	}
	cids := make([]blobcache.CID, 0, batch)
	yes := make([]bool, batch)
	for i0 := 0; i0 < len(ents); i0 += batch {
		i1 := min(i0+batch, len(ents))
		cids = cids[:0]
		for _, e := range ents[i0:i1] {
			cids = append(cids, e.Ref.CID)
		}
		if err := s.Exists(ctx, cids, yes[:len(cids)]); err != nil {
			if oerr := order(i0); oerr != nil { // Put checks the order first
				return oerr
			}
			return err // Put's first ExistsUnit fails the same way
		}
		for k, ok := range yes[:len(cids)] {
			if err := order(i0 + k); err != nil {
				return err
			}
			if !ok { // tree.go:304-308
				return fmt.Errorf("adding tree ent %v would violate referential integrity",
					ents[i0+k])
			}
		}
	}
	return nil
}

// encodeTreeLines runs glfsx_tree_encode over the sorted entries: the lines
// and each line's end offset.
func encodeTreeLines(ents []TreeEntry) ([]byte, []uint64, error) {
	n := len(ents)
	if n == 0 {
		return nil, nil, nil
	}
	var names, types []byte
	nameOffs := make([]uint64, n+1)
	typeOffs := make([]uint64, n+1)
	modes := make([]uint32, n)
	roots := make([]byte, 64*n)
	sizes := make([]uint64, n)
	bss := make([]uint64, n)
	for i, e := range ents {
		names = append(names, e.Name...)
		nameOffs[i+1] = uint64(len(names))
		types = append(types, string(e.Ref.Type)...)
		typeOffs[i+1] = uint64(len(types))
		modes[i] = uint32(e.FileMode)
		copy(roots[64*i:], e.Ref.CID[:])
		copy(roots[64*i+32:], e.Ref.DEK[:])
		sizes[i], bss[i] = e.Ref.Size, e.Ref.BlockSize
	}
	names = append(names, 0) // never empty: &names[0] is valid
	types = append(types, 0)
	ends := make([]uint64, n)
	var total C.uint64_t
	var cerr [512]C.char
	call := func(out []byte) C.int {
		var p *C.uint8_t
		if len(out) > 0 {
			p = (*C.uint8_t)(unsafe.Pointer(&out[0]))
		}
		return C.tree_encode(C.uint64_t(n), (*C.uint8_t)(unsafe.Pointer(&names[0])),
			(*C.uint64_t)(unsafe.Pointer(&nameOffs[0])), (*C.uint32_t)(unsafe.Pointer(&modes[0])),
			(*C.uint8_t)(unsafe.Pointer(&types[0])), (*C.uint64_t)(unsafe.Pointer(&typeOffs[0])),
			(*C.uint8_t)(unsafe.Pointer(&roots[0])), (*C.uint64_t)(unsafe.Pointer(&sizes[0])),
			(*C.uint64_t)(unsafe.Pointer(&bss[0])), p, C.uint64_t(len(out)), &total,
			(*C.uint64_t)(unsafe.Pointer(&ends[0])), &cerr[0], C.size_t(len(cerr)))
	}
	if rc := call(nil); rc != 0 { // the length
		return nil, nil, fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(&cerr[0]))
	}
	out := make([]byte, int(total))
	if rc := call(out); rc != 0 {
		return nil, nil, fmt.Errorf("glfsx %d: %s", int(rc), C.GoString(&cerr[0]))
	}
	return out, ends, nil
}
