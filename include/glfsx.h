/*
 * glfsx.h -- C-ABI of the MI355X-native GLFS bigblob write path.
 *
 * This is the drop-in boundary: plain pointers and sizes, no torch or HIP types
 * in the signatures (device pointers and streams travel as void*).  A Go
 * maintainer binds it with cgo; the Python mirror in
 * glfs_amd/ binds it with ctypes.  Every compute entry point runs on the GPU
 * (hand-written gfx950 HIP kernels); there is no CPU fallback -- without a
 * usable HIP device every call fails with GLFSX_E_DEVICE.
 *
 * Reference interfaces replaced (reference = blobcache/glfs, Go):
 *   glfsx_derive_key       bigblob/ref.go:152-161  DeriveKey(out, salt, input)
 *   glfsx_post             bigblob/ref.go:98-111   (*Machine).post, one message,
 *                          minus the store.Post call
 *   glfsx_post_batch*,     bigblob/ref.go:98-111   (*Machine).post, batched over
 *   glfsx_dek/cid_batch_device
 *                          equal-size blocks, minus the store.Post call
 *                          (ref.go:103), which stays with the caller
 *   glfsx_writer_*         bigblob/blob.go:71-206  Writer: NewWriter/Write/
 *                          Finish (postBuf/addRef/finishIndexes inside)
 *   glfsx_create           bigblob/blob.go:209-217 (*Machine).Create
 *   glfsx_create_device    Create over a device-resident blob (no host copies)
 *   glfsx_shard_device /   the same, split by disjoint block ranges across
 *   glfsx_root_from_level1 GPUs; the caller gathers the level-1 refs
 *   glfsx_post_blobs*      glfs machine.go:64 PostBlob, batched over many
 *                          single-block blobs (tree.go:300-316 callers)
 *   glfsx_depth            bigblob/blob.go:256-264 depth()
 *   glfsx_tree_encode      tree.go:300-316 TreeWriter.Put's JSON lines, batched
 *   glfsx_store_*          the store under ref.go:103 (bcsdk.WO / MemStore [ext])
 *                          with a pre-hashed Post that takes the GPU CID
 *   glfsx_chacha20_xor*    bigblob/ref.go:137-144  cryptoXOR (read side decrypt)
 *
 * Conventions:
 *   - 0 = ok, negative = status; glfsx_last_error() gives a thread-local text.
 *   - Where the reference panics (blob.go:91,94; ref.go:130) the C side returns
 *     GLFSX_E_BLOCKSIZE_GT_MAX / GLFSX_E_BLOCKSIZE_LT_MIN / GLFSX_E_ARG and the
 *     binding re-panics; store failures come back as GLFSX_E_STORE with the
 *     sink's code in glfsx_last_error().
 *   - The caller owns every buffer; nothing is retained after return (cgo rule).
 *   - Reentrant: each host thread gets its own HIP stream and staging buffers
 *     for the one-shot calls; glfsx_set_device() selects the GPU for the
 *     calling thread.  A writer owns its streams, staging, device and error
 *     text, so consecutive calls on one writer may come from different
 *     threads (a goroutine migrating between OS threads); one call at a time.
 *   - A thread waiting for a one-shot post (glfsx_post, glfsx_create of a
 *     small blob, a Writer's tail) either polls or, past half the host's
 *     threads, sleeps between polls; while it sleeps in that wait its timer
 *     slack is 1 us (prctl PR_SET_TIMERSLACK), and the thread's own slack
 *     is restored before the call returns.
 *   - glfsx_last_error() is thread-local: read it in the same C call that
 *     failed (a cgo binding does so in its C preamble), or use
 *     glfsx_writer_error() for writer calls.
 *   - Ref layout (ref.go:77-82): 64 bytes = CID[32] || DEK[32].
 */
#ifndef GLFSX_H
#define GLFSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLFSX_REF_SIZE 64   /* ref.go:52 RefSize = CIDSize + DEKSize */
#define GLFSX_CID_SIZE 32
#define GLFSX_DEK_SIZE 32   /* ref.go:16 */
#define GLFSX_MIN_BLOCK_SIZE 128 /* blob.go:93: 2*maxRefSize */

enum {
  GLFSX_OK = 0,
  GLFSX_E_BLOCKSIZE_GT_MAX = -1, /* blob.go:90-92 panic */
  GLFSX_E_BLOCKSIZE_LT_MIN = -2, /* blob.go:93-95 panic */
  GLFSX_E_STORE = -3,            /* store.Post returned an error */
  GLFSX_E_DEVICE = -4,           /* no HIP device / HIP runtime error */
  GLFSX_E_ARG = -5,              /* invalid argument */
  GLFSX_E_UNSUPPORTED = -6,      /* e.g. block size above the kernels' limit */
  GLFSX_E_NOMEM = -7,
  GLFSX_E_IO = -8                /* the input's read failed (io.Copy's read error) */
};

/* bigblob/blob.go:17-21 Root{Ref, Size, BlockSize} */
typedef struct glfsx_root {
  uint8_t ref[GLFSX_REF_SIZE];
  uint64_t size;
  uint64_t block_size;
} glfsx_root;

/* store.Post(ctx, ctext) (ref.go:103).  Called once per posted blob in the
 * reference's Post order (data blocks and index nodes interleaved exactly as
 * blob.go:152-206 does).  `ref` is the GPU-computed CID||DEK; a parity-mode
 * binding compares the store's returned CID with ref[0:32].  kind: 0 = data
 * block, 1 = index node.  Return 0, or nonzero to abort the write with
 * GLFSX_E_STORE. */
typedef int (*glfsx_post_fn)(void *ctx, int kind, const uint8_t *ref,
                             const void *ctext, uint64_t len);

/* --- runtime ----------------------------------------------------------- */
const char *glfsx_last_error(void);
int glfsx_device_count(void);
int glfsx_set_device(int dev);      /* for the calling thread */
const char *glfsx_version(void);
/* Tuning (no reference counterpart): a hashing launch of fewer than `wgs`
 * 256-lane workgroups spreads each block over up to 64 workgroups plus a
 * merge launch (index nodes, 1-2 GiB blobs, Writer batches).  0 disables
 * it; the default is 2048.  Results are identical either way.  Returns the
 * previous value; process-wide. */
uint32_t glfsx_set_split_target(uint32_t wgs);
/* Tuning (no reference counterpart): launches of at most `wgs` workgroups
 * (default 512, i.e. <= 2 waves per SIMD) use the latency-mode kernels
 * (compiler-scheduled ARX; CID as keystream launch + BLAKE3 pass).  Results
 * are identical either way.  Returns the previous value; process-wide. */
uint32_t glfsx_set_latency_wgs(uint32_t wgs);

/* Test hooks (no reference counterpart).  A split-mode post of many
 * workgroups runs both passes in one launch, each CID work item waiting for
 * its block's DEK; a wait that exceeds its bound fails the launch loudly:
 * the calls that synchronise repeat the post with two launches (Create,
 * post_batch, the Writer) and count it.
 * glfsx_debug_fused makes the next such launch leave block skip_msg's DEK
 * unpublished (~0u: none) and sets the
 * bound to wait_us microseconds (0: the default, 1 s).  Returns the number
 * of failed one-launch posts seen so far, process-wide. */
uint64_t glfsx_debug_fused(uint32_t skip_msg, uint64_t wait_us);
/* Measurement hook (no reference counterpart): the number of failed
 * one-launch split posts seen so far, process-wide -- each one was discarded
 * and re-run with two launches.  Reads a counter and nothing else (unlike
 * glfsx_debug_fused, it leaves the skip / bound state alone); bench.py
 * prints its delta over every timed leg as `fused_reruns`. */
uint64_t glfsx_fused_failures(void);
/* Test hook (no reference counterpart): the next one-shot launch (the
 * coalesced launch behind a single-block Create / PostBlob and the few-block
 * and medium-blob batches) withholds the result flag of its request k, as a
 * launch that failed on the device would; the waiting call fails with
 * GLFSX_E_DEVICE once that launch has completed.  ~0u: none. */
void glfsx_debug_one_drop(uint32_t k);

/* Measurement hook (no reference counterpart): the bulk hashing passes
 * (one workgroup per block) add each workgroup's lifetime in shader-clock
 * cycles (out[0]) and in 100 MHz real-time ticks (out[1]) to two counters
 * on the device; out[0] / out[1] x 0.1 GHz is the clock the chip held over
 * the launches since the last reset (bench.py's VALU roofline).  Reads the
 * calling thread's device, waiting for it; reset != 0 zeroes the counters
 * after reading.  out may be NULL. */
int glfsx_clock_probe(int reset, uint64_t out[2]);

/* Measurement hook (no reference counterpart): the one-shot poster's
 * process-wide counters since the last reset -- out[0] launches, out[1]
 * requests they carried (out[1] / out[0] = the mean group-commit batch),
 * out[2] times a leader found every launch lane busy.  reset != 0 zeroes
 * them after reading.  out may be NULL. */
int glfsx_one_stats(int reset, uint64_t out[3]);

/* --- primitives -------------------------------------------------------- */
/* ref.go:152 DeriveKey: BLAKE3 keyed with salt over input (any length),
 * the first out_len bytes of the XOF (any length; blake3.New(len(out), salt)
 * then h.XOF() and io.ReadFull).  out_len 0 writes nothing. */
int glfsx_derive_key(uint8_t *out, size_t out_len, const uint8_t salt[32],
                     const void *input, size_t n);

/* ref.go:98-111 (*Machine).post of ONE message of n bytes (n may be 0: the
 * empty blob's post(indexSalt, nil), blob.go:187-189), host buffers, minus
 * the store.Post call: writes the 64-byte ref (CID||DEK) and, if ctext_out is
 * non-NULL, the n bytes of ctext.  cid_key as for glfsx_post_batch. */
int glfsx_post(const uint8_t salt[32], const void *ptext, uint64_t n,
               void *ctext_out, uint8_t *ref_out, const uint8_t *cid_key);

/* ref.go:98 post() for ceil(total/block_size) blocks of `ptext` (the last one
 * short), host buffers.  refs_out: 64 bytes per block.  ctext_out nullable.
 * cid_key: NULL = CID is unkeyed BLAKE3-256(ctext) (blobcache MemStore with
 * a nil salt); non-NULL = keyed with cid_key. */
int glfsx_post_batch(const uint8_t salt[32], const void *ptext, uint64_t total,
                     uint64_t block_size, void *ctext_out, uint8_t *refs_out,
                     const uint8_t *cid_key);

/* Same, device-resident: d_* are device pointers on the current device;
 * enqueued on `stream` (hipStream_t, NULL = the thread's stream); returns
 * without synchronising.  d_ctext nullable; may equal d_ptext (in place). */
int glfsx_post_batch_device(const uint8_t salt[32], const void *d_ptext,
                            uint64_t total, uint64_t block_size, void *d_ctext,
                            void *d_refs, const uint8_t *cid_key, void *stream);

/* The two kernels of glfsx_post_batch_device, separately (profiling and
 * pipelining): the DEK pass writes DEKs to bytes [32,64) of each ref slot;
 * the ChaCha20 + CID pass reads them, writes ctext (nullable) and the CIDs to
 * bytes [0,32).  Same stream semantics as glfsx_post_batch_device. */
int glfsx_dek_batch_device(const uint8_t salt[32], const void *d_ptext,
                           uint64_t total, uint64_t block_size, void *d_refs,
                           void *stream);
int glfsx_cid_batch_device(const void *d_ptext, uint64_t total,
                           uint64_t block_size, void *d_ctext, void *d_refs,
                           const uint8_t *cid_key, void *stream);

/* --- bigblob Writer (blob.go:71-206) ------------------------------------ */
typedef struct glfsx_writer glfsx_writer;

/* blob.go:85-114.  block_size 0 = store_max (bigblob machine.go:22-30);
 * salt NULL = 0^32 (blob.go:96-98).  On error returns NULL, *err set. */
glfsx_writer *glfsx_writer_new(uint64_t block_size, uint64_t store_max,
                               const uint8_t *salt, const uint8_t *cid_key,
                               glfsx_post_fn post, void *post_ctx, int *err);
/* blob.go:120-133.  Data blocks are hashed in pipelined batches: by default
 * a store error is returned by the Write or Finish call whose batch contained
 * the failure (Posts are still delivered in the reference's order, and none
 * after the failing one).  In strict mode (glfsx_writer_set_strict) every
 * Write returns only after the Posts of all blocks it completed were
 * delivered, so the error comes from the Write that filled the failing block,
 * exactly as blob.go:120-133 returns it. */
int glfsx_writer_write(glfsx_writer *w, const void *data, size_t n);
/* blob.go:120-133 Write of n bytes already in device memory (current
 * device): a GPU producer feeds the Writer without a host round trip.
 * Ordered after the work already enqueued on `stream` (NULL: d_data is
 * ready now and the call returns once it has been consumed); work enqueued
 * on `stream` after the call may reuse d_data. */
int glfsx_writer_write_device(glfsx_writer *w, const void *d_data, size_t n,
                              void *stream);
/* Write the plaintext of a blob's data blocks given as ciphertext: block j
 * of ctext (host memory, block_size bytes, the last one short,
 * block_size % 64 == 0) is decrypted on the GPU with the DEK in bytes
 * [32,64) of refs[64 j] (ref.go:113-126 getF) and the plaintext goes into
 * the Writer without leaving the device -- blob.go:333-345 Concat's read
 * side fused with its Writer. */
int glfsx_writer_write_ctext(glfsx_writer *w, const void *ctext, uint64_t total,
                             uint64_t block_size, const uint8_t *refs);
/* The same with the ciphertext blocks at scattered addresses (nblocks =
 * ceil(total / block_size); block j at blocks[j], block_size bytes, the last
 * one short): Concat straight from a store's memory, each 64 MiB slab of
 * blocks gathered into pinned staging by the copy threads while the previous
 * one uploads and decrypts. */
int glfsx_writer_write_ctext_blocks(glfsx_writer *w, const void *const *blocks,
                                    uint64_t nblocks, uint64_t total, uint64_t block_size,
                                    const uint8_t *refs);
/* A Writer's io.ReaderFrom (no reference counterpart; io.Copy in Create and
 * Concat, blob.go:213,341, uses it when the Writer has it): reserve lends
 * the caller the next *cap >= 1 bytes of the writer's pinned staging at
 * *buf, the caller reads up to that many bytes of input into it (r.Read),
 * and commit(n) takes the first n as if glfsx_writer_write(buf, n) had been
 * called -- the input is copied once, by the reader, instead of into a
 * 32 KiB buffer and again into staging.  No other call on the writer
 * between the two; the area is the writer's again after commit. */
int glfsx_writer_reserve(glfsx_writer *w, void **buf, uint64_t *cap);
int glfsx_writer_commit(glfsx_writer *w, uint64_t n);
/* io.Copy(w, r) (blob.go:213, glfs.go:53) when r is an io.ReaderAt -- an
 * *os.File or *io.SectionReader (bigblob.Create's caller feeding a file): the
 * input is read straight into the writer's pinned staging by several threads
 * at once, each a >= 4 MiB piece of the batch being filled, while earlier
 * batches upload, hash and download (one host core's page-cache copy is the
 * limit of a single reader).  n bytes from input offset `offset` (UINT64_MAX:
 * to the end of the input); *got = bytes taken.  The Posts, index and root
 * are glfsx_writer_write's of the same bytes, in block order.
 *   read_at(ctx, buf, len, off): io.ReaderAt.ReadAt -- read up to len bytes
 *   at input offset off into buf; return the count (> 0), 0 at the end of
 *   the input, or negative on error.  Called from several threads at once,
 *   on disjoint ranges.
 * A failed read returns GLFSX_E_IO with *got = the bytes taken before it
 * (the writer stays usable, as after io.Copy's read error); glfsx_writer_read_fd
 * is the same over pread(2) of a file descriptor (its file offset unused). */
typedef int64_t (*glfsx_read_at_fn)(void *ctx, void *buf, uint64_t len, uint64_t off);
int glfsx_writer_read_at(glfsx_writer *w, glfsx_read_at_fn read_at, void *ctx,
                         uint64_t offset, uint64_t n, uint64_t *got);
int glfsx_writer_read_fd(glfsx_writer *w, int fd, uint64_t offset, uint64_t n,
                         uint64_t *got);
/* io.Copy(w, r) (blob.go:213, glfs.go:53) from an in-memory reader: n bytes
 * in glfsx_writer_write calls of `piece` bytes each (io.Copy's 32 KiB
 * buffer for a reader without WriterTo), stopping at the first error. */
int glfsx_writer_copy(glfsx_writer *w, const void *data, uint64_t n, uint64_t piece);
/* Deliver the Posts of every complete block written so far (no reference
 * counterpart: the reference never holds a complete block back). */
int glfsx_writer_flush(glfsx_writer *w);
/* Hash this writer's batches on several GPUs (no reference counterpart:
 * one bigblob.Writer fed from one io.Reader): batch k of
 * complete blocks runs on devs[k % ndev], each device with its own streams
 * and pinned staging (one PCIe link each); Posts and the index build still
 * replay in block order (blob.go:152-206), so the Post log and root are
 * those of the one-device writer.  Call before the first write.  Index
 * nodes and the tail block stay on the writer's own device; the device-input
 * calls (write_device / write_ctext) need a one-device writer. */
int glfsx_writer_set_devices(glfsx_writer *w, const int *devs, int ndev);
/* strict != 0: blob.go:120-133 error timing (see glfsx_writer_write). */
int glfsx_writer_set_strict(glfsx_writer *w, int strict);
/* Text of the last failed call on this writer (any thread). */
const char *glfsx_writer_error(const glfsx_writer *w);
/* blob.go:135-150 */
int glfsx_writer_finish(glfsx_writer *w, glfsx_root *out);
void glfsx_writer_free(glfsx_writer *w);

/* blob.go:209-217 Create over an in-memory (host) blob. */
int glfsx_create(uint64_t block_size, uint64_t store_max, const uint8_t *salt,
                 const uint8_t *cid_key, const void *data, uint64_t size,
                 glfsx_post_fn post, void *post_ctx, glfsx_root *out);

/* Create over a device-resident blob: every data block and index node is
 * posted on the GPU; ctext of the data blocks goes to d_ctext (nullable,
 * same layout as d_data).  No store callbacks; returns the root.  Writes the
 * number of posted blobs into *n_posts (nullable). Synchronises `stream`. */
int glfsx_create_device(uint64_t block_size, const uint8_t *salt,
                        const uint8_t *cid_key, const void *d_data,
                        uint64_t size, void *d_ctext, glfsx_root *out,
                        uint64_t *n_posts, void *stream);

/* Create over a blob whose bytes lie on several devices, in one process
 * (SURVEY 8e): the blob is the concatenation of nparts parts, part k of
 * part_sizes[k] bytes at device pointer d_parts[k] on device devs[k] (a
 * device may appear more than once).  Every part but the last must hold
 * whole level-1 nodes (a positive multiple of block_size * block_size/64
 * bytes: 16 GiB at 1 MiB blocks); the last is non-empty.  Each part's data
 * blocks and level-1 index nodes are posted on its device, all parts at
 * once (one host worker thread per part); the level-1 refs are gathered on
 * the host and the levels above posted on devs[0].  d_ctexts (nullable, or
 * entries NULL): ctext of part k, same layout as d_parts[k].  level1_out
 * (nullable): with nparts > 1, the ceil(n0/bf) level-1 refs (64 B each).
 * Calls are serialised.  Same root as glfsx_create_device over the whole
 * blob. */
int glfsx_create_devices(uint64_t block_size, const uint8_t *salt,
                         const uint8_t *cid_key, int nparts, const int *devs,
                         const void *const *d_parts, const uint64_t *part_sizes,
                         void *const *d_ctexts, uint8_t *level1_out,
                         glfsx_root *out, uint64_t *n_posts);

/* GPU time of the last glfsx_create_devices call (no reference
 * counterpart; measurement): ms[k] = part k's data blocks and level-1 nodes
 * on its device (HIP events on the stream that ran them), then one entry for
 * the levels above on devs[0] (with nparts > 1).  Writes min(count, cap)
 * entries and returns the count (-1 = not timed). */
int glfsx_create_devices_ms(float *ms, int cap);

/* Multi-GPU shard: posts blocks [first_block, first_block + nb)
 * of a blob of `size` bytes whose bytes for that range are at d_range, plus
 * the level-1 index nodes covering them.  first_block must be a multiple of
 * bf = block_size/64.  Writes ceil(nb/bf) level-1 refs (64 B each) to
 * level1_out (host).  Enqueued on stream and synchronised. */
int glfsx_shard_device(uint64_t block_size, const uint8_t *salt,
                       const uint8_t *cid_key, const void *d_range,
                       uint64_t size, uint64_t first_block, uint64_t nb,
                       void *d_ctext, uint8_t *level1_out, void *stream);
/* Combine the gathered level-1 refs of a blob with n0 > bf data blocks into
 * its root (levels >= 2 posted on the GPU). */
int glfsx_root_from_level1(uint64_t block_size, const uint8_t *salt,
                           const uint8_t *cid_key, const uint8_t *level1,
                           uint64_t n1, uint64_t size, glfsx_root *out);

/* --- many small blobs (glfs.PostBlob batched; BASELINE config 4) -------- */
/* n sequential glfs.PostBlob calls (machine.go:64) in one call: blob i is
 * data[offsets[i] .. offsets[i]+lengths[i]).  A blob of at most one block
 * has root post(rawSalt, blob) (blob.go:190-193), the empty blob
 * post(indexSalt, "") (blob.go:187-189); rawSalt / indexSalt derive from
 * `salt` (glfs: the type salt, machine.go:50-54).  Blobs of <= 16 KiB are
 * hashed one lane each in one launch pair; larger ones (any size, several
 * blocks included) go through the Writer.  Writes the 64-byte root ref
 * (CID||DEK) per blob; `post` is called for every Post of blob 0, then blob
 * 1, ... exactly as n sequential PostBlob calls would. */
int glfsx_post_blobs(uint64_t block_size, uint64_t store_max, const uint8_t *salt,
                     const uint8_t *cid_key, const void *data,
                     const uint64_t *offsets, const uint64_t *lengths, uint64_t n,
                     glfsx_post_fn post, void *post_ctx, uint8_t *roots_out);
/* Device-resident: d_offsets / d_lengths are device arrays; max_len is the
 * largest length (caller-known; when it exceeds 16 KiB the lengths are read
 * back and the larger blobs posted one by one, synchronising the stream).
 * Enqueued on stream. */
int glfsx_post_blobs_device(uint64_t block_size, const uint8_t *salt,
                            const uint8_t *cid_key, const void *d_data,
                            const uint64_t *d_offsets, const uint64_t *d_lengths,
                            uint64_t n, uint64_t max_len, void *d_ctext,
                            void *d_roots, void *stream);

/* --- tree blobs (tree.go:284-320; BASELINE config 4) -------------------- */
/* TreeWriter.Put's json.Encoder.Encode(TreeEntry) (tree.go:300-316) for n
 * entries at once, on host cores: line i =
 *   {"name":N,"mode":M,"ref":{"type":T,"cid":"<hex>","dek":"<hex>",
 *    "size":S,"blockSize":B}}\n
 * with encoding/json's string escaping (HTML-safe, invalid UTF-8 as \ufffd).
 * names / types: concatenated bytes, name_offs / type_offs: n+1 offsets;
 * roots: 64-byte CID||DEK per entry.  The cid field is written as a hex
 * string (blobcache.CID's JSON form is not in the reference: parity
 * unpinned).  Writes the lines to out (nullable: length only) and the total
 * length to *out_len; line_ends (nullable) receives each line's end offset. */
int glfsx_tree_encode(uint64_t n, const uint8_t *names, const uint64_t *name_offs,
                      const uint32_t *modes, const uint8_t *types,
                      const uint64_t *type_offs, const uint8_t *roots,
                      const uint64_t *sizes, const uint64_t *block_sizes,
                      uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                      uint64_t *line_ends);

/* The same lines encoded on the GPU from device-resident entries (d_roots
 * typically the roots glfsx_post_blobs_device just wrote), into d_out
 * (nullable: length only; nothing is written when the lines exceed out_cap,
 * which returns GLFSX_E_ARG).  d_line_ends nullable.  Synchronises `stream`
 * to return the total length in *out_len (host). */
int glfsx_tree_encode_device(uint64_t n, const uint8_t *d_names,
                             const uint64_t *d_name_offs, const uint32_t *d_modes,
                             const uint8_t *d_types, const uint64_t *d_type_offs,
                             const uint8_t *d_roots, const uint64_t *d_sizes,
                             const uint64_t *d_block_sizes, void *d_out,
                             uint64_t out_cap, uint64_t *d_line_ends,
                             uint64_t *out_len, void *stream);

/* BASELINE config 4 in one call (tree.go:250-320 PostTreeMap over n entries
 * whose blobs are glfs.PostBlob'd, machine.go:64), device-resident: blob i
 * (d_data + d_offsets[i], d_lengths[i] bytes, block size blob_bs, salt
 * blob_salt) -> root i in d_roots (ctext to d_ctext, nullable), then entry
 * i's JSON line (glfsx_tree_encode_device's bytes; its size field is
 * d_lengths[i], its blockSize d_block_sizes[i]) into d_lines, then the tree
 * blob of those lines Create'd with tree_salt at tree_bs (ctext to
 * d_tree_ctext, nullable): *tree_root and the lines' length.  All launches
 * are queued before the host reads the lines' total (the layout first, then
 * the hashing and the lines; the tree blob's posts on a second stream); the
 * results are those of glfsx_post_blobs_device, glfsx_tree_encode_device
 * and glfsx_create_device in sequence.  Synchronises `stream`. */
int glfsx_post_tree_device(uint64_t n, uint64_t blob_bs, const uint8_t *blob_salt,
                           const uint8_t *tree_salt, const uint8_t *cid_key,
                           const void *d_data, const uint64_t *d_offsets,
                           const uint64_t *d_lengths, uint64_t max_len, void *d_ctext,
                           void *d_roots, const uint8_t *d_names,
                           const uint64_t *d_name_offs, const uint32_t *d_modes,
                           const uint8_t *d_types, const uint64_t *d_type_offs,
                           const uint64_t *d_block_sizes, uint64_t tree_bs, void *d_lines,
                           uint64_t lines_cap, void *d_tree_ctext, glfsx_root *tree_root,
                           uint64_t *lines_len, void *stream);

/* --- read side (ref.go:113-126 getF decrypt) ---------- */
/* ChaCha20, zero nonce, counter 0, key = dek (ref.go:137-144). */
int glfsx_chacha20_xor(const uint8_t dek[32], const void *src, void *dst,
                       uint64_t n);

/* --- synthetic inputs (bench / tests; not a reference interface) -------- */
/* Device fill: byte o = byte (o & 7) of splitmix64(seed ^ (o >> 3)) where
 * splitmix64(x) is the SplitMix64 output function applied to x + golden
 * gamma; offset must be a multiple of 8.  Same stream as
 * oracle_fill_splitmix.  Enqueued on stream (NULL = the thread's stream). */
int glfsx_fill_splitmix_device(void *d_dst, uint64_t offset, uint64_t n,
                               uint64_t seed, void *stream);

/* n blobs of len bytes back to back (len % 8 == 0): blob b is the stream
 * above with seed seed0 + b at offset 0 (config 4: seed = blob index). */
int glfsx_fill_splitmix_blobs_device(void *d_dst, uint64_t n, uint64_t len,
                                     uint64_t seed0, void *stream);

/* A glfsx_post_fn that only counts: ctx points at uint64_t[2] = {posts,
 * bytes}.  For benchmarks of the host round trip without a store. */
int glfsx_sink_count(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                     uint64_t len);

/* Batched getF decrypt (ref.go:113-126): block j of d_ctext (block_size
 * bytes, the last one short; block_size % 64 == 0 as the reader requires,
 * blob.go:59) is decrypted with the DEK in bytes [32,64) of the 64-byte ref
 * j of d_refs into d_ptext.  Device pointers; enqueued on stream. */
int glfsx_decrypt_batch_device(const void *d_ctext, uint64_t total,
                               uint64_t block_size, const void *d_refs,
                               void *d_ptext, void *stream);

/* --- store boundary (bcsdk.WO [ext], ref.go:103) ----- */
/* An in-memory content-addressed store in blobcache MemStore's role (CID ->
 * ctext, MaxSize, Get, Exists) whose Post takes the GPU-computed CID.
 *   GLFSX_STORE_TRUST: a pre-hashed Post -- no host hashing; verify_every =
 *     k > 0 re-hashes every k-th Post on the host (parity mode) and fails it
 *     on a mismatch;
 *   GLFSX_STORE_HASH: every Post re-hashes the ctext on the calling thread,
 *     as MemStore.Post does behind ref.go:103 (today's cost of the drop-in),
 *     failing on a mismatch.
 * The host hash is the image's upstream BLAKE3 C (libclang-cpp.so); without
 * it the hashing modes return NULL.  keep_data 0 keeps CIDs and lengths
 * only.  cid_key: the store's BLAKE3 key (NULL = unkeyed, as glfsx's CID).
 * glfsx_store_post is a glfsx_post_fn: pass it with the store as post_ctx. */
typedef struct glfsx_store glfsx_store;
enum { GLFSX_STORE_TRUST = 0, GLFSX_STORE_HASH = 1 };
glfsx_store *glfsx_store_new(uint64_t max_size, int mode, uint64_t verify_every,
                             int keep_data, const uint8_t *cid_key);
void glfsx_store_free(glfsx_store *s);
int glfsx_store_post(void *store, int kind, const uint8_t *ref, const void *ctext,
                     uint64_t len);
int glfsx_store_exists(glfsx_store *s, const uint8_t cid[32]);
/* GLFSX_E_STORE when absent (blobcache.ErrNotFound); *data stays valid
 * until the store is freed. */
int glfsx_store_get(glfsx_store *s, const uint8_t cid[32], const void **data,
                    uint64_t *len);
/* number of distinct blobs; posts, bytes posted, posts re-hashed */
uint64_t glfsx_store_stats(glfsx_store *s, uint64_t *posts, uint64_t *bytes,
                           uint64_t *hashed);
/* The store's last error text; the pointer is valid on the calling thread
 * until its next glfsx_store_error call. */
const char *glfsx_store_error(glfsx_store *s);

/* Batched getF decrypt from host memory (ref.go:113-126 over a tree level:
 * index nodes, or a blob's data blocks): block j of ctext (block_size bytes,
 * the last one short; block_size % 64 == 0) decrypted with the DEK in bytes
 * [32,64) of the 64-byte ref j of refs (host) into ptext (host).  Uploads,
 * decrypts and downloads overlap in 64 MiB slabs. */
int glfsx_decrypt_batch(const void *ctext, uint64_t total, uint64_t block_size,
                        const uint8_t *refs, void *ptext);

/* --- tree shape (blob.go:219-268) -------------------------------------- */
int glfsx_depth(uint64_t size, uint64_t block_size);
uint64_t glfsx_branching_factor(uint64_t block_size);

#ifdef __cplusplus
}
#endif
#endif /* GLFSX_H */
