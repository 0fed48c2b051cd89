/*
 * oracle.h -- CPU restatement of the GLFS bigblob write path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under glfs_amd/ (the product) may include,
 * link or call this.  It is the checker for tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.
 *
 * What it restates (reference = /root/reference, Go, pinned 2026-03-13):
 *   bigblob/ref.go:98-111   (*Machine).post   -> oracle_post
 *   bigblob/ref.go:128-135  encrypt           -> oracle_post (DEK then XOR)
 *   bigblob/ref.go:137-144  cryptoXOR         -> oracle_chacha20_xor
 *   bigblob/ref.go:152-161  DeriveKey         -> oracle_derive_key
 *   bigblob/ref.go:77-82    Ref = CID || DEK  -> 64-byte ref layout
 *   bigblob/index.go:6-48   Index             -> zero-padded bs-byte nodes
 *   bigblob/blob.go:85-206  NewWriter/Write/Finish/postBuf/addRef/finishIndexes
 *                                             -> oracle_writer_*
 *   bigblob/blob.go:219-268 depth/branchingFactor -> oracle_depth
 *   machine.go:41-54        glfs salt derivation (salt always 0^32)
 *
 * The arithmetic lives in third-party Go modules that are NOT in /root/reference:
 *   lukechampine.com/blake3 v1.2.1 (go.mod:12)  -- BLAKE3 keyed hash + XOF
 *   golang.org/x/crypto v0.46.1-0.20251210140736-7dacc380ba00 (go.mod:10)
 *                                               -- chacha20, IETF 96-bit nonce
 *   blobcache.io/blobcache v0.5.1-0.20260313004939-67f9e150c2f9 (go.mod:16)
 *                                               -- store CID = BLAKE3-256(ctext)
 * They are restated from their published specifications (BLAKE3 paper/spec,
 * RFC 8439).  Pinning: tests/test_oracle.py checks BLAKE3 against the upstream C
 * BLAKE3 1.8.2 built into libclang-cpp.so (llvm_blake3_*) and ChaCha20 against
 * OpenSSL EVP_chacha20 / libsodium, plus the published RFC 8439 / BLAKE3
 * vectors; the bigblob layer is pinned by the reference's structural tests
 * (blob_test.go TestDepth, TestCreateFile "4 blobs") and by SURVEY.md's anchors
 * (an independent restatement).  The Go path itself cannot run here (no Go
 * toolchain), so byte parity with the Go binary is pinned through those.
 */
#ifndef GLFS_ORACLE_H
#define GLFS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* BLAKE3 over a whole message.  key == NULL -> unkeyed hash mode, else keyed
 * hash mode (KEYED_HASH flag, key words as IV).  Writes out_len bytes of XOF
 * output starting at output block counter 0. */
void oracle_blake3(uint8_t *out, size_t out_len, const uint8_t key[32],
                   const uint8_t *in, size_t n);

/* ChaCha20 (RFC 8439 block function), 96-bit nonce, initial counter `counter`,
 * XORed into dst (dst may alias src). */
void oracle_chacha20_xor(uint8_t *dst, const uint8_t *src, size_t n,
                         const uint8_t key[32], const uint8_t nonce[12],
                         uint32_t counter);

/* ref.go:152 DeriveKey(out[:32], salt, input) */
void oracle_derive_key(uint8_t out[32], const uint8_t salt[32],
                       const uint8_t *in, size_t n);

/* ref.go:98 post(): ref = CID || DEK.  ctext may be NULL.  cid_key NULL ->
 * CID = unkeyed BLAKE3-256(ctext) (blobcache HashAlgo_BLAKE3_256 with a nil
 * salt, the assumed MemStore behaviour); non-NULL -> keyed with cid_key. */
void oracle_post(uint8_t ref[64], uint8_t *ctext, const uint8_t salt[32],
                 const uint8_t *ptext, size_t n, const uint8_t *cid_key);

/* Store sink: called for every posted blob in the reference's Post order.
 * kind 0 = data block, 1 = index node.  Return nonzero to fail the write
 * (mirrors a store.Post error, blob.go:153-156 / 175-178). */
typedef int (*oracle_sink_fn)(void *ctx, int kind, const uint8_t ref[64],
                              const uint8_t *ctext, uint64_t len);

typedef struct oracle_writer oracle_writer;

/* blob.go:85-114.  Returns NULL and sets *err = -1 when block_size >
 * store_max (panic at blob.go:91), -2 when block_size < 128 (blob.go:94).
 * block_size == 0 means "use store_max" (machine.go:22-30 / blob.go:86-89).
 * salt NULL -> 0^32 (blob.go:96-98). */
oracle_writer *oracle_writer_new(uint64_t block_size, uint64_t store_max,
                                 const uint8_t *salt, const uint8_t *cid_key,
                                 oracle_sink_fn sink, void *sink_ctx, int *err);
int oracle_writer_write(oracle_writer *w, const uint8_t *data, size_t n);
/* blob.go:135-150: root ref (64 B), size, block size */
int oracle_writer_finish(oracle_writer *w, uint8_t root_ref[64],
                         uint64_t *size, uint64_t *block_size);
void oracle_writer_free(oracle_writer *w);

/* Closed-form level-by-level builder (equivalent to the streaming writer;
 * used to cross-check it).  Returns number of posted blobs, root in root_ref. */
int64_t oracle_create_closed(uint64_t block_size, const uint8_t *salt,
                             const uint8_t *cid_key, const uint8_t *data,
                             uint64_t size, uint8_t root_ref[64],
                             oracle_sink_fn sink, void *sink_ctx);

/* blob.go:256-264 */
int oracle_depth(uint64_t size, uint64_t block_size);

/* Multi-threaded post of equal chunks (CPU baseline leg of bench.py only).
 * refs: 64*ceil(total/chunk) bytes.  ctext may be NULL.  threads >= 1. */
void oracle_post_batch(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                       const uint8_t *ptext, uint64_t total, uint64_t chunk,
                       const uint8_t *cid_key, int threads);

/* The same post batch on the image's SIMD libraries (upstream BLAKE3 C with
 * AVX-512 from libclang-cpp.so, OpenSSL ChaCha20), cpu_simd.c: a second
 * CPU baseline for bench.py.  Returns -1 when a library is missing. */
int oracle_post_batch_simd(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                           const uint8_t *ptext, uint64_t total, uint64_t chunk,
                           const uint8_t *cid_key, int threads);
/* The Go path's primitive mix (cpu_simd.c): SIMD BLAKE3 for DEK and CID,
 * the portable scalar ChaCha20 above.  Returns -1 when BLAKE3 is missing. */
int oracle_post_batch_gomix(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                            const uint8_t *ptext, uint64_t total, uint64_t chunk,
                            const uint8_t *cid_key, int threads);

/* Deterministic data generator shared by tests/bench: byte offset o ->
 * byte (o & 7) of splitmix64(seed ^ (o >> 3)), little-endian. */
void oracle_fill_splitmix(uint8_t *dst, uint64_t offset, uint64_t n,
                          uint64_t seed);

/* n blobs of len bytes back to back, blob b = the stream above with seed
 * seed0 + b at offset 0 (config 4: seed = blob index). */
void oracle_fill_splitmix_blobs(uint8_t *dst, uint64_t n, uint64_t len,
                                uint64_t seed0);

#ifdef __cplusplus
}
#endif
#endif
