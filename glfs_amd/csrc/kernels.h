// kernels.h -- internal interface between the host runtime (glfsx.cpp) and the
// gfx950 kernels (post_kernels.hip).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace glfsx {

// Where ref j of a pass lands: refs + (j / ref_bf) * ref_stride + (j % ref_bf) * 64.
// Dense output: ref_bf = UINT64_MAX, ref_stride = 0.  Index-node output:
// ref_bf = bf, ref_stride = block_size (bigblob/index.go:33-38: slot i of a
// node is bytes [64i, 64i+64), the rest of the node stays zero).
struct RefLayout {
  uint8_t *refs;
  uint64_t bf;
  uint64_t stride;
};

// One "post" of n equal messages (the last one possibly short) laid out at
// src + j*stride: DEK pass then ChaCha20+CID pass (bigblob/ref.go:98-161).
struct PostJob {
  const uint8_t *src;
  uint8_t *ctext;       // nullable; may alias src
  uint64_t stride;      // bytes between message starts
  uint64_t msg_len;     // length of messages 0..n-2
  uint64_t last_len;    // length of message n-1
  uint64_t n;           // number of messages (>= 1)
  RefLayout out;
  uint32_t salt[8];     // DEK key words (little-endian words of the salt)
  uint32_t cid_key[8];  // CID key words (IV when unkeyed)
  bool cid_keyed;
};

// Largest message (bigblob block or index node) the post kernels accept:
// 256 workgroups x 256 lanes x 64 BLAKE3 chunks (split mode, 4 GiB).
constexpr uint64_t kMaxMsgLen = 256ull * 256 * 64 * 1024;

// fused = false: never the one-launch split form (k_pass_dc), for callers
// that return before the stream is synchronised (its failure is only
// visible to fused_errors_take after the stream has drained).
hipError_t launch_post(const PostJob &job, hipStream_t s, bool fused = true);

// After stream s has drained: nonzero when a one-launch split post on it
// gave up waiting for a DEK since the last call (its refs and ctext are
// invalid; the caller fails or repeats the post with fused = false).
uint32_t fused_errors_take(hipStream_t s);
// Test hooks: the next fused launch leaves message skip_msg's ready flag
// unset (~0u: none); wait_us bounds the DEK wait (0: the 1 s default).
void fused_debug(uint32_t skip_msg, uint64_t wait_us);
// Timeouts seen by fused_errors_take so far (process-wide).
uint64_t fused_timeouts();
// The bulk passes' clock probe on the current device (k_pass): out[0] =
// shader-clock cycles, out[1] = 100 MHz ticks summed over every k_pass
// workgroup since the last reset; reset: zero them after reading.
// Synchronous (waits for the device).
hipError_t clock_probe(int reset, uint64_t out[2]);

// The second half of launch_post alone: ChaCha20 keyed by the DEK already in
// bytes [32,64) of each ref slot, ctext store, CID into bytes [0,32).
hipError_t launch_cid_pass(const PostJob &job, hipStream_t s);

// DEK-only pass (keyed BLAKE3, first 32 XOF bytes) over the same layout,
// writing 32-byte digests to out (at byte offset `out_off` of each ref slot).
hipError_t launch_keyed_hash(const PostJob &job, uint32_t out_off,
                             hipStream_t s);

// ChaCha20 XOR (zero nonce, counter 0) of n bytes with key words k.
hipError_t launch_chacha_xor(const uint32_t k[8], const uint8_t *src,
                             uint8_t *dst, uint64_t n, hipStream_t s);

// Many small blobs, one lane each (glfs.PostBlob batched): blob i is
// src[offs[i] .. offs[i]+lens[i]); if lens[i] <= kMaxSmallLen its root ref
// (CID || DEK) goes to refs + 64*i (empty blobs use index_salt); longer blobs
// are skipped (the caller posts them).
constexpr uint64_t kMaxSmallLen = 16ull * 1024;
// entries per workgroup of the tree-line kernels (tree_kernels.hip)
constexpr uint32_t kTreeWG = 256;
struct SmallJob {
  const uint8_t *src;
  uint8_t *ctext;  // nullable; same offsets as src
  const uint64_t *offs, *lens;  // device arrays
  uint64_t n, max_len;
  uint8_t *refs;
  uint32_t raw_salt[8], index_salt[8], cid_key[8];
  bool cid_keyed;
  // blobs of at most small_max bytes are hashed here: min(kMaxSmallLen,
  // the blob block size) -- a longer blob has several blocks and an index
  // node (blob.go:120-206), so the caller Creates it (0 = kMaxSmallLen)
  uint64_t small_max;
  // hex_out != nullptr: the CID pass also writes blob i's root as the tree
  // line's hex fields -- 64 lower-case digits of the CID at hex_out +
  // hex_pos[i] and of the DEK kDekAfterCid bytes later (TreeJob::hex_pos)
  uint8_t *hex_out;
  const uint64_t *hex_pos;
  hipEvent_t cid_wait;  // nullable: the CID pass waits for it (after the DEK pass)
  uint32_t passes;      // 1: the DEK pass only, 2: the CID pass only, 0: both
};

// The small route's limit for blobs of block size bs.
inline uint64_t small_max_for(uint64_t bs) { return bs < kMaxSmallLen ? bs : kMaxSmallLen; }
hipError_t launch_post_small(const SmallJob &job, hipStream_t s);

// One-shot posts (ref.go:98-161 for one message of at most kMaxOneLen bytes:
// a glfs.PostBlob of a small blob, a Writer's tail block, an index node of a
// small-block blob): DEK, ChaCha20 and CID in one launch, one workgroup per
// descriptor.  src / ctext / ref may be pinned host memory (device pointers
// of it): the kernel reads the message once and writes ctext and ref
// straight into the caller's staging, so a post is one launch and a wait.
// Messages of kMaxOneLen < len <= kMaxMedLen take two launches (launch_med:
// one workgroup per 64 KiB span, the last-arriving one merges) and need the
// device scratch below.
constexpr uint64_t kMaxOneLen = 64ull * 1024;
constexpr uint64_t kMaxMedLen = 4ull << 20;
struct OneDesc {
  const uint8_t *src;  // 16-B aligned, device-accessible
  uint8_t *ctext;      // nullable, device-accessible, 16-B aligned
  uint8_t *ref;        // 64 B out: CID || DEK, 4-B aligned
  uint32_t len;        // <= kMaxMedLen
  uint32_t present;    // bytes [present, len) of the message are zero (not read)
  uint32_t cid_keyed;
  uint32_t salt[8];     // DEK key words
  uint32_t cid_key[8];  // CID key words (IV when unkeyed)
  // launch_med only (device memory): the staged message (len rounded up to
  // 64 B), 8 words per 64 KiB span, an arrival counter (zero before the
  // launch, left at zero) and the DEK
  uint8_t *dmsg;
  uint32_t *cvs, *cnt, *dek;
  // nullable, pinned host memory: set to seq (release, system scope) once
  // ctext and ref are in the caller's staging
  uint32_t *flag;
  uint32_t seq;
};
// descs: n descriptors in device-accessible memory; max_len bounds their len.
hipError_t launch_one(const OneDesc *descs, uint32_t n, uint64_t max_len,
                      hipStream_t s);
hipError_t launch_med(const OneDesc *descs, uint32_t n, uint64_t max_len,
                      hipStream_t s);
// One post, its descriptor passed by value: d.len <= kMaxOneLen (launch_one_v)
// or kMaxOneLen < d.len <= kMaxMedLen (launch_med_v).
hipError_t launch_one_v(const OneDesc &d, hipStream_t s);
hipError_t launch_med_v(const OneDesc &d, hipStream_t s);

// Read side: decrypt n contiguous blocks (bs % 64 == 0; the last one
// last_len bytes) with the DEKs in bytes [32,64) of refs[j] (dense).
hipError_t launch_decrypt(const uint8_t *ctext, uint8_t *ptext, uint64_t n,
                          uint64_t bs, uint64_t last_len, const uint8_t *refs,
                          hipStream_t s);

// Synthetic splitmix64 byte stream (see oracle_fill_splitmix); offset % 8 == 0.
hipError_t launch_fill(uint8_t *dst, uint64_t offset, uint64_t n, uint64_t seed,
                       hipStream_t s);

// Split mode (post_kernels.hip launch_pass): a launch of fewer than `wgs`
// workgroups spreads each message over up to 64 workgroups.  0 disables it.
// Returns the previous value.
uint32_t set_split_target(uint32_t wgs);
// Latency-mode threshold in workgroups (see post_kernels.hip); returns the
// previous value.
uint32_t set_latency_wgs(uint32_t wgs);
// Drop the split-mode scratch kept for stream s (call before destroying s,
// after it has drained).
void release_stream_scratch(hipStream_t s);

// Tree JSON lines on the device (tree_kernels.hip): see glfsx_tree_encode.
struct TreeJob {
  uint64_t n;
  const uint8_t *names;
  const uint64_t *name_offs;  // n + 1
  const uint32_t *modes;
  const uint8_t *types;
  const uint64_t *type_offs;  // n + 1
  const uint8_t *roots;       // 64 B per entry
  const uint64_t *sizes, *block_sizes;
  uint64_t *scratch;          // n + ceil(n / 256) words
  uint64_t *line_ends;        // nullable
  uint64_t *total;            // device word: total bytes
  uint8_t *out;               // nullable: lengths only
  uint64_t cap;               // bytes at out
  // hex_pos != nullptr: k_tree_write leaves the 64 hex digits of each cid
  // and dek unwritten and stores at hex_pos[i] the out offset of entry i's
  // first cid digit (its dek digits start kDekAfterCid bytes later); the
  // small-blob CID pass writes them (SmallJob::hex_out)
  uint64_t *hex_pos;
  // 1: the layout and static-line kernels run beside the small-blob DEK
  // pass (a 256-thread prefix, raised wave priority)
  uint32_t prio;
  // nullable, pinned host memory (device pointer) of ceil(n / 256) + 1
  // words: the layout's prefix kernel also stores the per-workgroup
  // exclusive prefix and then the total there (no copy kernel behind it)
  uint64_t *prefix_host;
};
// `<64 cid digits>","dek":"<64 dek digits>`: the dek's digits follow the
// cid's first digit by 64 + len("\",\"dek\":\"") bytes
constexpr uint32_t kDekAfterCid = 64 + 9;
hipError_t launch_tree_encode(const TreeJob &j, hipStream_t s);
// The same in two steps: the layout (line lengths, per-workgroup exclusive
// prefix at scratch + n, the total) -- it does not read the roots' values --
// and then the static lines (launch_tree_static).
hipError_t launch_tree_layout(const TreeJob &j, hipStream_t s);
// The lines without their hex digits (j.hex_pos set), in half workgroups
// small enough to run beside the small-blob DEK pass.
hipError_t launch_tree_static(const TreeJob &j, hipStream_t s);

// n blobs of len bytes (len % 8 == 0), blob b = the splitmix stream of seed
// seed0 + b (see oracle_fill_splitmix_blobs).
hipError_t launch_fill_blobs(uint8_t *dst, uint64_t n, uint64_t len, uint64_t seed0,
                             hipStream_t s);

#if GLFSX_WGTIME
hipError_t debug_wgtime(uint64_t *out);  // 8192 x 8 words (diagnostic builds)
#endif

// DeriveKey of any input length and output length (xof_kernels.hip): the
// hash state of one stream, carried across launches in device memory.
struct B3State {
  uint32_t key[8];
  uint32_t base;    // flags of every compression (kKeyed for DeriveKey)
  uint32_t depth;   // entries on the CV stack
  uint64_t chunks;  // chunks absorbed (a multiple of 256)
  uint32_t stack[64][8];
};
// `groups` whole 256-chunk groups at src, none of them holding the input's
// last byte.
hipError_t launch_b3_absorb(B3State *st, const uint8_t *src, uint64_t groups, hipStream_t s);
// The input's last n bytes (<= 256 KiB; 0 only for the empty input), then
// out_len bytes of XOF output.
hipError_t launch_b3_final(B3State *st, const uint8_t *src, uint64_t n, uint8_t *out,
                           uint64_t out_len, hipStream_t s);

void words_from_key(uint32_t w[8], const uint8_t key[32]);
void blake3_iv_words(uint32_t w[8]);

}  // namespace glfsx
