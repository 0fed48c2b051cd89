// post_kernels.hip -- gfx950 kernels for the bigblob write path.
//
// Per bigblob block ("message"), bigblob/ref.go:98-161 computes
//   DEK  = BLAKE3-keyed(salt, ptext)[0:32]                 (ref.go:146-161)
//   ctext = ChaCha20(DEK, nonce 0^12, counter 0) ^ ptext    (ref.go:137-144)
//   CID  = BLAKE3-256(ctext)   (store.Post, ref.go:103; blobcache [ext])
// Both hashes are BLAKE3 trees over 1 KiB chunks of 64 B blocks.
//
// Mapping (DESIGN.md "Kernels"):
//   * one 256-lane workgroup per message; lane t owns the G consecutive
//     BLAKE3 chunks [t*G, t*G+G) (G = power of two, template parameter) and
//     reduces them in registers to one subtree chaining value;
//   * the 16-word message schedule is applied at compile time (fully unrolled
//     rounds, the permutation is register renaming -- no LDS, no shuffles);
//   * the 256 subtree CVs are merged pairwise through LDS; the pairwise merge
//     with an odd element passing through is exactly BLAKE3's left-complete
//     tree, and the final parent gets ROOT;
//   * the ChaCha20 pass uses the message's DEK as wave-uniform SGPR operands
//     and fuses keystream XOR, the ctext store and the CID compression, so
//     ptext is read once per pass and ctext is never re-read.
// Integer ALU work only (v_add3_u32 / v_xor_b32 / v_alignbit_b32); no MFMA.
#include "kernels.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#ifndef GLFSX_LDS_CTEXT
#define GLFSX_LDS_CTEXT 1
#endif
#ifndef GLFSX_LDS_LOADS
#define GLFSX_LDS_LOADS 1
#endif
// CID pass: plaintext also arrives by buffer_load ... lds, into the ctext
// staging image (in place: the lane takes its pair out, writes the ctext pair
// back into the same slots, the wave stores full lines, then refills).
#ifndef GLFSX_CID_LDS_LOADS
#define GLFSX_CID_LDS_LOADS 1
#endif


namespace glfsx {
namespace {

constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u,
                             0xA54FF53Au, 0x510E527Fu, 0x9B05688Cu,
                             0x1F83D9ABu, 0x5BE0CD19u};
enum : uint32_t {
  kChunkStart = 1,
  kChunkEnd = 2,
  kParent = 4,
  kRoot = 8,
  kKeyed = 16,
};

struct Sched {
  int s[7][16];
};
constexpr Sched make_sched() {
  constexpr int perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  Sched t{};
  for (int i = 0; i < 16; ++i) t.s[0][i] = i;
  for (int r = 1; r < 7; ++r)
    for (int i = 0; i < 16; ++i) t.s[r][i] = t.s[r - 1][perm[i]];
  return t;
}
constexpr Sched kSched = make_sched();

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

// ARX steps as single-instruction asm statements (GLFSX_ASM_ARX): same
// instructions as the C form, but the compiler schedules them as opaque
// units, which on gfx950 issues measurably faster (DESIGN.md "Rooflines",
// tools/arx.hip).  Used from the second round on, so round 1 keeps the C
// form's constant folding (IV literals, uniform key words).
#ifndef GLFSX_ASM_ARX
#define GLFSX_ASM_ARX 1
#endif
template <int N>
__device__ __forceinline__ uint32_t rotr_a(uint32_t x) {
  uint32_t d;
  asm("v_alignbit_b32 %0, %1, %1, %2" : "=v"(d) : "v"(x), "i"(N));
  return d;
}
__device__ __forceinline__ uint32_t xor_a(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t add_a(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t add3_a(uint32_t a, uint32_t b, uint32_t c) {
#if GLFSX_ASM_ARX == 2
  return add_a(add_a(a, b), c);
#else
  uint32_t d;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
#endif
}

#define B3G_A(a, b, c, d, x, y)       \
  a = add3_a(a, b, (x));              \
  d = rotr_a<16>(xor_a(d, a));        \
  c = add_a(c, d);                    \
  b = rotr_a<12>(xor_a(b, c));        \
  a = add3_a(a, b, (y));              \
  d = rotr_a<8>(xor_a(d, a));         \
  c = add_a(c, d);                    \
  b = rotr_a<7>(xor_a(b, c));

#define CQR_A(a, b, c, d)             \
  a = add_a(a, b);                    \
  d = rotr_a<16>(xor_a(d, a));        \
  c = add_a(c, d);                    \
  b = rotr_a<20>(xor_a(b, c));        \
  a = add_a(a, b);                    \
  d = rotr_a<24>(xor_a(d, a));        \
  c = add_a(c, d);                    \
  b = rotr_a<25>(xor_a(b, c));

#define B3G_C(a, b, c, d, x, y) \
  a = a + b + (x);            \
  d = rotr(d ^ a, 16);        \
  c = c + d;                  \
  b = rotr(b ^ c, 12);        \
  a = a + b + (y);            \
  d = rotr(d ^ a, 8);         \
  c = c + d;                  \
  b = rotr(b ^ c, 7);

#if GLFSX_ASM_ARX
#define B3G(a, b, c, d, x, y)           \
  if constexpr (R == 0 || !A) {         \
    B3G_C(a, b, c, d, x, y)             \
  } else {                              \
    B3G_A(a, b, c, d, x, y)             \
  }
#else
#define B3G(a, b, c, d, x, y) B3G_C(a, b, c, d, x, y)
#endif

// GLFSX_SCHED: the ARX rounds of the many-wave kernels written step by step
// over all independent chains of a half-round (4 G or 4 QR; 8 when a BLAKE3
// round is fused with a ChaCha20 double round), with a scheduling barrier
// after each step, so the compiler cannot serialise the chains: two
// dependent instructions are always at least 3 (7 fused) independent ones
// apart.  1 = compiler-visible C form (no hazard nops), 2 = the one-asm-
// statement-per-instruction form (default: measured +2.5% config 2, +1-2%
// small blobs and read side; 1 was 5.7% slower).  0 = the plain macros
// above.  The kernels take the form as their int template parameter A
// (0 = compiler-scheduled C, 1 = asm in quarter-round order, 2 = asm step-
// interleaved); the headline's CID pass runs form 1 (GLFSX_HEAD_CID).
#ifndef GLFSX_SCHED
#define GLFSX_SCHED 2
#endif
#define SB() __builtin_amdgcn_sched_barrier(0)
constexpr int kCol[4][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15}};
constexpr int kDia[4][4] = {{0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};

template <int F>
__device__ __forceinline__ uint32_t s_add(uint32_t a, uint32_t b) {
  if constexpr (F == 2) return add_a(a, b); else return a + b;
}
template <int F>
__device__ __forceinline__ uint32_t s_add3(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (F == 2) return add3_a(a, b, c); else return a + b + c;
}
template <int F>
__device__ __forceinline__ uint32_t s_xor(uint32_t a, uint32_t b) {
  if constexpr (F == 2) return xor_a(a, b); else return a ^ b;
}
template <int F, int N>
__device__ __forceinline__ uint32_t s_rot(uint32_t x) {
  if constexpr (F == 2) return rotr_a<N>(x); else return rotr(x, N);
}

// One half-round, 12 steps: B3 (if G) = 4 BLAKE3 G's on v with message words
// m[s[mo + 2k]], m[s[mo + 2k + 1]]; Q (if Q) = 4 ChaCha20 quarter-rounds on x.
template <int F, bool DIAG, int R, bool G, bool Q>
__device__ __forceinline__ void half_il(uint32_t (&v)[16], const uint32_t (&m)[16],
                                        uint32_t (&x)[16]) {
  constexpr const int (*I)[4] = DIAG ? kDia : kCol;
  constexpr const int *s = kSched.s[R];
  constexpr int mo = DIAG ? 8 : 0;
#define IL_STEP(gstmt, qstmt)                        \
  _Pragma("unroll") for (int k = 0; k < 4; ++k) {    \
    if constexpr (G) { gstmt; }                      \
    if constexpr (Q) { qstmt; }                      \
  }                                                  \
  SB();
#define VA v[I[k][0]]
#define VB v[I[k][1]]
#define VC v[I[k][2]]
#define VD v[I[k][3]]
#define XA x[I[k][0]]
#define XB x[I[k][1]]
#define XC x[I[k][2]]
#define XD x[I[k][3]]
  IL_STEP(VA = s_add3<F>(VA, VB, m[s[mo + 2 * k]]), XA = s_add<F>(XA, XB))
  IL_STEP(VD = s_xor<F>(VD, VA), XD = s_xor<F>(XD, XA))
  IL_STEP(VD = (s_rot<F, 16>(VD)), XD = (s_rot<F, 16>(XD)))
  IL_STEP(VC = s_add<F>(VC, VD), XC = s_add<F>(XC, XD))
  IL_STEP(VB = s_xor<F>(VB, VC), XB = s_xor<F>(XB, XC))
  IL_STEP(VB = (s_rot<F, 12>(VB)), XB = (s_rot<F, 20>(XB)))
  IL_STEP(VA = s_add3<F>(VA, VB, m[s[mo + 2 * k + 1]]), XA = s_add<F>(XA, XB))
  IL_STEP(VD = s_xor<F>(VD, VA), XD = s_xor<F>(XD, XA))
  IL_STEP(VD = (s_rot<F, 8>(VD)), XD = (s_rot<F, 24>(XD)))
  IL_STEP(VC = s_add<F>(VC, VD), XC = s_add<F>(XC, XD))
  IL_STEP(VB = s_xor<F>(VB, VC), XB = s_xor<F>(XB, XC))
  IL_STEP(VB = (s_rot<F, 7>(VB)), XB = (s_rot<F, 25>(XB)))
#undef VA
#undef VB
#undef VC
#undef VD
#undef XA
#undef XB
#undef XC
#undef XD
#undef IL_STEP
}

template <int R, int A = 2>
__device__ __forceinline__ void b3_round(uint32_t (&v)[16],
                                         const uint32_t (&m)[16]) {
#if GLFSX_SCHED
  if constexpr (A == 2 && R > 0) {
    uint32_t x[16];
    half_il<GLFSX_SCHED, false, R, true, false>(v, m, x);
    half_il<GLFSX_SCHED, true, R, true, false>(v, m, x);
    return;
  }
#endif
  constexpr const int *s = kSched.s[R];
  B3G(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
  B3G(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
  B3G(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
  B3G(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
  B3G(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
  B3G(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
  B3G(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
  B3G(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
}

// cv <- first 8 words of compress(cv, m, counter, block_len, flags): the
// chaining value, or for a ROOT compression the first 32 output bytes
// (XOF block 0), which is all the write path ever reads.
template <int A = 2>
__device__ __forceinline__ void b3_compress(uint32_t (&cv)[8],
                                            const uint32_t (&m)[16],
                                            uint32_t ctr_lo, uint32_t ctr_hi,
                                            uint32_t blen, uint32_t flags) {
  uint32_t v[16] = {cv[0],  cv[1],  cv[2],  cv[3],  cv[4],  cv[5],
                    cv[6],  cv[7],  kIV[0], kIV[1], kIV[2], kIV[3],
                    ctr_lo, ctr_hi, blen,   flags};
  b3_round<0, A>(v, m);
  b3_round<1, A>(v, m);
  b3_round<2, A>(v, m);
  b3_round<3, A>(v, m);
  b3_round<4, A>(v, m);
  b3_round<5, A>(v, m);
  b3_round<6, A>(v, m);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
}

#define CQR(a, b, c, d) \
  a += b;               \
  d = rotr(d ^ a, 16);  \
  c += d;               \
  b = rotr(b ^ c, 20);  \
  a += b;               \
  d = rotr(d ^ a, 24);  \
  c += d;               \
  b = rotr(b ^ c, 25);

// RFC 8439 block function, nonce 0^12 (ref.go:138), 32-bit block counter.
template <int A = 2>
__device__ __forceinline__ void chacha_block(uint32_t (&x)[16],
                                             const uint32_t (&k)[8],
                                             uint32_t ctr) {
  constexpr uint32_t c0 = 0x61707865u, c1 = 0x3320646eu, c2 = 0x79622d32u,
                     c3 = 0x6b206574u;
  x[0] = c0;
  x[1] = c1;
  x[2] = c2;
  x[3] = c3;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] = k[i];
  x[12] = ctr;
  x[13] = 0;
  x[14] = 0;
  x[15] = 0;
  // round 1 in C: its key-only quarter-rounds are uniform and hoisted
  CQR(x[0], x[4], x[8], x[12]);
  CQR(x[1], x[5], x[9], x[13]);
  CQR(x[2], x[6], x[10], x[14]);
  CQR(x[3], x[7], x[11], x[15]);
  CQR(x[0], x[5], x[10], x[15]);
  CQR(x[1], x[6], x[11], x[12]);
  CQR(x[2], x[7], x[8], x[13]);
  CQR(x[3], x[4], x[9], x[14]);
#pragma unroll
  for (int i = 1; i < 10; ++i) {
#if GLFSX_SCHED
   if constexpr (A == 2) {
    uint32_t v[16], m[16];
    half_il<GLFSX_SCHED, false, 0, false, true>(v, m, x);
    half_il<GLFSX_SCHED, true, 0, false, true>(v, m, x);
    continue;
   }
#endif
#if GLFSX_ASM_ARX
   if constexpr (A) {
    CQR_A(x[0], x[4], x[8], x[12]);
    CQR_A(x[1], x[5], x[9], x[13]);
    CQR_A(x[2], x[6], x[10], x[14]);
    CQR_A(x[3], x[7], x[11], x[15]);
    CQR_A(x[0], x[5], x[10], x[15]);
    CQR_A(x[1], x[6], x[11], x[12]);
    CQR_A(x[2], x[7], x[8], x[13]);
    CQR_A(x[3], x[4], x[9], x[14]);
   } else {
    CQR(x[0], x[4], x[8], x[12]);
    CQR(x[1], x[5], x[9], x[13]);
    CQR(x[2], x[6], x[10], x[14]);
    CQR(x[3], x[7], x[11], x[15]);
    CQR(x[0], x[5], x[10], x[15]);
    CQR(x[1], x[6], x[11], x[12]);
    CQR(x[2], x[7], x[8], x[13]);
    CQR(x[3], x[4], x[9], x[14]);
   }
#else
    CQR(x[0], x[4], x[8], x[12]);
    CQR(x[1], x[5], x[9], x[13]);
    CQR(x[2], x[6], x[10], x[14]);
    CQR(x[3], x[7], x[11], x[15]);
    CQR(x[0], x[5], x[10], x[15]);
    CQR(x[1], x[6], x[11], x[12]);
    CQR(x[2], x[7], x[8], x[13]);
    CQR(x[3], x[4], x[9], x[14]);
#endif
  }
  x[0] += c0;
  x[1] += c1;
  x[2] += c2;
  x[3] += c3;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] += k[i];
  x[12] += ctr;
}

// 64-byte message block at p with `avail` valid bytes (zero padded).
template <bool ALIGNED>
__device__ __forceinline__ void load_block(uint32_t (&m)[16], const uint8_t *p,
                                           uint32_t avail) {
  if (ALIGNED && avail >= 64) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    m[0] = w0.x; m[1] = w0.y; m[2] = w0.z; m[3] = w0.w;
    m[4] = w1.x; m[5] = w1.y; m[6] = w1.z; m[7] = w1.w;
    m[8] = w2.x; m[9] = w2.y; m[10] = w2.z; m[11] = w2.w;
    m[12] = w3.x; m[13] = w3.y; m[14] = w3.z; m[15] = w3.w;
  } else {
    const uint32_t lim = avail < 64 ? avail : 64;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t idx = 4 * i + b;
        if (idx < lim) w |= uint32_t(p[idx]) << (8 * b);
      }
      m[i] = w;
    }
  }
}

template <bool ALIGNED>
__device__ __forceinline__ void store_block(uint8_t *p, const uint32_t (&c)[16],
                                            uint32_t avail) {
  if (ALIGNED && avail >= 64) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
    q[0] = make_uint4(c[0], c[1], c[2], c[3]);
    q[1] = make_uint4(c[4], c[5], c[6], c[7]);
    q[2] = make_uint4(c[8], c[9], c[10], c[11]);
    q[3] = make_uint4(c[12], c[13], c[14], c[15]);
  } else {
    const uint32_t lim = avail < 64 ? avail : 64;
    for (uint32_t idx = 0; idx < lim; ++idx)
      p[idx] = uint8_t(c[idx >> 2] >> (8 * (idx & 3)));
  }
}

// Zero the bytes of m at and beyond `avail` (only called when avail < 64).
__device__ __forceinline__ void mask_tail(uint32_t (&m)[16], uint32_t avail) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t lo = 4 * i;
    uint32_t keep;
    if (lo + 4 <= avail) keep = 0xffffffffu;
    else if (lo >= avail) keep = 0u;
    else keep = (1u << (8 * (avail - lo))) - 1u;
    m[i] &= keep;
  }
}

constexpr int ilog2(int g) { return g <= 1 ? 0 : 1 + ilog2(g / 2); }

struct KArgs {
  const uint8_t *src;
  uint8_t *ctext;
  uint64_t stride, msg_len, last_len, n;
  uint8_t *refs;
  uint64_t ref_bf, ref_stride;
  uint32_t key[8];
  uint32_t base;     // kKeyed or 0
  uint32_t out_off;  // byte offset of the 32-byte result inside the ref slot
  // split mode (few messages): 2^split_log2 workgroups per message, each over
  // 256*G consecutive chunks; their subtree CVs go to scratch (8 words per
  // workgroup) and the message's last-arriving workgroup (per-message
  // arrival counter in cnt, zero between launches) finishes the tree.
  // split_log2 == 0: one workgroup per message, no scratch.
  uint32_t split_log2;
  uint32_t *scratch;
  uint32_t *cnt;
  // the clock probe's two counters on this launch's device (g_clk), or
  // nullptr: probing is off until the process first calls clock_probe
  unsigned long long *clk;
};

// Split mode: thread 0 publishes this workgroup's subtree CV and counts it
// in; returns true in every thread of the workgroup that arrives last for
// its message, which then merges all W CVs.  The workgroups of a message
// run on different XCDs, whose L2s are not coherent with each other.  An
// agent-scope release fence would write back the whole L2 of the issuing
// XCD per workgroup (measured: +50 us per 1 GiB split pass); instead the CV
// words are agent-scope atomic stores (written through to the coherence
// point), the wave waits for them to complete, and only then increments the
// counter (an agent-scope atomic, performed device-wide); the last
// workgroup reads the CVs with agent-scope atomic loads.
__device__ __forceinline__ void publish_cv(uint32_t *dst, const uint32_t (&cv)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    __hip_atomic_store(dst + i, cv[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_cv_word(const uint32_t *src) {
  return __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool arrive_last(uint32_t *cnt, uint32_t W,
                                            uint32_t t, uint32_t *flag) {
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the CV stores are done
    const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    *flag = old + 1 == W;
  }
  __syncthreads();
  return *flag != 0;
}

// Merge step after the last block of local chunk jj: pop/parent/push on the
// lane's CV stack (eager merges = ctz(jj+1); final merges empty the stack).
template <int D, int A = 2>
__device__ __forceinline__ void lane_merge(uint32_t (&cv)[8],
                                           uint32_t (&stk)[D > 0 ? D : 1][8],
                                           uint32_t &depth, uint32_t jj,
                                           bool last, bool whole,
                                           const uint32_t (&key)[8],
                                           uint32_t base) {
  if constexpr (D > 0) {
    const uint32_t merges = last ? depth : uint32_t(__builtin_ctz(jj + 1));
    for (uint32_t i = 0; i < merges; ++i) {
      uint32_t m[16];
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        m[w] = stk[0][w];
        m[8 + w] = cv[w];
        cv[w] = key[w];
      }
#pragma unroll
      for (int d = 0; d + 1 < D; ++d)
#pragma unroll
        for (int w = 0; w < 8; ++w) stk[d][w] = stk[d + 1][w];
      --depth;
      const uint32_t fl =
          base | kParent | ((whole && last && depth == 0) ? kRoot : 0u);
      b3_compress<A>(cv, m, 0u, 0u, 64u, fl);
    }
    if (!last) {
#pragma unroll
      for (int d = D - 1; d > 0; --d)
#pragma unroll
        for (int w = 0; w < 8; ++w) stk[d][w] = stk[d - 1][w];
#pragma unroll
      for (int w = 0; w < 8; ++w) stk[0][w] = cv[w];
      ++depth;
    }
  }
}

// One full 64-B block of the fast path: (ChaCha20 keystream XOR, ctext
// store,) BLAKE3 compression.
// LDS staging of ctext (GLFSX_LDS_CTEXT): each wave owns 64 lines x 128 B;
// lane c puts 16-B piece p of its current 128-B line at byte
// c*128 + ((p ^ ((c>>1)&7)) << 4) (conflict-free ds_write_b128 in 8-lane
// groups and ds_read_b128 in its 16-lane groups), then the wave stores 8 full
// lines per buffer_store_dwordx4 instead of 64 sixteenths of lines.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

__device__ __forceinline__ uint32_t lds_offset(const void *p) {
  return uint32_t(reinterpret_cast<uintptr_t>(
      (const __attribute__((address_space(3))) void *)p));
}

// opaque to the optimiser: keeps per-piece addresses from being hoisted
// into 8-16 loop-invariant VGPRs (1 v_xor each instead)
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Staging-image swizzle: row L (one lane's pair of blocks, 128 B) keeps its
// 16-B piece p in slot p ^ img_swz(L).  The three access patterns must be
// conflict-free: the lane's own ds_write_b128 (groups of 8 consecutive
// lanes, 32 banks), its ds_read_b128 of its own row, and the store path's
// ds_read_b128 of (row 8k + l/8, piece l%8) (groups of 16 lanes, 64 banks;
// MI355X_MICROARCH.md LDS).  (L >> 1) & 7 (GLFSX_SWZ=0) gives pairs of
// lanes the same slot in the write groups: a 2-way conflict on every staged
// store (SQ_LDS_BANK_CONFLICT 8.3 cycles per ds_write_b128).  Both keep
// img_swz(8k + r) = img_swz(r) ^ ((k & 1) << 2), which the store path uses.
#ifndef GLFSX_SWZ
#define GLFSX_SWZ 1
#endif
__device__ __forceinline__ uint32_t img_swz(uint32_t L) {
#if GLFSX_SWZ
  return ((L >> 1) & 3u) | (((L ^ (L >> 3)) & 1u) << 2);
#else
  return (L >> 1) & 7u;
#endif
}

template <bool CHACHA, bool STAGE = false, int A = 2>
__device__ __forceinline__ void full_block(uint32_t (&cv)[8], const uint4 &w0,
                                           const uint4 &w1, const uint4 &w2,
                                           const uint4 &w3, uint32_t chunk,
                                           uint32_t b, uint32_t fl,
                                           const uint32_t (&dek)[8],
                                           uint4 *out, uint32_t wa = 0,
                                           uint32_t half = 0) {
  uint32_t m[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w,
                    w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
  if constexpr (CHACHA) {
    uint32_t x[16];
    chacha_block<A>(x, dek, (chunk << 4) + b);
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] ^= x[i];
    if (STAGE) {  // LDS staging: wa = this lane's swizzled line address
      wa = opaque(wa);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<lds_u32x4 *>(wa ^ ((4u * half + q) << 4)) =
            u32x4{m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]};
    } else if (out) {
      out[0] = make_uint4(m[0], m[1], m[2], m[3]);
      out[1] = make_uint4(m[4], m[5], m[6], m[7]);
      out[2] = make_uint4(m[8], m[9], m[10], m[11]);
      out[3] = make_uint4(m[12], m[13], m[14], m[15]);
    }
  }
  b3_compress<A>(cv, m, chunk, 0u, 64u, fl);
}

// GLFSX_PIPE: the pair's second keystream block is computed interleaved
// with the first block's compression (two independent ARX streams in one
// region instead of strict phases); same instructions, same results.
#ifndef GLFSX_PIPE
#define GLFSX_PIPE 1
#endif
#define CDR_A(x)                     \
  CQR_A(x[0], x[4], x[8], x[12]);    \
  CQR_A(x[1], x[5], x[9], x[13]);    \
  CQR_A(x[2], x[6], x[10], x[14]);   \
  CQR_A(x[3], x[7], x[11], x[15]);   \
  CQR_A(x[0], x[5], x[10], x[15]);   \
  CQR_A(x[1], x[6], x[11], x[12]);   \
  CQR_A(x[2], x[7], x[8], x[13]);    \
  CQR_A(x[3], x[4], x[9], x[14]);

// one BLAKE3 G and one ChaCha20 quarter-round, step by step (the two
// have the same add / xor-rotate shape): two independent chains per step
#define GQ_A(a, b, c, d, mx, my, e, f, g, h)                  \
  a = add3_a(a, b, (mx)); e = add_a(e, f);                    \
  d = rotr_a<16>(xor_a(d, a)); h = rotr_a<16>(xor_a(h, e));   \
  c = add_a(c, d); g = add_a(g, h);                           \
  b = rotr_a<12>(xor_a(b, c)); f = rotr_a<20>(xor_a(f, g));   \
  a = add3_a(a, b, (my)); e = add_a(e, f);                    \
  d = rotr_a<8>(xor_a(d, a)); h = rotr_a<24>(xor_a(h, e));    \
  c = add_a(c, d); g = add_a(g, h);                           \
  b = rotr_a<7>(xor_a(b, c)); f = rotr_a<25>(xor_a(f, g));

// BLAKE3 round R of v fused with one ChaCha20 double round of x
template <int R>
__device__ __forceinline__ void gq_round(uint32_t (&v)[16], const uint32_t (&m)[16],
                                         uint32_t (&x)[16]) {
  constexpr const int *s = kSched.s[R];
  GQ_A(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]], x[0], x[4], x[8], x[12]);
  GQ_A(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]], x[1], x[5], x[9], x[13]);
  GQ_A(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]], x[2], x[6], x[10], x[14]);
  GQ_A(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]], x[3], x[7], x[11], x[15]);
  GQ_A(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]], x[0], x[5], x[10], x[15]);
  GQ_A(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]], x[1], x[6], x[11], x[12]);
  GQ_A(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]], x[2], x[7], x[8], x[13]);
  GQ_A(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]], x[3], x[4], x[9], x[14]);
}

__device__ __forceinline__ void stage_half(uint32_t wa, uint32_t half,
                                           const uint32_t (&m)[16]) {
  wa = opaque(wa);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<lds_u32x4 *>(wa ^ ((4u * half + q) << 4)) =
        u32x4{m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]};
}

// Both blocks of a pair in the LDS-staged CID pass (asm ARX form):
// ChaCha(a); then BLAKE3(a) interleaved round by round with ChaCha(b);
// then BLAKE3(b).
template <int A>
__device__ __forceinline__ void pair_pipelined(
    uint32_t (&cv)[8], const uint4 &a0, const uint4 &a1, const uint4 &a2,
    const uint4 &a3, const uint4 &b0, const uint4 &b1, const uint4 &b2,
    const uint4 &b3, uint32_t chunk, uint32_t blk, uint32_t fla, uint32_t flb,
    const uint32_t (&dek)[8], uint32_t wa) {
  constexpr uint32_t c0 = 0x61707865u, c1 = 0x3320646eu, c2 = 0x79622d32u,
                     c3 = 0x6b206574u;
  uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                    a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
  const uint32_t ctr_a = (chunk << 4) + blk;
  {
    uint32_t x[16];
    chacha_block<A>(x, dek, ctr_a);
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] ^= x[i];
  }
  stage_half(wa, 0, m);
  // block b's keystream state, round 1 in C (key-only quarter-rounds hoist)
  const uint32_t ctr_b = ctr_a + 1;
  uint32_t x[16] = {c0, c1, c2, c3, dek[0], dek[1], dek[2], dek[3],
                    dek[4], dek[5], dek[6], dek[7], ctr_b, 0u, 0u, 0u};
  CQR(x[0], x[4], x[8], x[12]);
  CQR(x[1], x[5], x[9], x[13]);
  CQR(x[2], x[6], x[10], x[14]);
  CQR(x[3], x[7], x[11], x[15]);
  CQR(x[0], x[5], x[10], x[15]);
  CQR(x[1], x[6], x[11], x[12]);
  CQR(x[2], x[7], x[8], x[13]);
  CQR(x[3], x[4], x[9], x[14]);
  // BLAKE3(a): round 0 alone (C form, IV literals), rounds 1-6 step by
  // step with ChaCha(b)'s double rounds 2-7, then ChaCha(b)'s last three
  uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    kIV[0], kIV[1], kIV[2], kIV[3], chunk, 0u, 64u, fla};
  b3_round<0, true>(v, m);
#if GLFSX_SCHED
  if constexpr (A == 2) {
#define GQ_IL(R)                                           \
  half_il<GLFSX_SCHED, false, R, true, true>(v, m, x);     \
  half_il<GLFSX_SCHED, true, R, true, true>(v, m, x);
    GQ_IL(1) GQ_IL(2) GQ_IL(3) GQ_IL(4) GQ_IL(5) GQ_IL(6)
#undef GQ_IL
    for (int i = 0; i < 3; ++i) {
      half_il<GLFSX_SCHED, false, 0, false, true>(v, m, x);
      half_il<GLFSX_SCHED, true, 0, false, true>(v, m, x);
    }
  } else
#endif
  {
    gq_round<1>(v, m, x);
    gq_round<2>(v, m, x);
    gq_round<3>(v, m, x);
    gq_round<4>(v, m, x);
    gq_round<5>(v, m, x);
    gq_round<6>(v, m, x);
    CDR_A(x);
    CDR_A(x);
    CDR_A(x);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
  x[0] += c0;
  x[1] += c1;
  x[2] += c2;
  x[3] += c3;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] += dek[i];
  x[12] += ctr_b;
  uint32_t mb[16] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w,
                     b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w};
#pragma unroll
  for (int i = 0; i < 16; ++i) mb[i] ^= x[i];
  stage_half(wa, 1, mb);
  b3_compress<A>(cv, mb, chunk, 0u, 64u, flb);
}

// Fast path: the lane's G chunks are all full (16*G consecutive 64-B blocks,
// 16-B aligned).  Blocks go in pairs through two named register buffers: the
// odd block's loads are issued before the even block is compressed and the
// next even block's before the odd one, so HBM latency is covered and no
// buffer is copied on the loop back-edge.  Chunk-start / chunk-end flags and
// the chaining-value reset are per-chunk (scalar), not per-block selects.
// cst: bytes the staged ctext stores may write from cmsg (0: none -- the
// stores fall outside the buffer descriptor and are dropped; default: clen).
template <int G, bool CHACHA, bool STAGE = false, int A = 2>
__device__ __forceinline__ void lane_subtree_full(
    uint32_t (&cv)[8], const uint8_t *msg, uint8_t *cmsg, uint32_t first,
    bool whole, const uint32_t (&key)[8], uint32_t base,
    const uint32_t (&dek)[8], uint32_t sbase = 0, uint32_t clen = 0,
    uint32_t cbase = 0, uint32_t cst = ~0u) {
  constexpr int D = ilog2(G);
  constexpr uint32_t NB = 16u * G;
  uint32_t stk[D > 0 ? D : 1][8];
  uint32_t depth = 0;
  const uint4 *q = reinterpret_cast<const uint4 *>(msg + (uint64_t(first) << 10));
  uint4 *cq = cmsg ? reinterpret_cast<uint4 *>(cmsg + (uint64_t(first) << 10))
                   : nullptr;
  // LDS staging (STAGE: sbase = this wave's 8 KiB, the whole wave is on
  // this path).  CHACHA: ctext staged for full-line stores.  !CHACHA (DEK
  // pass): plaintext loaded by buffer_load ... lds, 8 full lines per
  // instruction, one pair of blocks ahead, into the same swizzled image.
  // CHACHA && gl: the image is shared by the plaintext pair (landing) and
  // the ctext pair (leaving), so the next pair is issued after the stores
  constexpr bool gl = STAGE && (!CHACHA || GLFSX_CID_LDS_LOADS);
  uint4 a0, a1, a2, a3;
  if constexpr (!gl) {
    a0 = q[0];
    a1 = q[1];
    a2 = q[2];
    a3 = q[3];
  }
  const uint32_t l = threadIdx.x & 63u, r = l >> 3, pc = l & 7u;
  const uint32_t wa = STAGE ? sbase + (l << 7) + (img_swz(l) << 4) : 0u;
  const uint32_t wst = CHACHA ? wa : 0u;  // full_block's staging target
  const uint32_t rb = sbase + (r << 7) + ((pc ^ img_swz(r)) << 4);
  // store voffset of (line r of this wave's 8-line group 0, piece pc); lane
  // l's data starts at chunk `first` of msg and lane 0's at first - l*G
  // (k_pass: first = t*G; k_small: msg = the wave's base, first = l*G)
  const uint32_t vo = ((first + (r - l) * uint32_t(G)) << 10) + (pc << 4);
  // wave-uniform descriptors (msg / cmsg, clen uniform over the wave)
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      CHACHA ? cmsg : const_cast<uint8_t *>(msg), 0, STAGE ? (cst == ~0u ? clen : cst) : 0u,
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_ld = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t *>(msg), 0, STAGE ? clen : 0u, 0x00020000);
  const uint32_t sb = __builtin_amdgcn_readfirstlane(sbase);
  // gl: source of (line 8k+r, image slot pc) = piece pc ^ swizzle(8k+r)
  const uint32_t lo0 = vo - (pc << 4) + ((pc ^ img_swz(r)) << 4);
  auto issue = [&](uint32_t s) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc_ld, (__attribute__((address_space(3))) void *)(uintptr_t)(sb + 1024u * k),
          16, (k & 1) ? (lo0 ^ 64u) : lo0, ((8u * k * uint32_t(G)) << 10) + 128u * s,
          0, 0);
  };
  if constexpr (gl) issue(0);
  for (uint32_t jj = 0; jj < uint32_t(G); ++jj) {
    // absolute chunk index (BLAKE3 chunk counter, ChaCha block counter / 16);
    // msg points at chunk cbase of the message
    const uint32_t chunk = cbase + first + jj;
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = key[i];
    for (uint32_t pp = 0; pp < 8; ++pp) {
      const uint32_t blk = jj * 16 + 2 * pp;
      uint4 b0, b1, b2, b3;
      if constexpr (gl) {
        // this pair's lines have landed; take them, then refill the image
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 v[8];
        const uint32_t w = opaque(wa);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          v[i] = *reinterpret_cast<const lds_u32x4 *>(w ^ (uint32_t(i) << 4));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (!CHACHA && blk + 2 < NB) issue(blk / 2 + 1);
        a0 = make_uint4(v[0].x, v[0].y, v[0].z, v[0].w);
        a1 = make_uint4(v[1].x, v[1].y, v[1].z, v[1].w);
        a2 = make_uint4(v[2].x, v[2].y, v[2].z, v[2].w);
        a3 = make_uint4(v[3].x, v[3].y, v[3].z, v[3].w);
        b0 = make_uint4(v[4].x, v[4].y, v[4].z, v[4].w);
        b1 = make_uint4(v[5].x, v[5].y, v[5].z, v[5].w);
        b2 = make_uint4(v[6].x, v[6].y, v[6].z, v[6].w);
        b3 = make_uint4(v[7].x, v[7].y, v[7].z, v[7].w);
      } else {
        const uint4 *nb = q + 4 * (blk + 1);
        b0 = nb[0];
        b1 = nb[1];
        b2 = nb[2];
        b3 = nb[3];
      }
      constexpr bool stg = CHACHA && STAGE;
      // (the other branch is the same template as the latency-mode C-form
      // pass, which tests/test_gpu_parity.py::test_arx_forms_vs_oracle runs)
      if constexpr (GLFSX_PIPE && GLFSX_ASM_ARX == 1 && gl && stg && A) {
        uint32_t fb = base;
        if (pp == 7) fb |= kChunkEnd | ((whole && G == 1) ? kRoot : 0u);
        pair_pipelined<A>(cv, a0, a1, a2, a3, b0, b1, b2, b3, chunk, 2 * pp,
                       base | (pp == 0 ? kChunkStart : 0u), fb, dek, wst);
      } else {
      full_block<CHACHA, stg, A>(cv, a0, a1, a2, a3, chunk, 2 * pp,
                         base | (pp == 0 ? kChunkStart : 0u), dek,
                         cq && !stg ? cq + 4 * blk : nullptr, wst, 0);
      if (!gl && blk + 2 < NB) {
        const uint4 *na = q + 4 * (blk + 2);
        a0 = na[0];
        a1 = na[1];
        a2 = na[2];
        a3 = na[3];
      }
      uint32_t fl = base;
      if (pp == 7) fl |= kChunkEnd | ((whole && G == 1) ? kRoot : 0u);
      full_block<CHACHA, stg, A>(cv, b0, b1, b2, b3, chunk, 2 * pp + 1, fl, dek,
                         cq && !stg ? cq + 4 * (blk + 1) : nullptr, wst, 1);
      }
      if (stg) {
        // lane l stores piece pc of line 8k + r: each store instruction
        // writes 8 whole 128-B lines.  Line 8k+r's slot for pc is
        // rb ^ ((k&1) << 6) + k*1024 (the swizzle's bit 2 is k's parity).
        const uint32_t r0 = opaque(rb), r1 = r0 ^ 64u, v0 = vo + blk * 64u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const u32x4 v = *reinterpret_cast<const lds_u32x4 *>(
              ((k & 1) ? r1 : r0) + 1024u * k);
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v0,
              (8u * k * uint32_t(G)) << 10, 0);
        }
        if (gl && blk + 2 < NB) {  // the image is free again: next pair
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          issue(blk / 2 + 1);
        }
      }
    }
    lane_merge<D, A>(cv, stk, depth, jj, jj + 1 == uint32_t(G), whole, key, base);
  }
}

// Lane-local subtree over chunks [first, first+n_my) of one message: returns
// its chaining value in cv (or the root output when `whole`: this lane holds
// the entire message).  Eager merges after chunk jj = ctz(jj+1), final merges
// right to left: the same tree as BLAKE3's incremental hasher.
template <int G, bool CHACHA, bool ALIGNED, int A = 2>
__device__ __forceinline__ void lane_subtree(
    uint32_t (&cv)[8], const uint8_t *msg, uint8_t *cmsg, uint64_t len,
    uint32_t first, uint32_t n_my, bool whole, const uint32_t (&key)[8],
    uint32_t base, const uint32_t (&dek)[8], uint32_t cbase = 0) {
  constexpr int D = ilog2(G);
  uint32_t stk[D > 0 ? D : 1][8];
  uint32_t depth = 0;
  for (uint32_t jj = 0; jj < n_my; ++jj) {
    const uint32_t lchunk = first + jj;           // within msg[0, len)
    const uint32_t chunk = cbase + lchunk;        // counter: absolute index
    const uint64_t coff = uint64_t(lchunk) << 10;
    const uint64_t rem = len - coff;
    const uint32_t clen = rem < 1024 ? uint32_t(rem) : 1024u;
    const uint32_t nb = clen ? (clen + 63) >> 6 : 1u;
    const bool last = jj + 1 == n_my;
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = key[i];
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t boff = b << 6;
      const uint32_t avail = clen - boff;
      uint32_t m[16];
      load_block<ALIGNED>(m, msg + coff + boff, avail);
      if constexpr (CHACHA) {
        uint32_t x[16];
        chacha_block<A>(x, dek, (chunk << 4) + b);
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] ^= x[i];
        if (avail < 64) mask_tail(m, avail);
        if (cmsg) store_block<ALIGNED>(cmsg + coff + boff, m, avail);
      }
      uint32_t fl = base;
      if (b == 0) fl |= kChunkStart;
      if (b + 1 == nb) {
        fl |= kChunkEnd;
        if (whole && n_my == 1) fl |= kRoot;
      }
      b3_compress<A>(cv, m, chunk, 0u, avail < 64 ? avail : 64u, fl);
    }
    lane_merge<D, A>(cv, stk, depth, jj, last, whole, key, base);
  }
}

// One lane writes the 32-byte result (CID or DEK) into its ref slot.  The
// slot is 16-B aligned for dense refs; index-node slots (node*bs + 64*i) may
// not be when bs % 16 != 0.
__device__ __forceinline__ void store_digest(uint8_t *dst, const uint32_t (&w)[8]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
  if ((a & 15) == 0) {
    uint4 *q = reinterpret_cast<uint4 *>(dst);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
  } else if ((a & 3) == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) reinterpret_cast<uint32_t *>(dst)[i] = w[i];
  } else {
#pragma unroll
    for (int i = 0; i < 32; ++i) dst[i] = uint8_t(w[i >> 2] >> (8 * (i & 3)));
  }
}

// Pairwise merge of the k subtree CVs in lds[0 .. 8k) (all but the last are
// perfect subtrees of one power-of-two size, so this is BLAKE3's left-complete
// tree); the last parent gets ROOT when `root`.  Every thread of the block
// calls it; on return thread 0 holds the result in p (p = its own value on
// entry when k == 1).
__device__ __forceinline__ void tree_reduce(uint32_t *lds, uint32_t k,
                                            uint32_t t, const uint32_t (&key)[8],
                                            uint32_t base, bool root,
                                            uint32_t (&p)[8]) {
  while (k > 1) {
    const uint32_t half = k >> 1, odd = k & 1u;
    if (t < half) {
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        m[i] = lds[(2 * t) * 8 + i];
        m[8 + i] = lds[(2 * t + 1) * 8 + i];
        p[i] = key[i];
      }
      b3_compress(p, m, 0u, 0u, 64u,
                  base | kParent | ((root && k == 2) ? kRoot : 0u));
    } else if (odd && t == half) {
#pragma unroll
      for (int i = 0; i < 8; ++i) p[i] = lds[(k - 1) * 8 + i];
    }
    __syncthreads();
    if (t < half + odd) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[t * 8 + i] = p[i];
    }
    __syncthreads();
    k = half + odd;
  }
}

// The same merge with four lanes per parent compression (quad layout, as
// k_quad): defined after quad_compress below.  GLFSX_QTREE=0 keeps the
// one-lane tree_reduce (A/B builds).
#ifndef GLFSX_QTREE
#define GLFSX_QTREE 1
#endif
__device__ __forceinline__ void tree_reduce_q(uint32_t *lds, uint32_t k, uint32_t t,
                              const uint32_t (&key)[8], uint32_t base, bool root,
                              uint32_t (&p)[8]);
__device__ __forceinline__ void tree_merge(uint32_t *lds, uint32_t k, uint32_t t,
                                           const uint32_t (&key)[8], uint32_t base,
                                           bool root, uint32_t (&p)[8]) {
  if (GLFSX_QTREE) tree_reduce_q(lds, k, t, key, base, root, p);
  else tree_reduce(lds, k, t, key, base, root, p);
}

#if GLFSX_WGTIME
// Phase timestamps per workgroup of the bulk passes (A/B diagnostics only,
// tools/build_variant.sh wgtime "-DGLFSX_WGTIME=1"): [start, chunks done,
// subtree done, end, HW_ID, XCC_ID, k_pass_dc entry, item fetched, DEK wait
// over (k_pass_dc CID items), 7 spare]; DEK pass at [0, 4096), CID pass at
// [4096, 8192).  s_memrealtime: 100 MHz.
__device__ uint64_t g_wgtime[8192][16];
__device__ __forceinline__ void wgt(bool chacha, uint32_t bid, int slot) {
  const uint32_t b = bid + (chacha ? 4096u : 0u);  // the pass's own workgroup number
  if (threadIdx.x == 0 && b < 8192) {
    g_wgtime[b][slot] = __builtin_amdgcn_s_memrealtime();
    if (slot == 0) {
      g_wgtime[b][4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_wgtime[b][5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
  }
}
#define WGT(bid, slot) wgt(CHACHA, bid, slot)
#else
#define WGT(bid, slot) (void)0
#endif

// A: ARX in the asm form (many waves per SIMD); false: the compiler's form,
// which issues faster when a launch leaves a SIMD one or two waves
// one LDS array: [0, 8 KiB) CV tree, then 4 waves x 8 KiB staging (ctext in
// the CHACHA pass, plaintext in the DEK pass): 40 KiB, 4 WGs per CU
template <bool CHACHA>
constexpr int kStageOf = (CHACHA ? GLFSX_LDS_CTEXT : GLFSX_LDS_LOADS) ? 4 * 512 : 0;

// State of a fused split launch (k_pass_dc).  Per (device, stream), in
// device memory (DcConst), read where it is used -- as kernel arguments
// these words would stay live in SGPRs through the whole body (the DEK/CID
// bodies then spilled SGPRs: 4 -> 33 at G = 2):
//  - ready[j] = epoch once message j's DEK is published (flags are never
//    reset: each launch has a new epoch, zero is never one);
//  - lists: two banks of kLists work-list counters, one per 128-B line
//    (k_pass_dc); launch e uses bank e & 1 and zeroes bank (e + 1) & 1 for
//    the next launch on the stream;
//  - err: a word in pinned host memory, set when a CID workgroup gave up
//    waiting for a DEK, or found no work item (the launch's results are
//    then invalid and the host fails or repeats the post);
//  - wait_ticks: that wait's bound in s_memrealtime ticks (100 MHz);
//  - skip_msg: test hook -- the DEK of this message is written but its
//    ready flag is not (~0u: none).
constexpr uint32_t kLists = 8;           // one per XCD
constexpr uint32_t kListStride = 32;     // words between counters (128 B)
struct DcConst {
  uint32_t *ready;
  uint32_t *lists;
  uint32_t *err;
  uint64_t wait_ticks;
  uint32_t skip_msg;
};
// Per launch (kernel argument): the epoch, and the messages and log2
// workgroups per message of both passes (a.n, a.split_log2, given again so
// the item search does not touch the pass arguments: reading those before
// the branch made the bodies spill SGPRs).
struct DcState {
  uint32_t epoch;
  uint32_t n;
  uint32_t sl;
  uint32_t fine_div;  // the last ceil(m / fine_div) messages of each list
                      // run their CID pass as fine items (0: none)
  const DcConst *c;
};

// Items of work list x (kLists lists, message j on list j % kLists): all DEK
// items of its m messages (2^sl each), then the CID items -- coarse (2^sl per
// message) for its first m - F messages, fine (2^(sl+1) per message, half the
// chunks per lane) for its last F.  The run-down at the end of a launch is
// then made of items half as long.
__host__ __device__ __forceinline__ uint32_t dc_list_msgs(uint32_t n, uint32_t x) {
  return n > x ? (n - x + kLists - 1u) / kLists : 0u;
}
__host__ __device__ __forceinline__ uint32_t dc_list_fine(uint32_t m, uint32_t fine_div) {
  return fine_div ? (m + fine_div - 1u) / fine_div : 0u;
}
__host__ __device__ __forceinline__ uint32_t dc_list_items(uint32_t m, uint32_t f, uint32_t sl) {
  return (2u * m + f) << sl;
}

// The DEK pass stores message j's DEK with agent-scope atomic stores, waits
// for them, then sets ready[j] = epoch; the CID workgroups of message j wait
// for that.
__device__ __forceinline__ void publish_dek(uint8_t *dst, const uint32_t (&w)[8],
                                            const DcState &d, uint64_t j) {
  publish_cv(reinterpret_cast<uint32_t *>(dst), w);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const DcConst *c = d.c;
  if (j != c->skip_msg)
    __hip_atomic_store(c->ready + j, d.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A CID item's wait for its message's DEK (k_pass_dc): from the DEK work
// items of the same launch.  Work items are taken from work lists
// (k_pass_dc), so every DEK item was taken by a workgroup that was already
// running before this one took its CID item: the wait depends only on
// running workgroups, whatever the dispatch order or other launches sharing
// the chip.  It is bounded anyway; a timeout marks the launch failed in
// d.err (the host then discards its results) and the workgroup finishes
// with whatever key it read, so counters and flags stay consistent for later
// launches.  Every thread of the workgroup calls it; dek is uniform.
__device__ __forceinline__ void dc_dek_wait(const DcState *dc, uint64_t j, uint32_t bid,
                                            const uint8_t *ref, uint32_t *lds,
                                            uint32_t (&dek)[8]) {
  (void)bid;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const DcConst *c = dc->c;  // (the DEK items this one waits for precede it in its list)
    while (__hip_atomic_load(c->ready + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
           dc->epoch) {
      __builtin_amdgcn_s_sleep(4);
      if (__builtin_amdgcn_s_memrealtime() - t0 > c->wait_ticks) {
        __hip_atomic_store(c->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    // the DEK loads below must not be hoisted above the flag load that
    // saw the epoch (a compiler barrier; the loads are agent-scope, so no
    // cache invalidate is needed)
    __atomic_signal_fence(__ATOMIC_ACQUIRE);
#if GLFSX_WGTIME
    if (bid + 4096u < 8192u) g_wgtime[bid + 4096u][8] = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i)
      lds[i] = load_cv_word(reinterpret_cast<const uint32_t *>(ref + 32) + i);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) dek[i] = __builtin_amdgcn_readfirstlane(lds[i]);
  __syncthreads();
}

// The body of one workgroup (number bid) of a pass.  FUSE: 0 = a pass of its
// own; 1 = the DEK part of k_pass_dc (publishes each DEK with its ready
// flag); 2 = the CID part (waits for its message's DEK).
template <int G, bool CHACHA, bool ALIGNED, int A, int FUSE>
__device__ __forceinline__ void pass_body(const KArgs &a, uint32_t bid, uint4 *lds_u4,
                                          const DcState *dc) {
  constexpr int kStageU4 = kStageOf<CHACHA>;
  uint32_t *lds = reinterpret_cast<uint32_t *>(lds_u4);
  WGT(bid, 0);
  // message j, sub-range sidx (split mode) = chunks [sidx*256G, +256G)
  const uint64_t j = bid >> a.split_log2;
  const uint32_t sidx = bid & ((1u << a.split_log2) - 1u);
  const uint64_t len_full = (j + 1 == a.n) ? a.last_len : a.msg_len;
  constexpr uint64_t kSpan = uint64_t(256 * G) << 10;  // bytes per workgroup
  const uint64_t c0b = uint64_t(sidx) * kSpan;
  if (sidx != 0 && c0b >= len_full) return;  // empty sub-range (uniform)
  const uint64_t len = min(len_full - c0b, kSpan);
  const bool split = len_full > kSpan;  // the message spans > 1 workgroup
  const uint32_t cbase = sidx * uint32_t(256 * G);
  const uint8_t *msg = a.src + j * a.stride + c0b;
  uint8_t *cmsg = (CHACHA && a.ctext) ? a.ctext + j * a.stride + c0b : nullptr;
  uint8_t *ref = a.refs + (j / a.ref_bf) * a.ref_stride + (j % a.ref_bf) * 64;
  const uint32_t t = threadIdx.x;

  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = a.key[i];
  uint32_t dek[8];
  if constexpr (FUSE == 2) {
    dc_dek_wait(dc, j, bid, ref, lds, dek);
  } else if constexpr (CHACHA) {
    // DEK written by the preceding pass into bytes [32,64) of this ref slot.
    const uint8_t *dp = ref + 32;
    if ((reinterpret_cast<uintptr_t>(dp) & 3) == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        dek[i] = __builtin_amdgcn_readfirstlane(
            reinterpret_cast<const uint32_t *>(dp)[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        dek[i] = __builtin_amdgcn_readfirstlane(
            uint32_t(dp[4 * i]) | (uint32_t(dp[4 * i + 1]) << 8) |
            (uint32_t(dp[4 * i + 2]) << 16) | (uint32_t(dp[4 * i + 3]) << 24));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) dek[i] = 0;
  }

  const uint32_t C = len ? uint32_t((len + 1023) >> 10) : 1u;
  const bool whole = !split && C <= uint32_t(G);
  const uint32_t first = t * G;
  const uint32_t n_my = first < C ? min(uint32_t(G), C - first) : 0u;
  uint32_t cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool fast = ALIGNED && n_my == uint32_t(G) &&
                    len >= (uint64_t(first) + G) << 10;
  // staged stores write other lanes' lines: only when the whole wave is fast
  const bool wave_fast = __ballot(fast) == ~0ull;
  if (fast) {
    if (kStageU4 && wave_fast && (cmsg || !CHACHA))  // wave-uniform
      lane_subtree_full<G, CHACHA, kStageU4 != 0, A>(
          cv, msg, cmsg, first, whole, key, a.base, dek,
          lds_offset(lds_u4 + 512 + (t >> 6) * 512), uint32_t(len), cbase);
    else
      lane_subtree_full<G, CHACHA, false, A>(cv, msg, cmsg, first, whole, key,
                                             a.base, dek, 0u, 0u, cbase);
  } else if (n_my) {
    lane_subtree<G, CHACHA, ALIGNED, A>(cv, msg, cmsg, len, first, n_my, whole,
                                     key, a.base, dek, cbase);
  }
  if (whole) {  // uniform: depends on len only; lane 0 holds the root output
    if (t == 0) {
      if constexpr (FUSE == 1) publish_dek(ref + a.out_off, cv, *dc, j);
      else store_digest(ref + a.out_off, cv);
    }
    return;
  }
  const uint32_t active = (C + G - 1) / G;
  if (t < active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
  }
  __syncthreads();
  WGT(bid, 1);
  tree_merge(lds, active, t, key, a.base, !split, cv);
  WGT(bid, 2);
  if (!split) {
    if (t == 0) {
      if constexpr (FUSE == 1) publish_dek(ref + a.out_off, cv, *dc, j);
      else store_digest(ref + a.out_off, cv);
    }
    return;
  }
  // split (uniform): this workgroup's subtree CV to scratch; the message's
  // last workgroup merges the W = ceil(len / span) CVs (left-complete tree,
  // ROOT on the last parent) and resets the counter for the next launch
  const uint64_t wbase = j << a.split_log2;
  if (t == 0) publish_cv(a.scratch + (wbase + sidx) * 8, cv);
  const uint32_t W = uint32_t((len_full + kSpan - 1) / kSpan);
  // the arrival flag lives in the (now idle) staging image: one more LDS
  // word would take the kernel past 40 KiB, i.e. from four workgroups per
  // CU to three (160 KiB / 40 KiB)
  uint32_t *flag;
  if constexpr (kStageU4 != 0) {
    flag = reinterpret_cast<uint32_t *>(lds_u4 + 512);
  } else {
    __shared__ uint32_t s_flag;
    flag = &s_flag;
  }
  if (!arrive_last(a.cnt + j, W, t, flag)) {
    WGT(bid, 3);
    return;
  }
  if (t < W) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      cv[i] = load_cv_word(a.scratch + (wbase + t) * 8 + i);
      lds[t * 8 + i] = cv[i];
    }
  }
  __syncthreads();
  tree_merge(lds, W, t, key, a.base, true, cv);
  if (t == 0) {
    if constexpr (FUSE == 1) publish_dek(ref + a.out_off, cv, *dc, j);
    else store_digest(ref + a.out_off, cv);
    a.cnt[j] = 0;
  }
  WGT(bid, 3);
}

// Clock probe of the bulk passes (glfsx_clock_probe): once a process has
// called it, every k_pass workgroup adds its lifetime in shader-clock cycles
// (s_memtime) and in 100 MHz ticks (s_memrealtime) to these two device
// words (KArgs::clk), so a caller reads the clock the chip held over the
// launches since its reset: cycles / ticks x 100 MHz.  Two scalar timer
// reads per wave and, when on, two atomic adds per workgroup (thread 0).
// The words are per device, not per launch: k_pass launches of other
// callers on the same device in that window are counted too.
__device__ unsigned long long g_clk[2];

template <int G, bool CHACHA, bool ALIGNED, int A = 2>
__global__ __launch_bounds__(256) void k_pass(KArgs a) {
  __shared__ uint4 lds_u4[512 + kStageOf<CHACHA>];
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  pass_body<G, CHACHA, ALIGNED, A, 0>(a, blockIdx.x, lds_u4, nullptr);
  if (threadIdx.x == 0 && a.clk) {
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_add(&a.clk[0], (unsigned long long)(c1 - c0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&a.clk[1], (unsigned long long)(r1 - r0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Both passes of a split-mode post in one launch: the DEK items run the DEK
// pass (a), the CID items the ChaCha20+CID pass (b), each CID item starting
// as soon as its message's DEK is published, so the CID pass fills the DEK
// pass's tail instead of waiting for the whole launch to drain.
//
// Work is taken from kLists lists, not by blockIdx: list x holds the items
// of messages j = x, x + 8, ... -- all their DEK items, then all their CID
// items -- and hands them out in that order through one device-wide
// counter.  A workgroup takes from the list of its own XCD first and moves
// on to the others when that one is used up.  A CID item then only ever
// waits for DEK items of its own list, which were handed out before it to
// workgroups that were already running: the wait needs no assumption about
// the order in which the hardware dispatches workgroups, how it places them
// on XCDs, or other launches (streams, processes) occupying the CUs.  Every
// workgroup finds an item (as many items as workgroups, each handed out
// once).  One counter per XCD keeps the start of the launch from queueing
// all 1024 first workgroups on one word (a single counter cost config 2
// 1.7 %), and keeps a message's DEK and CID items on one XCD.
template <int G>
__global__ __launch_bounds__(256) void k_pass_dc(KArgs a, KArgs b, KArgs c, DcState d) {
  __shared__ uint4 lds_u4[512 + kStageOf<true>];
  uint32_t *lds = reinterpret_cast<uint32_t *>(lds_u4);
  // thread 0 finds the item and leaves (workgroup number within its pass,
  // kind: 0 DEK, 1 CID, 2 none) in LDS; only those two words stay live
  if (threadIdx.x == 0) {
#if GLFSX_WGTIME
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t sl = d.sl;
    const uint32_t n = d.n;
    uint32_t *bank = d.c->lists + (d.epoch & 1u) * kLists * kListStride;
    if (blockIdx.x == 0) {  // the next launch's counters (this stream's last
      uint32_t *nb = d.c->lists + ((d.epoch + 1u) & 1u) * kLists * kListStride;
      for (uint32_t x = 0; x < kLists; ++x)  // user of them has completed)
        __hip_atomic_store(nb + x * kListStride, 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & (kLists - 1u);
    uint32_t bid = 0, kind = 2;
    for (uint32_t k = 0; k < kLists; ++k) {
      const uint32_t x = (xcc + k) & (kLists - 1u);
      const uint32_t msgs = dc_list_msgs(n, x);
      if (msgs == 0) continue;
      const uint32_t f = G > 1 ? dc_list_fine(msgs, d.fine_div) : 0u;
      const uint32_t t = __hip_atomic_fetch_add(bank + x * kListStride, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t nd = msgs << sl, nc = (msgs - f) << sl;
      if (t < nd + nc) {  // DEK, or coarse CID: the list's message u >> sl
        const uint32_t u = t < nd ? t : t - nd;
        bid = ((x + kLists * (u >> sl)) << sl) | (u & ((1u << sl) - 1u));
        kind = t < nd ? 0u : 1u;
        break;
      }
      if (t < dc_list_items(msgs, f, sl)) {  // fine CID: 2^(sl+1) per message
        const uint32_t u = t - nd - nc;
        bid = ((x + kLists * (msgs - f + (u >> (sl + 1u)))) << (sl + 1u)) |
              (u & ((2u << sl) - 1u));
        kind = 3u;
        break;
      }
    }
    lds[0] = bid;
    lds[1] = kind;
#if GLFSX_WGTIME
    if (kind != 2 && bid + (kind ? 4096u : 0u) < 8192u) {  // kernel entry, item fetched
      g_wgtime[bid + (kind ? 4096u : 0u)][6] = t_entry;
      g_wgtime[bid + (kind ? 4096u : 0u)][7] = __builtin_amdgcn_s_memrealtime();
    }
#endif
  }
  __syncthreads();
  const uint32_t bid = __builtin_amdgcn_readfirstlane(lds[0]);
  const uint32_t kind = __builtin_amdgcn_readfirstlane(lds[1]);
  __syncthreads();
  if (kind == 2) {  // no item left anywhere: counters were not at zero
    if (threadIdx.x == 0)
      __hip_atomic_store(d.c->err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (kind == 0) {
    pass_body<G, false, true, 2, 1>(a, bid, lds_u4, &d);
  } else if (kind == 1) {
    pass_body<G, true, true, 2, 2>(b, bid, lds_u4, &d);
  } else {
    if constexpr (G > 1) pass_body<G / 2, true, true, 2, 2>(c, bid, lds_u4, &d);
  }
}

// ---- Latency mode, BLAKE3-only passes: four lanes per chaining state ----
// A BLAKE3 chunk is 16 dependent compressions; in a launch that leaves one
// wave per SIMD their latency is the pass's latency.  Here lane q of a quad
// holds column q of the 4x4 state (a = v[q], b = v[4+q], c = v[8+q],
// d = v[12+q]) and runs one G per step; the diagonal step rotates rows b, c,
// d across the quad by DPP quad_perm and back.  The 16 message words sit in
// the quad's 64-B LDS slot; lane q reads the four it needs per round (words
// s_r[2q], s_r[2q+1], s_r[8+2q], s_r[9+2q]) at offsets fixed per lane.  A
// chaining value ends up as cv[q] = a ^ c, cv[4+q] = b ^ d in lane q.
// 1024-lane workgroups: 256 quads = 256 chunks (256 KiB) per workgroup; the
// workgroup's subtree is merged pairwise through the slots (the same
// left-complete tree as tree_reduce), and the last workgroup of a split
// message merges the workgroups' CVs.
__device__ __forceinline__ uint32_t qrot1(uint32_t x) {  // lane q <- lane q+1
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x39, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t qrot2(uint32_t x) {  // lane q <- lane q+2
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t qrot3(uint32_t x) {  // lane q <- lane q+3
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x93, 0xF, 0xF, true));
}

#define QG(a, b, c, d, x, y) \
  a = a + b + (x);           \
  d = rotr(d ^ a, 16);       \
  c = c + d;                 \
  b = rotr(b ^ c, 12);       \
  a = a + b + (y);           \
  d = rotr(d ^ a, 8);        \
  c = c + d;                 \
  b = rotr(b ^ c, 7);

// One round (column step, diagonal step) in quad layout as one asm block
// (round 6).  tools/chainlat.hip measured the chain's
// instructions at one wave per SIMD: a dependent v_add/v_xor/v_alignbit
// chain issues every ~5-8 cycles and the wave as a whole about one VALU
// instruction per ~4.8 cycles whatever the dependences, so the round costs
// what it issues.  Here the three row rotations per step change are
// v_mov_b32_dpp placed where their sources are already two instructions old
// (no wait states), the diagonal step's first add is split as t = a + m2
// (issued in the column step) then v_add_u32_dpp a = rot1(b) + t, and one
// s_nop 0 per step change covers the one DPP read of a just-written b.
// The compiler's form folded the rotations into the consumers instead and
// needed ~5.6 wait states per round for them (tools/qchain.hip: 1312 -> 1233
// cycles per compression with the loads below, 1 wave per SIMD).
// In: a, b, c, d unrotated (lane q holds column q), t = a + m0, m1..m3.
//   quad_perm [1,2,3,0]: lane q <- q+1; [2,3,0,1]: q+2; [3,0,1,2]: q+3.
#define QROUND_ASM                                                              \
  "v_add_u32 %0, %1, %4\n"                                                      \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %5\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_add_u32 %4, %0, %6\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_mov_b32_dpp %3, %3 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"       \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_mov_b32_dpp %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"       \
  "s_nop 0\n"                                                                   \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_mov_b32_dpp %1, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"       \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %7\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_mov_b32_dpp %3, %3 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"       \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_mov_b32_dpp %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"       \
  "s_nop 0\n"                                                                   \
  "v_mov_b32_dpp %1, %1 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"

#ifndef GLFSX_QASM
#define GLFSX_QASM 1
#endif

// Every row rotation folded into its first consumer (v_add_u32_dpp /
// v_xor_b32_dpp, the permute on src0): b, c, d stay in the diagonal frame
// (lanes q+1, q+2, q+3) from a diagonal step until the next column step
// reads them back; a never moves.  26 ARX instructions, one filler add and
// two s_nop 0 per round (a DPP read of a VGPR written one or two
// instructions before needs two wait states) against QROUND_ASM's 33.
// In: t = a + m0; the state in the column frame (QCOL0) or the diagonal
// frame (QCOL).  Out: the diagonal frame.  tools/qchain.hip v4: 1118 vs
// 1233 cycles per compression at one wave per SIMD; PostBlob 4 KiB p50
// 40.4 -> 37.7 us, config 2's index-node kernels 62.8 -> 57.9 us
// (scripts/ab_qfold.sh, profiles/r6/ab_qfold/).  GLFSX_QFOLD=0 (A/B builds):
// QROUND_ASM.
#ifndef GLFSX_QFOLD
#define GLFSX_QFOLD 1
#endif
#define QCOL0_ASM                                                               \
  "v_add_u32 %0, %1, %4\n"                                                      \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"
#define QCOL_ASM                                                                \
  "s_nop 0\n"                                                                   \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %3, %3, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32_dpp %2, %2, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %1, %1, %2 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %1, %1, %1, 12\n"
#define QREST_ASM                                                               \
  "v_add3_u32 %0, %0, %1, %5\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_add_u32 %4, %0, %6\n"                                                      \
  "s_nop 0\n"                                                                   \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %3, %3, %0 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32_dpp %2, %2, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %1, %1, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %7\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 7\n"

// One compression in quad layout.  addr[4r+k]: LDS byte address of the k-th
// message word this lane uses in round r.  On return (a, b) = (cv[q], cv[4+q]).
// Every lane of a quad must be active (the rotations read the other three).
// quad_compress_m: m holds round 0's four words, already read; with PF, the
// four words at nxt (the next compression's round 0) are read during round 6
// and left in m, so a chain of compressions over a static LDS image waits
// for LDS only once (k_one).
typedef const __attribute__((address_space(3))) uint32_t *lds_word;
template <bool PF>
__device__ __forceinline__ void quad_compress_m(uint32_t &a, uint32_t &b, uint32_t c,
                                                uint32_t d, const uint32_t (&addr)[28],
                                                uint32_t (&m)[4], const uint32_t *nxt) {
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t n[4] = {0, 0, 0, 0};
    if (r < 6) {
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] = *reinterpret_cast<lds_word>(addr[4 * r + 4 + k]);
    } else if (PF) {
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] = *reinterpret_cast<lds_word>(nxt[k]);
    }
    uint32_t t = a + m[0];
    if (!GLFSX_QFOLD)
      asm volatile(QROUND_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                   : "v"(m[1]), "v"(m[2]), "v"(m[3]));
    else if (r == 0)
      asm volatile(QCOL0_ASM QREST_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                   : "v"(m[1]), "v"(m[2]), "v"(m[3]));
    else
      asm volatile(QCOL_ASM QREST_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                   : "v"(m[1]), "v"(m[2]), "v"(m[3]));
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = n[k];
  }
  if (!GLFSX_QFOLD) {
    a ^= c;
    b ^= d;
  } else {  // back from the diagonal frame: a ^= c_q, b = b_q ^ d_q
    uint32_t u;
    asm volatile("v_xor_b32_dpp %0, %2, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
                 "s_nop 1\n"
                 "v_mov_b32_dpp %4, %1 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"
                 "v_xor_b32_dpp %1, %3, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&v"(u));
  }
}

__device__ __forceinline__ void quad_compress(uint32_t &a, uint32_t &b,
                                              uint32_t c, uint32_t d,
                                              const uint32_t (&addr)[28]) {
#if GLFSX_QASM
  // round r+1's four words are read while round r runs
  uint32_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = *reinterpret_cast<lds_word>(addr[k]);
  quad_compress_m<false>(a, b, c, d, addr, m, nullptr);
#else
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const uint32_t m0 = *reinterpret_cast<lds_word>(addr[4 * r]);
    const uint32_t m1 = *reinterpret_cast<lds_word>(addr[4 * r + 1]);
    const uint32_t m2 = *reinterpret_cast<lds_word>(addr[4 * r + 2]);
    const uint32_t m3 = *reinterpret_cast<lds_word>(addr[4 * r + 3]);
    QG(a, b, c, d, m0, m1);
    b = qrot1(b);
    c = qrot2(c);
    d = qrot3(d);
    QG(a, b, c, d, m2, m3);
    b = qrot3(b);
    c = qrot2(c);
    d = qrot1(d);
  }
  a ^= c;
  b ^= d;
#endif
}

__device__ __forceinline__ uint32_t qsel(uint32_t q, uint32_t x0, uint32_t x1,
                                         uint32_t x2, uint32_t x3) {
  return q == 0 ? x0 : q == 1 ? x1 : q == 2 ? x2 : x3;
}

// The 28 LDS addresses of a 64-B slot at byte `slot` for lane q; with x
// (a multiple of 4), word w of the slot lives at word w ^ x (the block
// slots of k_quad, below).
__device__ __forceinline__ void quad_addrs(uint32_t (&addr)[28], uint32_t slot,
                                           uint32_t q, uint32_t x = 0) {
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    constexpr int kk[4] = {0, 1, 8, 9};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = qsel(q, kSched.s[r][kk[k]], kSched.s[r][kk[k] + 2],
                              kSched.s[r][kk[k] + 4], kSched.s[r][kk[k] + 6]);
      addr[4 * r + k] = slot + 4u * (w ^ x);
    }
  }
}

// tree_reduce with four lanes per parent: the k CVs at lds[0 .. 8k) merge
// pairwise, parent i reading its message (CV 2i || CV 2i+1) in place as the
// 64-B slot at lds + 16i words, 64 parents per step (256 lanes).  A one-lane
// parent is a chain of ~700 dependent instructions; in quad layout it is
// ~200 plus LDS reads, so the 8 levels of a 256-lane subtree (pass_body's
// per-workgroup merge, 13-18 us in round 2's per-workgroup timeline) take
// 9 short steps.  Same tree and flags as tree_reduce (ROOT on the last
// parent when `root`); on return thread 0 holds the result in p.
__device__ __forceinline__ void tree_reduce_q(uint32_t *lds, uint32_t k, uint32_t t,
                              const uint32_t (&key)[8], uint32_t base, bool root,
                              uint32_t (&p)[8]) {
  const uint32_t q = t & 3u, quad = t >> 2;
  const uint32_t kq_lo = qsel(q, key[0], key[1], key[2], key[3]);
  const uint32_t kq_hi = qsel(q, key[4], key[5], key[6], key[7]);
  const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
  uint32_t rel[28];
  quad_addrs(rel, lds_offset(lds), q);
  while (k > 1) {  // uniform
    const uint32_t half = k >> 1, odd = k & 1u;
    const uint32_t fl = base | kParent | ((root && k == 2) ? kRoot : 0u);
    const uint32_t dq = qsel(q, 0u, 0u, 64u, fl);
    uint32_t rl[2] = {0, 0}, rh[2] = {0, 0};
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {  // half <= 128 parents: <= 2 per quad
      const uint32_t i = quad + 64u * r;
      if (i < half) {  // quad-uniform
        uint32_t addr[28];
#pragma unroll
        for (int x = 0; x < 28; ++x) addr[x] = rel[x] + 64u * i;
        uint32_t cl = kq_lo, ch = kq_hi;
        quad_compress(cl, ch, ivq, dq, addr);
        rl[r] = cl;
        rh[r] = ch;
      }
    }
    // the odd CV moves from index k-1 to index half (its words are not
    // among the slots being rewritten: (k-1)*8 >= half*8)
    const uint32_t ov = (odd && t < 8) ? lds[(k - 1) * 8 + t] : 0u;
    __syncthreads();  // every slot of this level has been read
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {
      const uint32_t i = quad + 64u * r;
      if (i < half) {
        lds[i * 8 + q] = rl[r];
        lds[i * 8 + 4 + q] = rh[r];
      }
    }
    if (odd && t < 8) lds[half * 8 + t] = ov;
    __syncthreads();
    k = half + odd;
  }
  if (t == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = lds[i];
  }
}

// QPW quads (chunks) per workgroup: 256 (1024 lanes, 4 waves per SIMD) or
// 64 (256 lanes, one wave per SIMD: the chain runs at its latency instead
// of sharing its SIMD with three more waves; a 2 MiB node spreads over 32
// CUs instead of 8).
template <int QPW>
__global__ __launch_bounds__(QPW * 4) void k_quad(KArgs a) {
  // Block slots of the chunk phase: one 64-B slot per quad; QPW = 64 has a
  // second set QPW x 64 B further on (block b+1 is stored while block b
  // compresses, and its first words are read in block b's last round).
  // The subtree merges use the first set's 64-B slots as parent slots.
  constexpr bool kTwo = QPW == 64;
  __shared__ uint4 slots[QPW * (kTwo ? 8 : 4)];
  __shared__ uint32_t passbuf[8];       // the odd subtree passing up a level
  const uint32_t tid = threadIdx.x, q = tid & 3u, quad = tid >> 2;
  const uint64_t j = blockIdx.x >> a.split_log2;
  const uint32_t sidx = blockIdx.x & ((1u << a.split_log2) - 1u);
  const uint64_t len = (j + 1 == a.n) ? a.last_len : a.msg_len;
  constexpr uint64_t kSpan = uint64_t(QPW) << 10;
  const uint64_t c0b = uint64_t(sidx) * kSpan;
  if (sidx != 0 && c0b >= len) return;  // empty sub-range (uniform)
  const bool whole = len <= kSpan;       // the message fits this workgroup
  const uint64_t mylen = min(len - c0b, kSpan);
  const uint32_t cnt = mylen ? uint32_t((mylen + 1023) >> 10) : 1u;
  const uint8_t *msg = a.src + j * a.stride + c0b;
  const uint32_t slot = lds_offset(slots + quad * 4);
  const uint32_t kq_lo = qsel(q, a.key[0], a.key[1], a.key[2], a.key[3]);
  const uint32_t kq_hi = qsel(q, a.key[4], a.key[5], a.key[6], a.key[7]);
  const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
  uint32_t addr[28];
  quad_addrs(addr, slot, q);
  uint32_t cl = kq_lo, ch = kq_hi;  // this quad's chaining value
  if (quad < cnt) {
    const uint64_t coff = uint64_t(quad) << 10;
    const uint32_t clen = uint32_t(min<uint64_t>(mylen - coff, 1024));
    const uint32_t nb = clen ? (clen + 63) >> 6 : 1u;
    const uint32_t ctr = sidx * uint32_t(QPW) + quad;  // chunk counter (messages < 4 GiB)
    const uint8_t *cp = msg + coff + 16u * q;
    uint4 blk[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      blk[b] = make_uint4(0, 0, 0, 0);
      const int32_t avail = int32_t(clen) - 64 * b - 16 * int32_t(q);
      if (avail >= 16) {
        blk[b] = *reinterpret_cast<const uint4 *>(cp + 64 * b);
      } else if (avail > 0) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int i = 0; i < avail; ++i) w[i >> 2] |= uint32_t(cp[64 * b + i]) << (8 * (i & 3));
        blk[b] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    // The quad's four lanes are one wave's, and a wave's LDS instructions
    // are performed in issue order: a compression's reads after its
    // block's store see it, and a later store into the slot comes after
    // them, so neither needs a wait (round 5 waited for both: two LDS round
    // trips per block on the chain); the empty asm keeps the compiler's
    // order.
    // Block slots are word-swizzled: word w of quad i's slot sits at word
    // w ^ x_i, x_i = 4 ((i >> 1) & 3), so the eight quads of a 32-lane LDS
    // group (ds_read_b32 banks = word mod 32) reading the same word hit
    // eight banks instead of two (plain 64-B slots: 4-way conflicts on every
    // message read); a lane's 16-B block store stays one aligned granule.
    // (QPW = 256 keeps plain slots: a second 28-address set would spill the
    // 1024-lane workgroup's 128 registers)
    const uint32_t x = kTwo ? 4u * ((quad >> 1) & 3u) : 0u;
    const uint32_t gq = 16u * (q ^ (x >> 2));  // this lane's granule in a slot
    constexpr uint32_t kB = kTwo ? QPW * 64u : 0u;  // the second slot set
    uint32_t caddr[28];
    if constexpr (kTwo) {
      quad_addrs(caddr, slot, q, x);
#pragma unroll
      for (int k = 0; k < 28; ++k) asm volatile("" : "+v"(caddr[k]));  // kept, not rebuilt per read
    }
    uint32_t m[4];
    if constexpr (kTwo) {
      *reinterpret_cast<lds_u32x4 *>(slot + gq) =
          u32x4{blk[0].x, blk[0].y, blk[0].z, blk[0].w};
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 4; ++k) m[k] = *reinterpret_cast<lds_word>(caddr[k]);
    }
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      if (uint32_t(b) < nb) {
        const bool more = uint32_t(b) + 1 < nb;
        if constexpr (kTwo) {
          if (b + 1 < 16 && more)
            *reinterpret_cast<lds_u32x4 *>(slot + kB * ((b + 1) & 1) + gq) =
                u32x4{blk[(b + 1) & 15].x, blk[(b + 1) & 15].y, blk[(b + 1) & 15].z,
                      blk[(b + 1) & 15].w};
        } else {
          *reinterpret_cast<lds_u32x4 *>(slot + gq) =
              u32x4{blk[b].x, blk[b].y, blk[b].z, blk[b].w};
        }
        asm volatile("" ::: "memory");
        const uint32_t blen = min(clen - min(clen, 64u * b), 64u);
        uint32_t fl = a.base;
        if (b == 0) fl |= kChunkStart;
        if (uint32_t(b) + 1 == nb) {
          fl |= kChunkEnd;
          if (whole && cnt == 1) fl |= kRoot;
        }
        const uint32_t dq = qsel(q, ctr, 0u, blen, fl);
        if constexpr (kTwo) {
          uint32_t ab[28], nxt[4];
#pragma unroll
          for (int k = 0; k < 28; ++k) ab[k] = caddr[k] + kB * (b & 1);
          const uint32_t noff = more ? kB * ((b + 1) & 1) : kB * (b & 1);
#pragma unroll
          for (int k = 0; k < 4; ++k) nxt[k] = caddr[k] + noff;
          quad_compress_m<true>(cl, ch, ivq, dq, ab, m, nxt);
        } else {
          quad_compress(cl, ch, ivq, dq, addr);
        }
        asm volatile("" ::: "memory");
      }
    }
  }
  // the workgroup's subtree: pairwise through the slots
  uint32_t count = cnt;
  while (count > 1) {  // uniform
    const uint32_t half = count >> 1, odd = count & 1u;
    __syncthreads();  // slots of the previous level have been read
    if (quad < count) {
      if (odd && quad == count - 1) {
        passbuf[q] = cl;
        passbuf[4 + q] = ch;
      } else {
        uint32_t *ps = reinterpret_cast<uint32_t *>(slots + (quad >> 1) * 4);
        ps[(quad & 1u) * 8 + q] = cl;
        ps[(quad & 1u) * 8 + 4 + q] = ch;
      }
    }
    __syncthreads();
    if (quad < half) {
      const uint32_t fl = a.base | kParent | ((whole && count == 2) ? kRoot : 0u);
      cl = kq_lo;
      ch = kq_hi;
      const uint32_t dq = qsel(q, 0u, 0u, 64u, fl);
      quad_compress(cl, ch, ivq, dq, addr);
    } else if (odd && quad == half) {
      cl = passbuf[q];
      ch = passbuf[4 + q];
    }
    count = half + odd;
  }
  uint32_t *const out = reinterpret_cast<uint32_t *>(
      a.refs + (j / a.ref_bf) * a.ref_stride + (j % a.ref_bf) * 64 + a.out_off);
  if (whole) {
    if (quad == 0) {  // lanes 0-3: words q and 4+q of the result
      out[q] = cl;
      out[4 + q] = ch;
    }
    return;
  }
  // split: subtree CV to scratch; the message's last workgroup merges the W
  // CVs through the slots exactly like its own subtree (ROOT at the top)
  const uint64_t wbase = j << a.split_log2;
  if (tid < 64) {  // wave 0: quad 0's CV into lane 0, which stores it and
                   // then releases it (arrive_last) in program order
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] = __builtin_amdgcn_readlane(cl, k);
      w[4 + k] = __builtin_amdgcn_readlane(ch, k);
    }
    if (tid == 0) publish_cv(a.scratch + (wbase + sidx) * 8, w);
  }
  const uint32_t W = uint32_t((len + kSpan - 1) / kSpan);
  __shared__ uint32_t s_flag;
  if (!arrive_last(a.cnt + j, W, tid, &s_flag)) return;
  if (quad < W) {
    cl = load_cv_word(a.scratch + (wbase + quad) * 8 + q);
    ch = load_cv_word(a.scratch + (wbase + quad) * 8 + 4 + q);
  }
  count = W;
  while (count > 1) {  // uniform
    const uint32_t half = count >> 1, odd = count & 1u;
    __syncthreads();
    if (quad < count) {
      if (odd && quad == count - 1) {
        passbuf[q] = cl;
        passbuf[4 + q] = ch;
      } else {
        uint32_t *ps = reinterpret_cast<uint32_t *>(slots + (quad >> 1) * 4);
        ps[(quad & 1u) * 8 + q] = cl;
        ps[(quad & 1u) * 8 + 4 + q] = ch;
      }
    }
    __syncthreads();
    if (quad < half) {
      const uint32_t fl = a.base | kParent | (count == 2 ? kRoot : 0u);
      cl = kq_lo;
      ch = kq_hi;
      const uint32_t dq = qsel(q, 0u, 0u, 64u, fl);
      quad_compress(cl, ch, ivq, dq, addr);
    } else if (odd && quad == half) {
      cl = passbuf[q];
      ch = passbuf[4 + q];
    }
    count = half + odd;
  }
  if (quad == 0) {
    out[q] = cl;
    out[4 + q] = ch;
    if (q == 0) a.cnt[j] = 0;
  }
}

// ---- One-shot posts: a whole message of <= kMaxOneLen bytes per workgroup ----
// The message is staged once into LDS (zero padded to 64 B), then
//   DEK  : quad i hashes chunk i from the image (k_quad's quad layout, the
//          16 blocks' LDS addresses are immediates), the quads' CVs merge
//          pairwise through `tslot` (left-complete tree, ROOT at the top);
//   ctext: lane t makes keystream block t (+ k * lanes) with the DEK and XORs
//          it into the image in place (tail bytes masked: the image past len
//          stays zero, as BLAKE3's last block needs), then stores it out;
//   CID  : the same quad hash over the image, now ctext.
// QUADS = 16 (one wave: messages <= 16 KiB) or 64 (four waves).
// Messages of up to kMaxMedLen bytes span several such workgroups (64 KiB
// each) in two launches, k_med_dek and k_med_cid (below).

// The one-shot image's 16-B granules are swizzled per 1 KiB chunk: granule
// g sits at g ^ ((g >> 6) & 3), i.e. word w of a chunk c's block at word
// w ^ 4 (c & 3) of that block.  The quads of a 32-lane LDS group read the
// same word of their chunks (1 KiB apart, so one bank unswizzled: 4-way at
// 4 KiB, 8-way at 16 KiB and up); swizzled it is 2-way at most.  Every
// access to the image goes through img_g.
__device__ __forceinline__ uint32_t img_g(uint32_t g) { return g ^ ((g >> 6) & 3u); }

// Quad `quad` hashes chunk `quad` of the image (len bytes from the image
// start; chunk counter ctr0 + quad); root: the image is the whole message.
__device__ __forceinline__ void one_chunks(uint32_t &cl, uint32_t &ch, uint32_t img,
                                           uint32_t len, uint32_t ctr0, bool root,
                                           uint32_t kq_lo, uint32_t kq_hi, uint32_t ivq,
                                           uint32_t base, uint32_t q, uint32_t quad,
                                           const uint32_t (&rel)[28]) {
  const uint32_t C = len ? (len + 1023) >> 10 : 1u;
  cl = kq_lo;
  ch = kq_hi;
  if (quad < C) {
    const uint32_t clen = min(len - min(len, quad << 10), 1024u);
    const uint32_t nb = clen ? (clen + 63) >> 6 : 1u;
    // the chunk's 28 word addresses once (opaque to the optimiser, which
    // otherwise rebuilt each from the lane's offset with an add per read);
    // block b's reads carry its 64 b as the instruction offset
    uint32_t addr[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) {
      addr[k] = img + (quad << 10) + (rel[k] ^ (16u * (quad & 3u)));  // (img_g)
      asm volatile("" : "+v"(addr[k]));
    }
    uint32_t m[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = *reinterpret_cast<lds_word>(addr[k]);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      if (uint32_t(b) < nb) {
        const uint32_t blen = min(clen - min(clen, 64u * b), 64u);
        uint32_t fl = base;
        if (b == 0) fl |= kChunkStart;
        if (uint32_t(b) + 1 == nb) {
          fl |= kChunkEnd;
          if (root && C == 1) fl |= kRoot;
        }
        const uint32_t dq = qsel(q, ctr0 + quad, 0u, blen, fl);
        uint32_t ab[28], nxt[4];
#pragma unroll
        for (int k = 0; k < 28; ++k) ab[k] = addr[k] + 64u * b;
        // the next block's round-0 words (this block's again after the last)
        const uint32_t nb_off = uint32_t(b) + 1 < nb ? 64u * (b + 1) : 64u * b;
#pragma unroll
        for (int k = 0; k < 4; ++k) nxt[k] = addr[k] + nb_off;
        quad_compress_m<true>(cl, ch, ivq, dq, ab, m, nxt);
      }
    }
  }
}

// Pairwise merge of the `count` CVs held by quads 0..count-1 (left-complete
// tree) through the parent slots at ts; ROOT on the top parent if root.
// Every thread of the workgroup calls it (count is uniform).
__device__ __forceinline__ void one_tree(uint32_t &cl, uint32_t &ch, uint32_t count,
                                         bool root, uint32_t ts, uint32_t *passbuf,
                                         uint32_t kq_lo, uint32_t kq_hi, uint32_t ivq,
                                         uint32_t base, uint32_t q, uint32_t quad,
                                         const uint32_t (&rel)[28]) {
  while (count > 1) {  // uniform
    const uint32_t half = count >> 1, odd = count & 1u;
    __syncthreads();  // the previous level's slots have been read
    if (quad < count) {
      if (odd && quad == count - 1) {
        passbuf[q] = cl;
        passbuf[4 + q] = ch;
      } else {
        // left child: words 0-7 of the parent's slot, right child: 8-15
        const uint32_t sa = ts + ((quad >> 1) << 6) + ((quad & 1u) << 5) + 4u * q;
        *reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(sa) = cl;
        *reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(sa + 16u) = ch;
      }
    }
    __syncthreads();
    if (quad < half) {
      const uint32_t fl = base | kParent | ((root && count == 2) ? kRoot : 0u);
      cl = kq_lo;
      ch = kq_hi;
      const uint32_t dq = qsel(q, 0u, 0u, 64u, fl);
      uint32_t addr[28];
#pragma unroll
      for (int k = 0; k < 28; ++k) addr[k] = ts + (quad << 6) + rel[k];
      quad_compress(cl, ch, ivq, dq, addr);
    } else if (odd && quad == half) {
      cl = passbuf[q];
      ch = passbuf[4 + q];
    }
    count = half + odd;
  }
}

// BLAKE3 (keyed when base has kKeyed) of the image as a whole message, or as
// the subtree of chunks [ctr0, ctr0 + chunks) when !root.  Result in quad 0:
// lane q holds words q (cl) and 4+q (ch).
__device__ __forceinline__ void one_hash(uint32_t &cl, uint32_t &ch, uint32_t img,
                                         uint32_t ts, uint32_t *passbuf,
                                         uint32_t len, const uint32_t (&key)[8],
                                         uint32_t base, uint32_t q, uint32_t quad,
                                         const uint32_t (&rel)[28], uint32_t ctr0 = 0,
                                         bool root = true) {
  const uint32_t kq_lo = qsel(q, key[0], key[1], key[2], key[3]);
  const uint32_t kq_hi = qsel(q, key[4], key[5], key[6], key[7]);
  const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
  one_chunks(cl, ch, img, len, ctr0, root, kq_lo, kq_hi, ivq, base, q, quad, rel);
  const uint32_t C = len ? (len + 1023) >> 10 : 1u;
  one_tree(cl, ch, C, root, ts, passbuf, kq_lo, kq_hi, ivq, base, q, quad, rel);
}

// Stage bytes [0, len) of a message into the image, zero padded to a whole
// 64-B block (one block when empty): bytes at and past `present` read as
// zero (an index node posted from its refs alone).  dcopy (nullable): the
// staged image is also stored there (the medium path's device copy).
// Every lane's loads are issued before any is waited for: the source is
// the caller's pinned staging, one PCIe round trip (~1.7 us) per wave of
// loads, which a loop that waits per iteration paid 4x at 4 KiB and 16x at
// 16 KiB.  padded <= 16 x LANES x 16 B (k_one<16>: 16 KiB, k_one<64> and a
// k_med span: 64 KiB).
template <int LANES>
__device__ __forceinline__ void one_stage(uint4 *img_u4, const uint8_t *src, uint32_t len,
                                          uint32_t present, uint8_t *dcopy) {
  const uint32_t padded = len ? (len + 63) & ~63u : 64u;
  const uint32_t have = min(len, present);
  constexpr int IT = 16;
  uint4 v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const uint32_t p = (threadIdx.x + uint32_t(i) * LANES) * 16u;
    v[i] = make_uint4(0, 0, 0, 0);
    if (p + 16u <= have) v[i] = *reinterpret_cast<const uint4 *>(src + p);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const uint32_t p = (threadIdx.x + uint32_t(i) * LANES) * 16u;
    if (p < padded) {
      if (p < have && p + 16u > have) {  // the one partial granule
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; p + k < have; ++k) w[k >> 2] |= uint32_t(src[p + k]) << (8 * (k & 3));
        v[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
      img_u4[img_g(p >> 4)] = v[i];
      if (dcopy) *reinterpret_cast<uint4 *>(dcopy + p) = v[i];
    }
  }
}

// ChaCha20 (key dek, block counter kb0 + local block) XOR of the image's
// first len bytes in place; the tail is masked so the image past len stays
// zero.
template <int LANES>
__device__ __forceinline__ void one_xor(uint4 *img_u4, uint32_t len, const uint32_t (&dek)[8],
                                        uint32_t kb0) {
  const uint32_t nks = (len + 63) >> 6;
  for (uint32_t kb = threadIdx.x; kb < nks; kb += LANES) {
    uint32_t x[16];
    chacha_block<0>(x, dek, kb0 + kb);
    const uint32_t avail = min(len - kb * 64u, 64u);
    if (avail < 64) mask_tail(x, avail);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = img_u4[img_g(kb * 4 + i)];
      v.x ^= x[4 * i];
      v.y ^= x[4 * i + 1];
      v.z ^= x[4 * i + 2];
      v.w ^= x[4 * i + 3];
      img_u4[img_g(kb * 4 + i)] = v;
    }
  }
}

// Store the image's first len bytes to dst (16-B aligned).
template <int LANES>
__device__ __forceinline__ void one_store(const uint4 *img_u4, uint8_t *dst, uint32_t len) {
  for (uint32_t p = threadIdx.x * 16u; p < len; p += LANES * 16u) {
    const uint4 v = img_u4[img_g(p >> 4)];
    if (p + 16u <= len) {
      *reinterpret_cast<uint4 *>(dst + p) = v;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      for (uint32_t i = 0; p + i < len; ++i) dst[p + i] = uint8_t(w[i >> 2] >> (8 * (i & 3)));
    }
  }
}

// The descriptor, staged into LDS by one load per word, all issued at once
// (round 6).  It lives in pinned host memory, and reading its fields where
// they are used made each group of them a PCIe round trip (~1.7 us) on the
// post's critical path: round 5's k_one waited for the salt words after the
// message, then for the CID key, the output pointers, the flag and the
// sequence number (s_load ... s_waitcnt pairs in the code object).
#ifndef GLFSX_DESC_LDS
#define GLFSX_DESC_LDS 1
#endif
__device__ __forceinline__ const OneDesc *one_desc(OneDesc *s, const OneDesc *g) {
  if (!GLFSX_DESC_LDS) return g;  // (A/B builds: fields read where used)
  constexpr uint32_t kW = sizeof(OneDesc) / 4;
  static_assert(sizeof(OneDesc) % 4 == 0 && kW <= 64, "wave 0 stages the descriptor");
  if (threadIdx.x < kW)
    reinterpret_cast<uint32_t *>(s)[threadIdx.x] =
        reinterpret_cast<const uint32_t *>(g)[threadIdx.x];
  __syncthreads();
  return s;
}

// The post's results (ctext, ref) are in the caller's staging: every lane's
// stores are done, then one release store of the descriptor's sequence
// number into its flag (pinned host memory) tells the waiting caller, with
// no stream query (OneDesc::flag; nullable).
__device__ __forceinline__ void one_signal(const OneDesc *dp) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && dp->flag)
    __hip_atomic_store(dp->flag, dp->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Phase timing of k_one (A/B variant builds only: GLFSX_ONE_TIMING=1,
// scripts/one_trace.py): workgroup 0 adds s_memrealtime ticks since its
// start at each phase boundary.
#if GLFSX_ONE_TIMING
__device__ unsigned long long g_one_t[16];
#define ONE_T(i)                                                                        \
  do {                                                                                  \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                            \
      __hip_atomic_fetch_add(&g_one_t[i],                                               \
                             (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0), \
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);               \
  } while (0)
#else
#define ONE_T(i) \
  do {           \
  } while (0)
#endif

// The body of a one-shot post (k_one, k_one_v).  V: dp is the descriptor
// itself (a kernel argument); otherwise the launch's array in pinned host
// memory, staged by one_desc.
template <int QUADS, bool V>
__device__ __forceinline__ void one_run(const OneDesc *g) {
#if GLFSX_ONE_TIMING
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
#endif
  __shared__ uint4 img_u4[QUADS * 64];       // the message, then its ctext
  __shared__ uint4 ts_u4[QUADS / 2 * 4];     // parent inputs of the merge
  __shared__ uint32_t passbuf[8];
  __shared__ uint32_t s_dek[8];
  constexpr int kLanes = QUADS * 4;
  const OneDesc *dp;
  if constexpr (V) {
    dp = g;
  } else {
    __shared__ OneDesc s_desc;
    dp = one_desc(&s_desc, g + blockIdx.x);
  }
  const uint32_t len = dp->len;
  const uint32_t tid = threadIdx.x, q = tid & 3u, quad = tid >> 2;
  const uint32_t img = lds_offset(img_u4), ts = lds_offset(ts_u4);
  ONE_T(0);
  one_stage<kLanes>(img_u4, dp->src, len, dp->present, nullptr);
  uint32_t rel[28];
  quad_addrs(rel, 0u, q);
  __syncthreads();
  ONE_T(1);
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = dp->salt[i];
  uint32_t cl, ch;
#if GLFSX_ONE_TIMING  // one_hash with a stamp between its chunks and its merges
  {
    const uint32_t kq_lo = qsel(q, key[0], key[1], key[2], key[3]);
    const uint32_t kq_hi = qsel(q, key[4], key[5], key[6], key[7]);
    const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
    one_chunks(cl, ch, img, len, 0u, true, kq_lo, kq_hi, ivq, kKeyed, q, quad, rel);
    ONE_T(6);
    one_tree(cl, ch, len ? (len + 1023) >> 10 : 1u, true, ts, passbuf, kq_lo, kq_hi, ivq,
             kKeyed, q, quad, rel);
  }
#else
  one_hash(cl, ch, img, ts, passbuf, len, key, kKeyed, q, quad, rel);
#endif
  if (quad == 0) {  // lanes 0-3: DEK words q and 4+q
    s_dek[q] = cl;
    s_dek[4 + q] = ch;
  }
  __syncthreads();
  ONE_T(2);
  uint32_t dek[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dek[i] = s_dek[i];
  one_xor<kLanes>(img_u4, len, dek, 0u);
  __syncthreads();
  ONE_T(3);
  if (dp->ctext) one_store<kLanes>(img_u4, dp->ctext, len);  // drains during the CID
  uint32_t ckey[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ckey[i] = dp->cid_key[i];
#if GLFSX_ONE_TIMING
  {
    const uint32_t cb = dp->cid_keyed ? kKeyed : 0u;
    const uint32_t kq_lo = qsel(q, ckey[0], ckey[1], ckey[2], ckey[3]);
    const uint32_t kq_hi = qsel(q, ckey[4], ckey[5], ckey[6], ckey[7]);
    const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
    one_chunks(cl, ch, img, len, 0u, true, kq_lo, kq_hi, ivq, cb, q, quad, rel);
    ONE_T(7);
    one_tree(cl, ch, len ? (len + 1023) >> 10 : 1u, true, ts, passbuf, kq_lo, kq_hi, ivq, cb,
             q, quad, rel);
  }
#else
  one_hash(cl, ch, img, ts, passbuf, len, ckey, dp->cid_keyed ? kKeyed : 0u, q, quad, rel);
#endif
  if (quad == 0) {
    uint32_t *r = reinterpret_cast<uint32_t *>(dp->ref);
    r[q] = cl;
    r[4 + q] = ch;
    r[8 + q] = dek[q];
    r[12 + q] = dek[4 + q];
  }
  ONE_T(4);
  one_signal(dp);
  ONE_T(5);
#if GLFSX_ONE_TIMING
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // shader clock over the kernel: [13] / [14]
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_add(&g_one_t[13], (unsigned long long)(c1 - c0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&g_one_t[14], (unsigned long long)(t1 - t0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&g_one_t[15], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
}

template <int QUADS>
__global__ __launch_bounds__(QUADS * 4) void k_one(const OneDesc *descs) {
  one_run<QUADS, false>(descs);
}

// A launch of one post (the common case of a caller posting alone): the
// descriptor travels as the kernel argument, so its fields are read from the
// kernarg segment instead of one PCIe round trip to pinned host memory ahead
// of everything else (round 6).
template <int QUADS>
__global__ __launch_bounds__(QUADS * 4) void k_one_v(const OneDesc d) {
  one_run<QUADS, true>(&d);
}

// ---- Medium one-shot posts (kMaxOneLen < len <= kMaxMedLen) ----
// Workgroup s of a message owns its 64 KiB span s (64 chunks, one per quad).
// k_med_dek stages the span from the caller's staging (pinned host memory)
// into LDS and into the descriptor's device copy, hashes its subtree and
// publishes the CV; the message's last-arriving workgroup merges the W CVs
// (ROOT on top) into the DEK.  k_med_cid reads the span back from the device
// copy, XORs the keystream in, stores the ctext to the caller's staging and
// hashes the CID the same way.  Same cross-XCD protocol as the split passes
// (publish_cv / arrive_last / load_cv_word); the counter is left at zero.
// Grid: n x wmax workgroups; workgroups past a message's span exit at once.
__device__ __forceinline__ void med_publish_merge(uint32_t &cl, uint32_t &ch, const OneDesc *dp,
                                                  uint32_t sidx, uint32_t W, uint32_t ts,
                                                  uint32_t *passbuf, uint32_t *flag,
                                                  const uint32_t (&key)[8], uint32_t base,
                                                  uint32_t q, uint32_t quad,
                                                  const uint32_t (&rel)[28], bool *last) {
  const uint32_t tid = threadIdx.x;
  if (quad == 0) {  // lanes 0-3 of wave 0: one store instruction per word pair
    __hip_atomic_store(dp->cvs + sidx * 8 + q, cl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dp->cvs + sidx * 8 + 4 + q, ch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  *last = arrive_last(dp->cnt, W, tid, flag);
  if (!*last) return;
  const uint32_t kq_lo = qsel(q, key[0], key[1], key[2], key[3]);
  const uint32_t kq_hi = qsel(q, key[4], key[5], key[6], key[7]);
  const uint32_t ivq = qsel(q, kIV[0], kIV[1], kIV[2], kIV[3]);
  if (quad < W) {
    cl = load_cv_word(dp->cvs + quad * 8 + q);
    ch = load_cv_word(dp->cvs + quad * 8 + 4 + q);
  }
  one_tree(cl, ch, W, true, ts, passbuf, kq_lo, kq_hi, ivq, base, q, quad, rel);
  if (tid == 0) *dp->cnt = 0;
}

// V: g is the descriptor itself (a kernel argument, one message); else the
// launch's array (as one_run)
template <bool V>
__device__ __forceinline__ void med_dek_run(const OneDesc *g, uint32_t wmax) {
  __shared__ uint4 img_u4[64 * 64];
  __shared__ uint4 ts_u4[32 * 4];
  __shared__ uint32_t passbuf[8];
  __shared__ uint32_t s_flag;
  const OneDesc *dp;
  if constexpr (V) {
    dp = g;
  } else {
    __shared__ OneDesc s_desc;
    dp = one_desc(&s_desc, g + blockIdx.x / wmax);
  }
  const uint32_t sidx = blockIdx.x % wmax;
  const uint32_t len = dp->len;
  const uint32_t W = (len + 65535u) >> 16;
  if (sidx >= W) return;  // uniform: past this message's spans
  const uint32_t off = sidx << 16, slen = min(len - off, 65536u);
  const uint32_t present = dp->present > off ? dp->present - off : 0u;
  const uint32_t tid = threadIdx.x, q = tid & 3u, quad = tid >> 2;
  const uint32_t img = lds_offset(img_u4), ts = lds_offset(ts_u4);
  one_stage<256>(img_u4, dp->src + off, slen, present, dp->dmsg + off);
  uint32_t rel[28];
  quad_addrs(rel, 0u, q);
  __syncthreads();
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = dp->salt[i];
  uint32_t cl, ch;
  one_hash(cl, ch, img, ts, passbuf, slen, key, kKeyed, q, quad, rel, sidx << 6, false);
  bool last;
  med_publish_merge(cl, ch, dp, sidx, W, ts, passbuf, &s_flag, key, kKeyed, q, quad, rel,
                    &last);
  if (last && quad == 0) {
    dp->dek[q] = cl;
    dp->dek[4 + q] = ch;
    uint32_t *r = reinterpret_cast<uint32_t *>(dp->ref);
    r[8 + q] = cl;
    r[12 + q] = ch;
  }
}

template <bool V>
__device__ __forceinline__ void med_cid_run(const OneDesc *g, uint32_t wmax) {
  __shared__ uint4 img_u4[64 * 64];
  __shared__ uint4 ts_u4[32 * 4];
  __shared__ uint32_t passbuf[8];
  __shared__ uint32_t s_flag;
  const OneDesc *dp;
  if constexpr (V) {
    dp = g;
  } else {
    __shared__ OneDesc s_desc;
    dp = one_desc(&s_desc, g + blockIdx.x / wmax);
  }
  const uint32_t sidx = blockIdx.x % wmax;
  const uint32_t len = dp->len;
  const uint32_t W = (len + 65535u) >> 16;
  if (sidx >= W) return;
  const uint32_t off = sidx << 16, slen = min(len - off, 65536u);
  const uint32_t tid = threadIdx.x, q = tid & 3u, quad = tid >> 2;
  const uint32_t img = lds_offset(img_u4), ts = lds_offset(ts_u4);
  // the device copy holds the span zero padded to 64 B (k_med_dek)
  const uint32_t padded = (slen + 63) & ~63u;
  {
    // all loads in flight at once (see one_stage).  Zero-initialised: left
    // partly unassigned, the array stayed in scratch -- each load waited for
    // and spilled before the next was issued (the code object of rounds 5-6)
    uint4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t p = (tid + uint32_t(i) * 256u) * 16u;
      v[i] = make_uint4(0, 0, 0, 0);
      if (p < padded) v[i] = *reinterpret_cast<const uint4 *>(dp->dmsg + off + p);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t p = (tid + uint32_t(i) * 256u) * 16u;
      if (p < padded) img_u4[img_g(p >> 4)] = v[i];
    }
  }
  uint32_t dek[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dek[i] = dp->dek[i];
  uint32_t rel[28];
  quad_addrs(rel, 0u, q);
  __syncthreads();
  one_xor<256>(img_u4, slen, dek, sidx << 10);
  __syncthreads();
  if (dp->ctext) one_store<256>(img_u4, dp->ctext + off, slen);
  uint32_t ckey[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ckey[i] = dp->cid_key[i];
  const uint32_t base = dp->cid_keyed ? kKeyed : 0u;
  uint32_t cl, ch;
  one_hash(cl, ch, img, ts, passbuf, slen, ckey, base, q, quad, rel, sidx << 6, false);
  // this span's ctext is in the caller's staging before the span counts in
  // (the last workgroup signals the caller): the stores are done, and a
  // system-scope release writes back what this XCD's L2 holds of them --
  // the staging may be non-coherent host memory, and the last workgroup's
  // own release covers only its XCD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && dp->flag) __threadfence_system();
  bool last;
  med_publish_merge(cl, ch, dp, sidx, W, ts, passbuf, &s_flag, ckey, base, q, quad, rel,
                    &last);
  if (last && quad == 0) {
    uint32_t *r = reinterpret_cast<uint32_t *>(dp->ref);
    r[q] = cl;
    r[4 + q] = ch;
  }
  if (last) one_signal(dp);
}

__global__ __launch_bounds__(256) void k_med_dek(const OneDesc *descs, uint32_t wmax) {
  med_dek_run<false>(descs, wmax);
}
__global__ __launch_bounds__(256) void k_med_cid(const OneDesc *descs, uint32_t wmax) {
  med_cid_run<false>(descs, wmax);
}
// One medium post, its descriptor as the kernel argument (k_one_v)
__global__ __launch_bounds__(256) void k_med_dek_v(const OneDesc d, uint32_t wmax) {
  med_dek_run<true>(&d, wmax);
}
__global__ __launch_bounds__(256) void k_med_cid_v(const OneDesc d, uint32_t wmax) {
  med_cid_run<true>(&d, wmax);
}

// Small blobs (glfs.PostBlob of many blobs that each fit one bigblob block,
// e.g. BASELINE config 4's 1M x 4 KiB): one lane per blob.  A blob of
// 0 < len <= block_size has root = post(rawSalt, blob) (blob.go:190-193); the
// empty blob has root = post(indexSalt, "") (blob.go:187-189), so the key is
// selected per lane.  Every lane finishes its own BLAKE3 tree (G >= chunks).
struct SArgs {
  const uint8_t *src;
  uint8_t *ctext;
  const uint64_t *offs;
  const uint64_t *lens;
  uint64_t n;
  uint8_t *refs;      // 64 B per blob, dense
  uint32_t key[8];    // DEK pass: rawSalt words; CID pass: CID key words
  uint32_t key0[8];   // DEK pass: indexSalt words (empty blobs); CID pass: = key
  uint32_t base;
  uint32_t out_off;
  uint64_t n_coarse;  // k_small_q: items [0, n_coarse) are 64 blobs (one per
                      // lane); the blobs after them go as fine items
  uint64_t small_max;  // longer blobs are skipped (SmallJob::small_max)
  uint8_t *hex_out;    // CID pass, nullable: the root as tree-line hex digits
  const uint64_t *hex_pos;
};

// Lower-case hex digits of bytes 0 and 1 of x, in output order (hi(b0)
// lo(b0) hi(b1) lo(b1)) as one little-endian word (tree_kernels.hip hex4).
__device__ __forceinline__ uint32_t hex4(uint32_t x) {
  const uint32_t n = ((x >> 4) & 0xFu) | ((x & 0xFu) << 8) |
                     ((x >> 12) & 0xFu) << 16 | ((x >> 8) & 0xFu) << 24;
  const uint32_t ge10 = ((n + 0x06060606u) >> 4) & 0x01010101u;  // nibble >= 10
  return n + 0x30303030u + ge10 * 39u;
}

// The 64 hex digits of the 32 bytes in w (tree.go:309's "cid"/"dek" field
// of a TreeEntry line, encoding as tree_kernels.hip's hex32) at dst, any
// alignment: aligned 4-byte stores of the digits shifted into place
// (alignbyte), the two partial words at the ends byte by byte -- no byte
// outside [dst, dst + 64) is written.
__device__ __forceinline__ void put_hex32(uint8_t *dst, const uint32_t w[8]) {
  const uint32_t s = uint32_t(reinterpret_cast<uintptr_t>(dst) & 3u);
  const uint32_t sh = 8u * (4u - s);  // s = 0: the whole next word
  uint32_t *base = reinterpret_cast<uint32_t *>(dst - s);
  uint32_t prev = 0;  // streamed one digit word at a time: few live values
#pragma unroll
  for (int k = 0; k <= 16; ++k) {
    const uint32_t cur = k < 16 ? hex4(w[k >> 1] >> (16 * (k & 1))) : 0u;
    const uint32_t v = uint32_t(((uint64_t(cur) << 32) | prev) >> sh);
    if ((k >= 1 && k <= 15) || (k == 0 && s == 0)) {
      base[k] = v;
    } else {
      const uint32_t lo = k == 0 ? s : 0u, hi = k == 0 ? 4u : s;
      uint8_t *b = reinterpret_cast<uint8_t *>(base + k);
      for (uint32_t x = lo; x < hi; ++x) b[x] = uint8_t(v >> (8u * x));
    }
    prev = cur;
  }
}

// Blob i for the calling lane (nothing when i >= n); lds_u4: the
// workgroup's 4 x 8 KiB staging images.  No barriers.
template <int G, bool CHACHA, int A>
__device__ __forceinline__ void small_blob(const SArgs &a, uint64_t i, uint4 *lds_u4) {
  if (i >= a.n) return;
  const uint64_t off = a.offs[i], len = a.lens[i];
  if (len > a.small_max) return;  // posted by the host's large-blob route
  const uint8_t *msg = a.src + off;
  uint8_t *cmsg = (CHACHA && a.ctext) ? a.ctext + off : nullptr;
  uint8_t *ref = a.refs + i * 64;
  uint32_t key[8], dek[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) key[w] = len ? a.key[w] : a.key0[w];
  if constexpr (CHACHA) {
    const uint32_t *dp = reinterpret_cast<const uint32_t *>(ref + 32);
#pragma unroll
    for (int w = 0; w < 8; ++w) dek[w] = dp[w];
  } else {
#pragma unroll
    for (int w = 0; w < 8; ++w) dek[w] = 0;
  }
  const uint32_t C = len ? uint32_t((len + 1023) >> 10) : 1u;
  const bool aligned = ((reinterpret_cast<uintptr_t>(msg) |
                         reinterpret_cast<uintptr_t>(cmsg)) & 15) == 0;
  uint32_t cv[8];
  // a full wave of back-to-back blobs of exactly G KiB (config 4: 4 KiB
  // blobs packed densely) has k_pass's lane layout: stage through LDS for
  // full-line loads (and ctext stores)
  const uint32_t l = threadIdx.x & 63u;
  // (readfirstlane returns int: widen through uint32_t, or a low word of
  // 2^31 or more sign-extends into the high word -- every wave of blobs in
  // the upper 2 GiB of each 4 GiB then failed the density test below and
  // took the per-lane path)
  const uint64_t o0 =
      (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(off >> 32)))) << 32) |
      uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(off)));
  const bool dense = aligned && len == uint64_t(G) << 10 &&
                     off == o0 + (uint64_t(l) * G << 10) && (!CHACHA || cmsg);
  if (__ballot(dense) == ~0ull) {  // wave-uniform
    lane_subtree_full<G, CHACHA, true, A>(
        cv, a.src + o0, cmsg ? a.ctext + o0 : nullptr, l * G, true, key, a.base,
        dek, lds_offset(lds_u4 + (threadIdx.x >> 6) * 512), 64u * G << 10,
        0u - l * G);
  } else if (aligned && len == uint64_t(G) << 10) {
    lane_subtree_full<G, CHACHA, false, A>(cv, msg, cmsg, 0u, true, key, a.base, dek);
  } else if (aligned) {
    lane_subtree<G, CHACHA, true, A>(cv, msg, cmsg, len, 0u, C, true, key, a.base, dek);
  } else {
    lane_subtree<G, CHACHA, false, A>(cv, msg, cmsg, len, 0u, C, true, key, a.base, dek);
  }
  store_digest(ref + a.out_off, cv);
  if (CHACHA && a.hex_out) {  // the tree line's cid and dek digits
    const uint64_t pos = a.hex_pos[i];
    if (pos != ~0ull) {  // ~0: the lines did not fit their buffer
      put_hex32(a.hex_out + pos, cv);
      put_hex32(a.hex_out + pos + kDekAfterCid, dek);
    }
  }
}

// A fine item of k_small_q: 64/G blobs, G lanes per blob (lane l hashes
// chunk l % G of blob b0 + l / G), so the item takes about 1/G of a
// one-lane-per-blob item's time.  Handed out last, they shorten the run-down
// at the end of the launch.  Dense blobs of exactly G KiB take k_pass's
// staged G = 1 lane layout over the wave's contiguous 64 KiB; the G chunk
// CVs of a blob then merge through lane shuffles (log2 G parent levels, ROOT
// on the last: the same tree as a lane's own stack).  Anything else: one
// lane per blob on the first 64/G lanes.
template <int G, bool CHACHA, int A>
__device__ __forceinline__ void small_fine(const SArgs &a, uint64_t b0, uint4 *lds_u4) {
  constexpr uint32_t BPI = 64u / G;
  const uint32_t l = threadIdx.x & 63u, c = l % G;
  const uint64_t i = b0 + l / G;
  const bool valid = i < a.n;
  const uint64_t off = valid ? a.offs[i] : 0, len = valid ? a.lens[i] : 0;
  const uint8_t *msg = a.src + off;
  uint8_t *cmsg = (CHACHA && a.ctext) ? a.ctext + off : nullptr;
  const uint64_t o0 =
      (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(off >> 32)))) << 32) |
      uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(off)));
  const bool aligned = ((reinterpret_cast<uintptr_t>(msg) |
                         reinterpret_cast<uintptr_t>(cmsg)) & 15) == 0;
  const bool dense = valid && aligned && len == uint64_t(G) << 10 && len <= a.small_max &&
                     off == o0 + (uint64_t(l) << 10) - (uint64_t(c) << 10) &&
                     (!CHACHA || cmsg);
  if (__ballot(dense) != ~0ull) {
    small_blob<G, CHACHA, A>(a, l < BPI ? b0 + l : ~0ull, lds_u4);
    return;
  }
  uint8_t *ref = a.refs + i * 64;
  uint32_t key[8], dek[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) key[w] = a.key[w];
  if constexpr (CHACHA) {
    const uint32_t *dp = reinterpret_cast<const uint32_t *>(ref + 32);
#pragma unroll
    for (int w = 0; w < 8; ++w) dek[w] = dp[w];
  } else {
#pragma unroll
    for (int w = 0; w < 8; ++w) dek[w] = 0;
  }
  uint32_t cv[8];
  lane_subtree_full<1, CHACHA, true, A>(
      cv, a.src + o0, CHACHA ? a.ctext + o0 : nullptr, l, false, key, a.base, dek,
      lds_offset(lds_u4 + (threadIdx.x >> 6) * 512), 64u << 10, c - l);
#pragma unroll
  for (uint32_t st = 1; st < uint32_t(G); st <<= 1) {
    uint32_t m[16];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      m[w] = cv[w];
      m[8 + w] = uint32_t(__shfl_down(int(cv[w]), st, 64));
      cv[w] = key[w];
    }
    b3_compress<A>(cv, m, 0u, 0u, 64u, a.base | kParent | (2 * st == G ? kRoot : 0u));
  }
  if (c == 0) {
    store_digest(ref + a.out_off, cv);
    if (CHACHA && a.hex_out) {
      const uint64_t pos = a.hex_pos[i];
      if (pos != ~0ull) {
        put_hex32(a.hex_out + pos, cv);
        put_hex32(a.hex_out + pos + kDekAfterCid, dek);
      }
    }
  }
}

template <int G, bool CHACHA, int A = 2>
__global__ __launch_bounds__(256) void k_small(SArgs a) {
  // 4 waves x 8 KiB staging image (same layout as k_pass's)
  __shared__ uint4 lds_u4[4 * 512];
  small_blob<G, CHACHA, A>(a, blockIdx.x * uint64_t(blockDim.x) + threadIdx.x, lds_u4);
}

// The same with as many workgroups as the chip holds at once, each WAVE
// taking items of 64 consecutive blobs: its first by its number, the next
// ones from a device-wide counter (bank epoch & 1 of two, the other zeroed
// by workgroup 0 for the next launch on the stream).  A wave that finishes
// early takes more, so the launch ends within about one item of its last
// wave instead of with whole workgroups' worth of CUs idle (config 4's
// 4096-workgroup launches lost ~12 % to that tail: scripts/sb_sizes.py).
// GLFSX_SMALLQ_WPE waves per SIMD at least (4: at most 128 VGPRs, like
// k_small; the loop let the CID form grow to 133 VGPRs, i.e. three waves,
// and capping it spills 5 VGPRs: both measured)
#ifndef GLFSX_SMALLQ_WPE
#define GLFSX_SMALLQ_WPE 4
#endif
template <int G, bool CHACHA, int A = 2>
__global__ __launch_bounds__(256, GLFSX_SMALLQ_WPE) void k_small_q(SArgs a, uint32_t *ctr,
                                                                   uint32_t epoch) {
  __shared__ uint4 lds_u4[4 * 512];
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(ctr + ((epoch + 1u) & 1u) * 32u, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  uint32_t *mine = ctr + (epoch & 1u) * 32u;
  constexpr uint32_t BPI = G > 1 ? 64u / G : 64u;
  const uint64_t fine0 = a.n_coarse << 6;
  const uint64_t items = a.n_coarse + (a.n > fine0 ? (a.n - fine0 + BPI - 1) / BPI : 0);
  const uint32_t waves = gridDim.x * 4u;
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t item = blockIdx.x * 4u + (threadIdx.x >> 6);
  while (item < items) {  // wave-uniform
    if (G == 1 || item < a.n_coarse)
      small_blob<G, CHACHA, A>(a, (item << 6) | lane, lds_u4);
    else if constexpr (G > 1)
      small_fine<G, CHACHA, A>(a, fine0 + (item - a.n_coarse) * BPI, lds_u4);
    uint32_t t = 0;
    if (lane == 0)
      t = __hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    item = waves + uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(t)));
  }
}

// Read side (bigblob/ref.go:113-126 getF -> cryptoXOR, blob.go:31-69): decrypt
// n blocks of bs bytes (bs % 64 == 0) laid out contiguously, block j with
// the DEK in bytes [32,64) of refs[j].  One thread per 64-B keystream block.
__global__ __launch_bounds__(256) void k_decrypt(KArgs a) {
  const uint64_t per = a.msg_len >> 6;  // keystream blocks per bigblob block
  const uint64_t total_kb = (a.n - 1) * per + ((a.last_len + 63) >> 6);
  // a.stride: first keystream block (the part before it went through
  // k_decrypt_lines)
  for (uint64_t kb = a.stride + blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; kb < total_kb;
       kb += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t j = kb / per;
    const uint32_t ctr = uint32_t(kb - j * per);
    const uint64_t off = kb << 6;
    const uint64_t end = j * a.msg_len + ((j + 1 == a.n) ? a.last_len : a.msg_len);
    const uint32_t avail = uint32_t(min<uint64_t>(64, end - off));
    const uint32_t *dp = reinterpret_cast<const uint32_t *>(a.refs + j * 64 + 32);
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = dp[i];
    uint32_t m[16], x[16];
    const bool al = ((reinterpret_cast<uintptr_t>(a.src) |
                      reinterpret_cast<uintptr_t>(a.ctext)) & 15) == 0;
    if (al) load_block<true>(m, a.src + off, avail);
    else load_block<false>(m, a.src + off, avail);
    chacha_block(x, k, ctr);
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] ^= x[i];
    if (al) store_block<true>(a.ctext + off, m, avail);
    else store_block<false>(a.ctext + off, m, avail);
  }
}

// Read side, bulk: one wave per 4 KiB unit of ctext (lane l = keystream
// block l of the unit), bs % 4096 == 0 so the unit's DEK is uniform (scalar
// loads into SGPRs; the key-only quarter-rounds of round 1 are hoisted by the
// compiler).  Each wave has two 4 KiB images: unit u+stride arrives by
// buffer_load ... lds (4 instructions x 8 full 128-B lines) while unit u is
// decrypted.  Image layout: piece p (16 B) of lane L's block sits at
// 64L + 16 (p ^ ((L >> 2) & 3)), so the lane's ds_read_b128s are conflict-free
// and the loader / storer lane l of instruction k touches image byte
// 1024k + 16l <-> unit byte 1024k + vo(l).  Covers units [0, n_units);
// k_decrypt does the rest.
template <int A>
__global__ __launch_bounds__(256) void k_decrypt_lines(KArgs a, uint64_t n_units,
                                                       uint32_t upb_shift,
                                                       uint32_t run_shift) {
  __shared__ uint4 img[4 * 512];
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wbase = lds_offset(img + wv * 512);
  const uint32_t sb = __builtin_amdgcn_readfirstlane(wbase);
  const uint32_t vo = ((l >> 2) << 6) + (((l & 3u) ^ ((l >> 4) & 3u)) << 4);
  const uint32_t wa = wbase + (l << 6) + (((l >> 2) & 3u) << 4);
  const uint32_t rl = wbase + (l << 4);  // linear slot for the stores
  const uint64_t upb = a.msg_len >> 12;  // units per bigblob block
  // the wave walks runs of R = 2^run_shift consecutive units inside one
  // bigblob block (R divides the units per block): the DEK and its key-only
  // quarter-rounds are loop-invariant over a run
  const uint64_t n_runs = (n_units + (1ull << run_shift) - 1) >> run_shift;
  const uint64_t wstride = uint64_t(gridDim.x) * 4;
  auto issue = [&](uint64_t uu, uint32_t buf) {
    const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.src) + (uu << 12), 0, 4096u, 0x00020000);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          src, (__attribute__((address_space(3))) void *)(uintptr_t)(sb + 4096u * buf + 1024u * k),
          16, vo, 1024u * k, 0, 0);
  };
  uint64_t run = uint64_t(blockIdx.x) * 4 + wv;
  if (run < n_runs) issue(run << run_shift, 0);
  uint32_t buf = 0;
  for (; run < n_runs; run += wstride) {
    const uint64_t u0 = run << run_shift;
    const uint64_t u1 = min(u0 + (1ull << run_shift), n_units);
    // bigblob block (uniform): its DEK.  upb_shift = log2(units per block)
    // when that is a power of two (no 64-bit scalar division per run)
    const uint64_t j = upb_shift < 64 ? u0 >> upb_shift : u0 / upb;
    const __attribute__((address_space(4))) uint32_t *kp =
        (const __attribute__((address_space(4))) uint32_t *)(uintptr_t)(
            a.refs + j * 64 + 32);
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = kp[i];
    const uint64_t nrun = run + wstride;
   for (uint64_t u = u0; u < u1; ++u, buf ^= 1u) {
    const uint64_t un = u + 1 < u1 ? u + 1 : (nrun << run_shift);
    // the other image was last read by the previous unit's store ds_reads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool more = u + 1 < u1 || nrun < n_runs;
    if (more) issue(un, buf ^ 1u);
    // this unit's lines: all but the 4 youngest vector-memory ops (the next
    // unit's loads) are done -- the previous unit's stores included
    if (more)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t w = opaque(wa) + 4096u * buf;
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = *reinterpret_cast<const lds_u32x4 *>(w ^ (uint32_t(q) << 4));
    uint32_t x[16];
    chacha_block<A>(x, key, uint32_t((u - j * upb) << 6) + l);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 c = v[q];
      c.x ^= x[4 * q];
      c.y ^= x[4 * q + 1];
      c.z ^= x[4 * q + 2];
      c.w ^= x[4 * q + 3];
      *reinterpret_cast<lds_u32x4 *>(w ^ (uint32_t(q) << 4)) = c;
    }
    const __amdgpu_buffer_rsrc_t dst =
        __builtin_amdgcn_make_buffer_rsrc(a.ctext + (u << 12), 0, 4096u, 0x00020000);
    const uint32_t r0 = opaque(rl) + 4096u * buf;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 c = *reinterpret_cast<const lds_u32x4 *>(r0 + 1024u * k);
      __builtin_amdgcn_raw_buffer_store_b128(c, dst, vo, 1024u * k, 0);
    }
   }
  }
}

__global__ __launch_bounds__(256) void k_chacha_xor(KArgs a) {
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = a.key[i];
  const uint64_t nblk = (a.msg_len + 63) >> 6;
  for (uint64_t b = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; b < nblk;
       b += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t off = b << 6;
    const uint64_t rem = a.msg_len - off;
    const uint32_t avail = rem < 64 ? uint32_t(rem) : 64u;
    uint32_t m[16], x[16];
    const bool al = ((reinterpret_cast<uintptr_t>(a.src + off) |
                      reinterpret_cast<uintptr_t>(a.ctext + off)) & 15) == 0;
    if (al) load_block<true>(m, a.src + off, avail);
    else load_block<false>(m, a.src + off, avail);
    chacha_block(x, k, uint32_t(b));
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] ^= x[i];
    if (al) store_block<true>(a.ctext + off, m, avail);
    else store_block<false>(a.ctext + off, m, avail);
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Synthetic data (bench/test inputs): byte o = byte (o & 7) of
// splitmix64(seed ^ (o >> 3)); same generator as oracle_fill_splitmix.
__global__ __launch_bounds__(256) void k_fill(uint8_t *dst, uint64_t offset,
                                              uint64_t n, uint64_t seed) {
  const uint64_t words = (n + 7) >> 3;
  for (uint64_t w = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; w < words;
       w += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t v = splitmix64(seed ^ ((offset >> 3) + w));
    if ((w + 1) * 8 <= n && ((reinterpret_cast<uintptr_t>(dst) & 7) == 0)) {
      reinterpret_cast<uint64_t *>(dst)[w] = v;
    } else {
      for (uint64_t i = w * 8; i < n && i < w * 8 + 8; ++i)
        dst[i] = uint8_t(v >> (8 * (i & 7)));
    }
  }
}

// Latency mode: launches of at most this many 256-lane workgroups (default
// 512 = 2 waves per SIMD) run the compiler-scheduled ARX form, and the CID
// pass splits into a per-block keystream launch + a BLAKE3 pass.
// glfsx_set_latency_wgs overrides it (tuning, tests of both forms).
std::atomic<uint32_t> g_latency_wgs{512};
uint32_t latency_wgs() { return g_latency_wgs.load(std::memory_order_relaxed); }

// ARX form of the many-round launches (no split, G >= 4: the headline's
// passes): 2 = step-interleaved, 1 = quarter-round order (both one asm
// statement per instruction).  Split / small-G launches always use 2.
// Measured (scripts/ab_head.sh, one box, 2 interleaved reps): CID form 1
// headline 992-995 vs 979-983 GiB/s with form 2, config 2 unchanged
// (855-860); the DEK pass is indifferent.
#ifndef GLFSX_HEAD_DEK
#define GLFSX_HEAD_DEK 2
#endif
#ifndef GLFSX_HEAD_CID
#define GLFSX_HEAD_CID 1
#endif

template <int G, bool CHACHA>
hipError_t launch_g(const KArgs &a, bool aligned, hipStream_t s) {
  const dim3 grid(uint32_t(a.n << a.split_log2)), block(256);
  // <= 2 waves per SIMD (512 workgroups of 4 waves on 1024 SIMDs): the
  // compiler-scheduled ARX issues faster than the asm form (tools/arx.hip)
  const bool lat = grid.x <= latency_wgs();
  constexpr int kHead = CHACHA ? GLFSX_HEAD_CID : GLFSX_HEAD_DEK;
  if (aligned && lat)
    hipLaunchKernelGGL((k_pass<G, CHACHA, true, 0>), grid, block, 0, s, a);
  else if (kHead != 2 && G >= 4 && aligned && a.split_log2 == 0)
    hipLaunchKernelGGL((k_pass<G, CHACHA, true, (kHead != 2 ? kHead : 2)>), grid, block, 0,
                       s, a);
  else if (aligned)
    hipLaunchKernelGGL((k_pass<G, CHACHA, true>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_pass<G, CHACHA, false>), grid, block, 0, s, a);
  return hipGetLastError();
}

// Split-mode target: workgroups per launch below which a message is spread
// over more workgroups (fewer chunks per lane).  0 disables split mode
// (glfsx_set_split_target: tests of both forms).
std::atomic<uint32_t> g_split_target{2048u};
constexpr uint32_t kMaxSplitLog2 = 8;  // the last workgroup merges <= 256 CVs
constexpr uint64_t kDcMinWgs = 1024;   // see pass_plan
// A/B switches (tools/build_variant.sh): GLFSX_LAT_ADJ=0 keeps pass_plan's
// plan for 320-1023 workgroups instead of moving it to the latency form;
// GLFSX_DC=0 never runs the one-launch split post (k_pass_dc)
#ifndef GLFSX_LAT_ADJ
#define GLFSX_LAT_ADJ 1
#endif
#ifndef GLFSX_DC
#define GLFSX_DC 1
#endif

// Split-mode scratch (32 B per workgroup) and arrival counters (4 B per
// message, zero between launches: each message's last workgroup resets its
// own): one persistent pair of buffers per (device, stream), reused by every
// launch on that stream -- launches on one stream are ordered, so they are
// never shared by two in flight.  The stream-ordered pool (hipMallocAsync /
// hipFreeAsync per launch) serialised the Writer's three-stream pipeline
// (host round trip 43.5 -> 24 GiB/s).  A buffer only grows when a launch
// needs more; the old one is released after its stream drains.
struct ScratchSlot {
  int dev;
  hipStream_t stream;
  uint32_t *p;
  size_t bytes;
  uint32_t *cnt;
  size_t cnt_words;
  uint32_t *ready;     // k_pass_dc: per-message DEK ready flags (= epoch)
  size_t ready_words;
  uint32_t epoch;
  uint32_t *lists;     // k_pass_dc: 2 banks of work-list counters (device)
  uint32_t *err;       // k_pass_dc: DEK-wait timeouts (pinned host word)
  uint32_t *d_err;     // the same word as the kernels address it
  DcConst *dcc;        // k_pass_dc's DcConst (device memory)
  DcConst dcc_host;    // what was last copied there
  uint32_t *qctr;      // k_small_q: two banks of its item counter
  uint32_t qepoch;
};
std::mutex g_scratch_mu;
std::vector<ScratchSlot> g_scratch;

// The device stream s belongs to (the current device for the null stream),
// current for the scope.  The scratch slots are keyed by (device, stream)
// and allocated on the current device; a caller driving several GPUs may
// reach here with another device current than its stream's (a
// multi-device Writer checked a lane's error word under the wrong device
// and missed it), so the stream, not the thread, names the device.
struct StreamDevice {
  int dev = 0, prev = 0;
  hipError_t e = hipSuccess;
  explicit StreamDevice(hipStream_t s) {
    e = hipGetDevice(&prev);
    if (e != hipSuccess) return;
    dev = prev;
    hipDevice_t d = 0;
    if (s && hipStreamGetDevice(s, &d) == hipSuccess) dev = d;
    if (dev != prev) e = hipSetDevice(dev);
  }
  ~StreamDevice() {
    if (dev != prev) (void)hipSetDevice(prev);
  }
};

hipError_t scratch_get(KArgs *a, uint64_t wgs, uint64_t msgs, hipStream_t s) {
  const size_t bytes = size_t(wgs) * 32, words = size_t(msgs);
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return sd.e;
  const int dev = sd.dev;
  hipError_t e = hipSuccess;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  ScratchSlot *sl = nullptr;
  for (ScratchSlot &x : g_scratch)
    if (x.dev == dev && x.stream == s) sl = &x;
  if (!sl) {
    g_scratch.push_back({dev, s, nullptr, 0, nullptr, 0, nullptr, 0, 0, nullptr,
                         nullptr, nullptr, nullptr, DcConst{}, nullptr, 0});
    sl = &g_scratch.back();
  }
  if (sl->bytes < bytes || sl->cnt_words < words) {
    if (sl->p || sl->cnt) {
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return e;
    }
    if (sl->bytes < bytes) {
      if (sl->p) (void)hipFree(sl->p);
      sl->p = nullptr;
      sl->bytes = 0;
      // at least the default target's worst case, so it rarely grows
      const size_t want = std::max(bytes, size_t(2) << 16);
      e = hipMalloc(reinterpret_cast<void **>(&sl->p), want);
      if (e != hipSuccess) return e;
      sl->bytes = want;
    }
    if (sl->cnt_words < words) {
      if (sl->cnt) (void)hipFree(sl->cnt);
      sl->cnt = nullptr;
      sl->cnt_words = 0;
      const size_t want = std::max(words, size_t(4096));
      e = hipMalloc(reinterpret_cast<void **>(&sl->cnt), want * 4);
      if (e != hipSuccess) return e;
      e = hipMemsetAsync(sl->cnt, 0, want * 4, s);
      if (e != hipSuccess) return e;
      sl->cnt_words = want;
    }
  }
  a->scratch = sl->p;
  a->cnt = sl->cnt;
  return hipSuccess;
}

// k_pass_dc's state for a launch over msgs messages on stream s: the ready
// flags and this launch's epoch (flags hold the epoch of the launch that set
// them, so they are never reset; zero is never an epoch), the work-list
// counters (bank epoch & 1, at zero), the error word.
std::atomic<uint64_t> g_dc_wait_ticks{100000000ull};  // 1 s of s_memrealtime
std::atomic<uint32_t> g_dc_skip_msg{~0u};
std::atomic<uint64_t> g_dc_timeouts{0};

constexpr size_t kListWords = 2 * kLists * kListStride;

hipError_t dc_get(uint64_t msgs, hipStream_t s, DcState *d) {
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return sd.e;
  const int dev = sd.dev;
  hipError_t e = hipSuccess;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  ScratchSlot *sl = nullptr;
  for (ScratchSlot &x : g_scratch)
    if (x.dev == dev && x.stream == s) sl = &x;
  if (!sl) return hipErrorInvalidValue;  // scratch_get first
  if (!sl->lists) {
    e = hipMalloc(reinterpret_cast<void **>(&sl->lists), kListWords * 4);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(sl->lists, 0, kListWords * 4, s);
    if (e != hipSuccess) return e;
    void *h = nullptr, *dp = nullptr;
    e = hipHostMalloc(&h, 64, hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    e = hipHostGetDevicePointer(&dp, h, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(h);
      return e;
    }
    sl->err = static_cast<uint32_t *>(h);
    sl->d_err = static_cast<uint32_t *>(dp);
    __atomic_store_n(sl->err, 0u, __ATOMIC_RELAXED);
  }
  if (sl->ready_words < msgs) {
    if (sl->ready) {
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return e;
      (void)hipFree(sl->ready);
    }
    sl->ready = nullptr;
    sl->ready_words = 0;
    const size_t want = std::max<size_t>(msgs, 4096);
    e = hipMalloc(reinterpret_cast<void **>(&sl->ready), want * 4);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(sl->ready, 0, want * 4, s);
    if (e != hipSuccess) return e;
    sl->ready_words = want;  // the epoch goes on: the new flags are zero
  }
  DcConst want{sl->ready, sl->lists, sl->d_err,
               g_dc_wait_ticks.load(std::memory_order_relaxed),
               g_dc_skip_msg.exchange(~0u, std::memory_order_relaxed)};
  if (!sl->dcc) {
    e = hipMalloc(reinterpret_cast<void **>(&sl->dcc), sizeof(DcConst));
    if (e != hipSuccess) return e;
    sl->dcc_host = DcConst{};
  }
  const DcConst &h = sl->dcc_host;
  if (want.ready != h.ready || want.lists != h.lists || want.err != h.err ||
      want.wait_ticks != h.wait_ticks || want.skip_msg != h.skip_msg) {
    // rare (new buffers, a test hook): ordered on s before the launch; the
    // copy is staged from pageable memory, so `want` may go out of scope
    e = hipMemcpyAsync(sl->dcc, &want, sizeof want, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    sl->dcc_host = want;
  }
  // The epoch advances only here, once nothing before the launch can fail
  // (ADVICE r3): a launch with epoch e clears the counter bank of epoch e+1,
  // so an epoch used up without a launch would leave the bank of e+2 stale.
  // Zero is never an epoch; the bank parity must alternate across the wrap.
  if (++sl->epoch == 0) sl->epoch = 2;
  d->epoch = sl->epoch;
  d->c = sl->dcc;
  return hipSuccess;
}

// A k_pass_dc launch failed after dc_get: its epoch was used without the
// launch that clears the next bank, so both banks start over at zero.
void dc_launch_failed(hipStream_t s) {
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (ScratchSlot &x : g_scratch)
    if (x.dev == sd.dev && x.stream == s && x.lists)
      (void)hipMemsetAsync(x.lists, 0, kListWords * 4, s);
}

// Chunks per lane (g) and log2 workgroups per message (sl) of a launch over
// n messages of at most maxlen bytes.
void pass_plan(uint64_t n, uint64_t maxlen, int *g_out, uint32_t *sl_out) {
  const uint64_t C = maxlen ? (maxlen + 1023) >> 10 : 1;
  int g = 1;
  while (256ull * g < C && g < 64) g *= 2;
  // messages above 256 lanes x 64 chunks (16 MiB) always span several
  // workgroups
  uint32_t sl = 0;
  while ((256ull * g << sl) < C) ++sl;
  // few messages: halve the chunks per lane and double the workgroups per
  // message until the launch fills the chip (256 CUs x 8 workgroups)
  const uint64_t target = g_split_target.load(std::memory_order_relaxed);
  const int g0 = g;
  const uint32_t sl0 = sl;
  while (g > 1 && sl < kMaxSplitLog2 && (n << sl) < target) {
    g /= 2;
    ++sl;
  }
  // ... but a one-launch split post (k_pass_dc: more than latency_wgs * 5/8
  // workgroups, G <= 4) of fewer than ~1024 workgroups runs its DEK and CID
  // items in about one round each and loses to the two-pass latency form:
  // take the plan with the most workgroups that stays in that form.  Create
  // at 2 MiB blocks, 64 / 115 blocks (the config-4 tree blob): 355 -> 499 /
  // 546 -> 590 GiB/s; 128 x 1 MiB 362 -> 506; 200 x 2 MiB and up, or 256 x
  // 1 MiB and up, keep the one-launch plan (scripts/r4_plan_sweep.py,
  // DESIGN.md section 5)
  const uint64_t lat = uint64_t(g_latency_wgs.load(std::memory_order_relaxed)) * 5 / 8;
  if (GLFSX_LAT_ADJ && sl > 0 && g <= 4 && (n << sl) > lat && (n << sl) < kDcMinWgs) {
    int bg = 0;
    uint32_t bsl = 0;
    for (int gg = g0, s = int(sl0); gg >= 1 && s <= int(kMaxSplitLog2); gg /= 2, ++s)
      if ((n << s) <= lat) {
        bg = gg;
        bsl = uint32_t(s);
      }
    if (bg && bsl > 0) {
      g = bg;
      sl = bsl;
    }
  }
  *g_out = g;
  *sl_out = sl;
}

// BLAKE3-only pass in quad layout (k_quad): latency-bound launches of at
// most 16384 chunks, messages of at most 64 x 256 KiB.  Messages of up to
// 64 x 64 KiB (4 MiB: index nodes at 1-4 MiB blocks) use 64 quads per
// workgroup, larger ones 256 (the last workgroup merges <= 64 CVs, one per
// quad of its own).
int quad_qpw(uint64_t maxlen) { return maxlen <= (64ull << 16) ? 64 : 256; }

hipError_t launch_quad(KArgs a, uint64_t maxlen, hipStream_t s) {
  const int qpw = quad_qpw(maxlen);
  const uint64_t kSpan = uint64_t(qpw) << 10;
  const uint64_t W = maxlen > kSpan ? (maxlen + kSpan - 1) / kSpan : 1;
  uint32_t sl = 0;
  while ((1ull << sl) < W) ++sl;
  a.split_log2 = sl;
  a.scratch = nullptr;
  a.cnt = nullptr;
  if (sl) {
    hipError_t e = scratch_get(&a, a.n << sl, a.n, s);
    if (e != hipSuccess) return e;
  }
  if (qpw == 64)
    hipLaunchKernelGGL(k_quad<64>, dim3(uint32_t(a.n << sl)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_quad<256>, dim3(uint32_t(a.n << sl)), dim3(1024), 0, s, a);
  return hipGetLastError();
}

bool quad_ok(const KArgs &a, uint64_t maxlen, bool aligned, uint32_t sl) {
  const uint64_t chunks = a.n * (maxlen ? (maxlen + 1023) >> 10 : 1);
  const bool refs4 = ((reinterpret_cast<uintptr_t>(a.refs) | a.out_off |
                       a.ref_stride) & 3) == 0;
  return aligned && refs4 && (a.n << sl) <= latency_wgs() &&
         chunks <= 16384 && maxlen <= (64ull * 256) << 10;
}

template <bool CHACHA>
hipError_t launch_pass(KArgs a, uint64_t maxlen, bool aligned,
                       hipStream_t s) {
  int g;
  uint32_t sl;
  pass_plan(a.n, maxlen, &g, &sl);
  if constexpr (!CHACHA) {
    if (quad_ok(a, maxlen, aligned, sl)) return launch_quad(a, maxlen, s);
  }
  a.split_log2 = sl;
  a.scratch = nullptr;
  a.cnt = nullptr;
  if (sl) {
    hipError_t e = scratch_get(&a, a.n << sl, a.n, s);
    if (e != hipSuccess) return e;
  }
  hipError_t e;
  switch (g) {
    case 1: e = launch_g<1, CHACHA>(a, aligned, s); break;
    case 2: e = launch_g<2, CHACHA>(a, aligned, s); break;
    case 4: e = launch_g<4, CHACHA>(a, aligned, s); break;
    case 8: e = launch_g<8, CHACHA>(a, aligned, s); break;
    case 16: e = launch_g<16, CHACHA>(a, aligned, s); break;
    case 32: e = launch_g<32, CHACHA>(a, aligned, s); break;
    case 64: e = launch_g<64, CHACHA>(a, aligned, s); break;
    default: e = hipErrorInvalidValue;
  }
  return e;
}

#ifndef GLFSX_SMALL_DEK
#define GLFSX_SMALL_DEK 2
#endif
#ifndef GLFSX_SMALL_CID
// form 1 (quarter-round order), as the headline's CID pass: 928.8 vs 913.3
// GiB/s small blobs, config 4 798.1 vs 787.3 (3 interleaved reps, after the
// wave-offset fix; round 2 measured form 2 ahead when half the waves took
// the per-lane path)
#define GLFSX_SMALL_CID 1
#endif
// k_small_q's counter banks on stream s (current device) and this launch's
// epoch.
hipError_t small_q_get(hipStream_t s, uint32_t **ctr, uint32_t *epoch) {
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return sd.e;
  const int dev = sd.dev;
  hipError_t e = hipSuccess;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  ScratchSlot *sl = nullptr;
  for (ScratchSlot &x : g_scratch)
    if (x.dev == dev && x.stream == s) sl = &x;
  if (!sl) {
    g_scratch.push_back({dev, s, nullptr, 0, nullptr, 0, nullptr, 0, 0, nullptr,
                         nullptr, nullptr, nullptr, DcConst{}, nullptr, 0});
    sl = &g_scratch.back();
  }
  if (!sl->qctr) {
    e = hipMalloc(reinterpret_cast<void **>(&sl->qctr), 64 * 4);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(sl->qctr, 0, 64 * 4, s);
    if (e != hipSuccess) return e;
  }
  *ctr = sl->qctr;
  *epoch = ++sl->qepoch;
  return hipSuccess;
}

// Workgroups of kernel k the whole chip holds at once.
template <class K>
uint32_t resident_wgs(K k) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return uint32_t(std::max(per_cu, 1) * std::max(cus, 1));
}

// k_small_q hands out the last 1/kSmallFineDiv of the blobs as fine items.
// 1 M x 4 KiB blobs, 3 interleaved reps: small blobs 911 / 919 / 926 GiB/s
// at none / 1/4 / 1/8, config 4 end to end 780 / 791 / 801.
constexpr uint32_t kSmallFineDiv = 8;

template <int G, bool CHACHA, int A>
hipError_t launch_small_q(const SArgs &a0, hipStream_t s) {
  static const uint32_t slots = resident_wgs(k_small_q<G, CHACHA, A>);
  uint32_t *ctr;
  uint32_t epoch;
  hipError_t e = small_q_get(s, &ctr, &epoch);
  if (e != hipSuccess) return e;
  SArgs a = a0;
  const uint64_t fine = G > 1 ? a.n / kSmallFineDiv : 0;
  a.n_coarse = (a.n - fine) >> 6;  // whole coarse items; the rest goes fine
  const uint64_t rest = a.n - (a.n_coarse << 6), bpi = G > 1 ? 64 / G : 64;
  const uint64_t items = a.n_coarse + (rest + bpi - 1) / bpi;
  const uint64_t wgs = (items + 3) / 4;
  const uint32_t grid = uint32_t(std::min<uint64_t>(wgs, slots ? slots : wgs));
  hipLaunchKernelGGL((k_small_q<G, CHACHA, A>), dim3(grid), dim3(256), 0, s, a, ctr, epoch);
  return hipGetLastError();
}

template <bool CHACHA>
hipError_t launch_small_pass(const SArgs &a, uint64_t max_len, hipStream_t s) {
  const uint64_t C = max_len ? (max_len + 1023) >> 10 : 1;
  const dim3 grid(uint32_t((a.n + 255) / 256)), block(256);
  const int gsel = C <= 1 ? 1 : C <= 2 ? 2 : C <= 4 ? 4 : C <= 8 ? 8 : C <= 16 ? 16 : 0;
  if (grid.x <= latency_wgs()) {  // few blobs: the compiler's ARX form
    switch (gsel) {
      case 1: hipLaunchKernelGGL((k_small<1, CHACHA, false>), grid, block, 0, s, a); break;
      case 2: hipLaunchKernelGGL((k_small<2, CHACHA, false>), grid, block, 0, s, a); break;
      case 4: hipLaunchKernelGGL((k_small<4, CHACHA, false>), grid, block, 0, s, a); break;
      case 8: hipLaunchKernelGGL((k_small<8, CHACHA, false>), grid, block, 0, s, a); break;
      case 16: hipLaunchKernelGGL((k_small<16, CHACHA, false>), grid, block, 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  // more workgroups than the chip holds: per-wave items (k_small_q), in the
  // ARX form GLFSX_SMALL_DEK / _CID
  constexpr int F = CHACHA ? GLFSX_SMALL_CID : GLFSX_SMALL_DEK;
  switch (gsel) {
    case 1: return launch_small_q<1, CHACHA, F>(a, s);
    case 2: return launch_small_q<2, CHACHA, F>(a, s);
    case 4: return launch_small_q<4, CHACHA, F>(a, s);
    case 8: return launch_small_q<8, CHACHA, F>(a, s);
    case 16: return launch_small_q<16, CHACHA, F>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// The clock probe (g_clk): off until clock_probe is first called.
std::atomic<bool> g_clk_on{false};
std::atomic<unsigned long long *> g_clk_addr[64];
unsigned long long *clk_words() {
  if (!g_clk_on.load(std::memory_order_relaxed)) return nullptr;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
  unsigned long long *p = g_clk_addr[d].load(std::memory_order_acquire);
  if (!p) {
    void *q = nullptr;
    if (hipGetSymbolAddress(&q, HIP_SYMBOL(g_clk)) != hipSuccess) return nullptr;
    p = static_cast<unsigned long long *>(q);
    g_clk_addr[d].store(p, std::memory_order_release);
  }
  return p;
}

KArgs make_args(const PostJob &job) {
  KArgs a{};
  a.clk = clk_words();
  a.src = job.src;
  a.ctext = job.ctext;
  a.stride = job.stride;
  a.msg_len = job.msg_len;
  a.last_len = job.last_len;
  a.n = job.n;
  a.refs = job.out.refs;
  a.ref_bf = job.out.bf;
  a.ref_stride = job.out.stride;
  return a;
}

bool is_aligned(const PostJob &job) {
  const uintptr_t x = reinterpret_cast<uintptr_t>(job.src) |
                      reinterpret_cast<uintptr_t>(job.ctext) |
                      uintptr_t(job.stride);
  return (x & 15) == 0;
}

}  // namespace

void words_from_key(uint32_t w[8], const uint8_t key[32]) {
  for (int i = 0; i < 8; ++i)
    w[i] = uint32_t(key[4 * i]) | (uint32_t(key[4 * i + 1]) << 8) |
           (uint32_t(key[4 * i + 2]) << 16) | (uint32_t(key[4 * i + 3]) << 24);
}

uint32_t set_split_target(uint32_t wgs) { return g_split_target.exchange(wgs); }

uint32_t set_latency_wgs(uint32_t wgs) { return g_latency_wgs.exchange(wgs); }

void release_stream_scratch(hipStream_t s) {
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (size_t i = 0; i < g_scratch.size(); ++i) {
    if (g_scratch[i].stream != s) continue;
    if (sd.dev == g_scratch[i].dev) {
      if (g_scratch[i].p) (void)hipFree(g_scratch[i].p);
      if (g_scratch[i].cnt) (void)hipFree(g_scratch[i].cnt);
      if (g_scratch[i].ready) (void)hipFree(g_scratch[i].ready);
      if (g_scratch[i].lists) (void)hipFree(g_scratch[i].lists);
      if (g_scratch[i].err) (void)hipHostFree(g_scratch[i].err);
      if (g_scratch[i].dcc) (void)hipFree(g_scratch[i].dcc);
      if (g_scratch[i].qctr) (void)hipFree(g_scratch[i].qctr);
    } else {
      continue;  // another device's stream of the same handle value
    }
    g_scratch[i] = g_scratch.back();
    g_scratch.pop_back();
    --i;
  }
}

uint32_t fused_errors_take(hipStream_t s) {
  StreamDevice sd(s);
  if (sd.e != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (ScratchSlot &x : g_scratch)
    if (x.dev == sd.dev && x.stream == s && x.err) {
      const uint32_t v = __atomic_exchange_n(x.err, 0u, __ATOMIC_ACQ_REL);
      if (v) {
        g_dc_timeouts.fetch_add(1, std::memory_order_relaxed);
        // a failed launch may leave its counters off zero (it zeroes the
        // other bank); both banks start over at zero
        (void)hipMemsetAsync(x.lists, 0, kListWords * 4, s);
      }
      return v;
    }
  return 0;
}

void fused_debug(uint32_t skip_msg, uint64_t wait_us) {
  g_dc_skip_msg.store(skip_msg, std::memory_order_relaxed);
  g_dc_wait_ticks.store(wait_us ? wait_us * 100 : 100000000ull, std::memory_order_relaxed);
}

uint64_t fused_timeouts() { return g_dc_timeouts.load(std::memory_order_relaxed); }

void blake3_iv_words(uint32_t w[8]) {
  for (int i = 0; i < 8; ++i) w[i] = kIV[i];
}

hipError_t launch_keyed_hash(const PostJob &job, uint32_t out_off,
                             hipStream_t s) {
  if (job.n == 0) return hipSuccess;
  KArgs a = make_args(job);
  for (int i = 0; i < 8; ++i) a.key[i] = job.salt[i];
  a.base = kKeyed;
  a.out_off = out_off;
  const uint64_t maxlen = job.n > 1 ? std::max(job.msg_len, job.last_len)
                                    : job.last_len;
  return launch_pass<false>(a, maxlen, is_aligned(job), s);
}

// The fine-item share of k_pass_dc's CID items: the last ceil(m / 4)
// messages of each work list.
#ifndef GLFSX_DC_FINE_DIV  // A/B switch (tools/build_variant.sh); 0: no fine items
#define GLFSX_DC_FINE_DIV 4
#endif
constexpr uint32_t kDcFineDiv = GLFSX_DC_FINE_DIV;


// Split-mode post of many-wave size in one launch (k_pass_dc): both passes
// of launch_keyed_hash + launch_cid_pass when each would be one k_pass<G,
// CHACHA, true, 2> launch with the same plan.
hipError_t launch_post_fused(const PostJob &job, hipStream_t s, bool *done) {
  *done = false;
  if (!GLFSX_DC || job.n < 2 || !is_aligned(job)) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(job.out.refs) | job.out.stride) & 3) return hipSuccess;
  const uint64_t maxlen = std::max(job.msg_len, job.last_len);
  int g;
  uint32_t sl;
  pass_plan(job.n, maxlen, &g, &sl);
  const uint64_t wgs = job.n << sl;
  // launches of 320-512 workgroups (default threshold) also run fused in the
  // many-wave form: Create of 96 / 128 MiB at 1 MiB blocks (384 / 512
  // workgroups) 359 -> 368 / 451 -> 487 GiB/s, 80 MiB a tie, 64 MiB (256)
  // 6 % slower, so it stays in latency mode (scripts/lat_thr.py)
  if (sl == 0 || wgs * 8 <= uint64_t(latency_wgs()) * 5 || (g != 1 && g != 2 && g != 4))
    return hipSuccess;
  const uint64_t chunks = job.n * ((maxlen + 1023) >> 10);
  KArgs a = make_args(job);
  for (int i = 0; i < 8; ++i) a.key[i] = job.salt[i];
  a.base = kKeyed;
  a.out_off = 32;
  if (quad_ok(a, maxlen, true, sl) || chunks == 0) return hipSuccess;
  a.split_log2 = sl;
  // scratch: DEK CVs (wgs), coarse CID CVs (wgs), fine CID CVs (2 wgs)
  hipError_t e = scratch_get(&a, 4 * wgs, 2 * job.n, s);
  if (e != hipSuccess) return e;
  DcState d{};
  e = dc_get(job.n, s, &d);
  if (e != hipSuccess) return e;
  d.n = uint32_t(job.n);
  d.sl = sl;
  d.fine_div = (g > 1 && sl < kMaxSplitLog2) ? kDcFineDiv : 0u;
  KArgs b = a;
  for (int i = 0; i < 8; ++i) b.key[i] = job.cid_key[i];
  b.base = job.cid_keyed ? kKeyed : 0u;
  b.out_off = 0;
  b.scratch = a.scratch + wgs * 8;
  b.cnt = a.cnt + job.n;
  KArgs c = b;  // fine CID items: twice the workgroups per message
  c.split_log2 = sl + 1;
  c.scratch = b.scratch + wgs * 8;
  uint64_t items = 0;
  for (uint32_t x = 0; x < kLists; ++x) {
    const uint32_t m = dc_list_msgs(d.n, x);
    items += dc_list_items(m, dc_list_fine(m, d.fine_div), sl);
  }
  const dim3 grid{uint32_t(items)}, block{256};
  switch (g) {
    case 1: hipLaunchKernelGGL(k_pass_dc<1>, grid, block, 0, s, a, b, c, d); break;
    case 2: hipLaunchKernelGGL(k_pass_dc<2>, grid, block, 0, s, a, b, c, d); break;
    default: hipLaunchKernelGGL(k_pass_dc<4>, grid, block, 0, s, a, b, c, d); break;
  }
  *done = true;
  e = hipGetLastError();
  if (e != hipSuccess) dc_launch_failed(s);
  return e;
}

hipError_t launch_post(const PostJob &job, hipStream_t s, bool fused) {
  if (job.n == 0) return hipSuccess;
  bool done = false;
  hipError_t e = fused ? launch_post_fused(job, s, &done) : hipSuccess;
  if (e != hipSuccess || done) return e;
  e = launch_keyed_hash(job, 32, s);
  if (e != hipSuccess) return e;
  return launch_cid_pass(job, s);
}

hipError_t launch_cid_pass(const PostJob &job, hipStream_t s) {
  if (job.n == 0) return hipSuccess;
  KArgs a = make_args(job);
  for (int i = 0; i < 8; ++i) a.key[i] = job.cid_key[i];
  a.base = job.cid_keyed ? kKeyed : 0u;
  a.out_off = 0;
  const uint64_t maxlen = job.n > 1 ? std::max(job.msg_len, job.last_len)
                                    : job.last_len;
  int g;
  uint32_t sl;
  pass_plan(job.n, maxlen, &g, &sl);
  // Latency-bound launches (index nodes, single posts, small batches): the
  // fused pass leaves one wave per SIMD running ChaCha20 and BLAKE3 in
  // series.  The keystream has no chaining, so instead every 64-B block gets
  // its own lane (the read side's kernels: ctext = ptext ^ ChaCha20(DEK_j)),
  // and the CID is a BLAKE3 pass over the ctext like the DEK pass.  Needs
  // the ctext in memory, DEKs in dense slots, contiguous messages.
  const bool dense = job.out.bf >= job.n;
  const bool contiguous = job.n == 1 || job.stride == job.msg_len;
  if ((job.n << sl) <= latency_wgs() && job.ctext && dense && contiguous &&
      (job.n == 1 || job.msg_len % 64 == 0)) {
    const uint64_t bs = job.n > 1 ? job.msg_len
                                  : std::max<uint64_t>(4096, (job.last_len + 4095) & ~4095ull);
    hipError_t e = launch_decrypt(job.src, job.ctext, job.n, bs, job.last_len,
                                  job.out.refs, s);
    if (e != hipSuccess) return e;
    KArgs b = a;
    b.src = job.ctext;
    b.ctext = nullptr;
    const bool aligned = ((reinterpret_cast<uintptr_t>(job.ctext) |
                           uintptr_t(job.stride)) & 15) == 0;
    return launch_pass<false>(b, maxlen, aligned, s);
  }
  return launch_pass<true>(a, maxlen, is_aligned(job), s);
}

hipError_t launch_fill(uint8_t *dst, uint64_t offset, uint64_t n, uint64_t seed,
                       hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (offset & 7) return hipErrorInvalidValue;
  const uint64_t words = (n + 7) >> 3;
  uint64_t grid = (words + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(k_fill, dim3(uint32_t(grid)), dim3(256), 0, s, dst, offset,
                     n, seed);
  return hipGetLastError();
}

hipError_t launch_post_small(const SmallJob &job, hipStream_t s) {
  if (job.n == 0) return hipSuccess;
  // blobs above small_max are skipped by k_small (posted elsewhere)
  const uint64_t small_max = job.small_max ? std::min(job.small_max, kMaxSmallLen)
                                           : kMaxSmallLen;
  const uint64_t max_len = std::min(job.max_len, small_max);
  SArgs a{};
  a.small_max = small_max;
  a.src = job.src;
  a.ctext = job.ctext;
  a.offs = job.offs;
  a.lens = job.lens;
  a.n = job.n;
  a.refs = job.refs;
  for (int i = 0; i < 8; ++i) {
    a.key[i] = job.raw_salt[i];
    a.key0[i] = job.index_salt[i];
  }
  a.base = kKeyed;
  a.out_off = 32;
  hipError_t e = hipSuccess;
  if (job.passes != 2) {
    e = launch_small_pass<false>(a, max_len, s);
    if (e != hipSuccess || job.passes == 1) return e;
  }
  for (int i = 0; i < 8; ++i) a.key[i] = a.key0[i] = job.cid_key[i];
  a.base = job.cid_keyed ? kKeyed : 0u;
  a.out_off = 0;
  a.hex_out = job.hex_out;
  a.hex_pos = job.hex_pos;
  if (job.cid_wait) {  // e.g. the tree lines' static parts, on another stream
    e = hipStreamWaitEvent(s, job.cid_wait, 0);
    if (e != hipSuccess) return e;
  }
  return launch_small_pass<true>(a, max_len, s);
}

#if GLFSX_ONE_TIMING
extern "C" int glfsx_debug_one_timing(int reset, uint64_t out[16]) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_one_t), 16 * sizeof(uint64_t), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (!reset) return 0;
  const unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_one_t), z, sizeof z, 0, hipMemcpyHostToDevice) ==
                 hipSuccess ? 0 : -1;
}
#endif

hipError_t clock_probe(int reset, uint64_t out[2]) {
  g_clk_on.store(true, std::memory_order_relaxed);
  unsigned long long v[2] = {0, 0};
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_clk), sizeof v, 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  if (out) {
    out[0] = v[0];
    out[1] = v[1];
  }
  if (!reset) return hipSuccess;
  const unsigned long long z[2] = {0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_clk), z, sizeof z, 0, hipMemcpyHostToDevice);
}

#if GLFSX_WGTIME
hipError_t debug_wgtime(uint64_t *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wgtime), sizeof(g_wgtime), 0,
                             hipMemcpyDeviceToHost);
}
#endif

hipError_t launch_med(const OneDesc *descs, uint32_t n, uint64_t max_len,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (max_len > kMaxMedLen || max_len <= kMaxOneLen) return hipErrorInvalidValue;
  const uint32_t wmax = uint32_t((max_len + 65535) >> 16);
  hipLaunchKernelGGL(k_med_dek, dim3(n * wmax), dim3(256), 0, s, descs, wmax);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_med_cid, dim3(n * wmax), dim3(256), 0, s, descs, wmax);
  return hipGetLastError();
}

hipError_t launch_one(const OneDesc *descs, uint32_t n, uint64_t max_len,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (max_len > kMaxOneLen) return hipErrorInvalidValue;
  if (max_len <= 16 * 1024)
    hipLaunchKernelGGL(k_one<16>, dim3(n), dim3(64), 0, s, descs);
  else
    hipLaunchKernelGGL(k_one<64>, dim3(n), dim3(256), 0, s, descs);
  return hipGetLastError();
}

hipError_t launch_med_v(const OneDesc &d, hipStream_t s) {
  if (d.len > kMaxMedLen || d.len <= kMaxOneLen) return hipErrorInvalidValue;
  const uint32_t wmax = uint32_t((uint64_t(d.len) + 65535) >> 16);
  hipLaunchKernelGGL(k_med_dek_v, dim3(wmax), dim3(256), 0, s, d, wmax);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_med_cid_v, dim3(wmax), dim3(256), 0, s, d, wmax);
  return hipGetLastError();
}

hipError_t launch_one_v(const OneDesc &d, hipStream_t s) {
  if (d.len > kMaxOneLen) return hipErrorInvalidValue;
  if (d.len <= 16 * 1024)
    hipLaunchKernelGGL(k_one_v<16>, dim3(1), dim3(64), 0, s, d);
  else
    hipLaunchKernelGGL(k_one_v<64>, dim3(1), dim3(256), 0, s, d);
  return hipGetLastError();
}

hipError_t launch_decrypt(const uint8_t *ctext, uint8_t *ptext, uint64_t n,
                          uint64_t bs, uint64_t last_len, const uint8_t *refs,
                          hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (bs % 64) return hipErrorInvalidValue;
  KArgs a{};
  a.src = ctext;
  a.ctext = ptext;
  a.msg_len = bs;
  a.last_len = last_len;
  a.n = n;
  a.refs = const_cast<uint8_t *>(refs);
  const uint64_t total = (n - 1) * bs + last_len;
  const uint64_t kbs = (total + 63) >> 6;
  // bulk: whole 4 KiB units through the line kernel (uniform DEK per unit)
  uint64_t units = 0;
  if (bs % 4096 == 0 && ((reinterpret_cast<uintptr_t>(ctext) |
                          reinterpret_cast<uintptr_t>(ptext)) & 15) == 0)
    units = total >> 12;
  if (units) {
    const uint64_t upb = bs >> 12;
    const uint32_t upb_shift =
        (upb & (upb - 1)) == 0 ? uint32_t(__builtin_ctzll(upb)) : 64u;
    // runs of 2^run_shift units per wave (inside one block), as long as
    // there are still >= 65536 runs: the grid (<= 16384 workgroups of 4
    // waves) stays as fine-grained as with one unit per step
    uint32_t run_shift = 0;
    if (upb_shift < 64)
      while (run_shift < upb_shift && (units >> (run_shift + 1)) >= 65536) ++run_shift;
    const uint64_t runs = (units + (1ull << run_shift) - 1) >> run_shift;
    uint64_t grid = (runs + 3) / 4;
    if (grid > 16384) grid = 16384;
    if (grid <= latency_wgs())
      hipLaunchKernelGGL(k_decrypt_lines<0>, dim3(uint32_t(grid)), dim3(256), 0, s,
                         a, units, upb_shift, run_shift);
    else
      hipLaunchKernelGGL(k_decrypt_lines<2>, dim3(uint32_t(grid)), dim3(256), 0, s,
                         a, units, upb_shift, run_shift);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  a.stride = units << 6;  // first keystream block left for k_decrypt
  if (a.stride >= kbs) return hipSuccess;
  uint64_t grid = (kbs - a.stride + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(k_decrypt, dim3(uint32_t(grid)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_chacha_xor(const uint32_t k[8], const uint8_t *src,
                             uint8_t *dst, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  KArgs a{};
  a.src = src;
  a.ctext = dst;
  a.msg_len = n;
  for (int i = 0; i < 8; ++i) a.key[i] = k[i];
  const uint64_t nblk = (n + 63) >> 6;
  uint64_t grid = (nblk + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(k_chacha_xor, dim3(uint32_t(grid)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace glfsx
