"""Generate tools/burst.hip: does the order of full-rate (F: v_xor_b32,
v_add_u32) and half-rate (H: v_alignbit_b32, v_add3_u32) instructions inside
a wave's stream change the SIMD's issue rate when several waves share it?

tools/mix.hip found 2 cycles per wave64 instruction for F alone, 4 for H
alone, 3.5 for any F/H mix inside one wave and 2.5 when the classes sit in
different waves.  This asks whether bursts of one class (k F then k H) let
the SIMD overlap one wave's H burst with another wave's F burst, and whether
waves started half a period apart (phase by the hardware wave slot) help.

One 64-lane workgroup per wave; 16 independent register chains; the loop
body is 64 instructions.  Cycles from s_memtime over s_memrealtime (100 MHz)
give the clock; cycles per wave-instruction per SIMD = kernel time x clock /
(waves per SIMD x instructions per wave)."""
import itertools

F_OPS = ["x", "a"]      # v_xor_b32, v_add_u32
H_OPS = ["r", "a3"]     # v_alignbit_b32, v_add3_u32


CHAINS = [16]


def ins(op, i):
    c = CHAINS[0]
    r = f"%{i % c}"
    n = f"%{(i % c + 8) % 16}" if c <= 8 else f"%{(i + 5) % 16}"
    return {
        "x": f"v_xor_b32 {r}, {r}, {n}",
        "a": f"v_add_u32 {r}, {r}, {n}",
        "r": f"v_alignbit_b32 {r}, {r}, {r}, 7",
        "a3": f"v_add3_u32 {r}, {r}, {n}, %16",
    }[op]


def seq(pattern):
    """pattern: list of 'F'/'H' -> alternating concrete ops per class"""
    fi = itertools.cycle(F_OPS)
    hi = itertools.cycle(H_OPS)
    return [next(fi) if c == "F" else next(hi) for c in pattern]


def burst(k):
    return (["F"] * k + ["H"] * k) * (32 // k)


PATTERNS = {
    "F": ["F"] * 64,
    "H": ["H"] * 64,
    "alt1": burst(1),
    "b2": burst(2),
    "b4": burst(4),
    "b8": burst(8),
    "b16": burst(16),
    "b32": burst(32),
    # ChaCha QR step order over 4 QRs: 4 add, 4 xor, 4 rot -> 8F:4H
    "qr4": (["F"] * 8 + ["H"] * 4) * 5 + ["F"] * 4,
    "qr_b16": (["F"] * 16 + ["H"] * 8) * 2 + ["F"] * 16,
}


def body(name, ops, chains=16, nop=False):
    CHAINS[0] = chains
    sep = "\\ns_nop 0\\n" if nop else "\\n"
    text = sep.join(ins(op, i) for i, op in enumerate(ops))
    outs = ",".join(f'"+v"(r[{i}])' for i in range(16))
    return f"""
__device__ __forceinline__ void body_{name}(uint32_t *r, uint32_t k) {{
  asm volatile("{text}" : {outs} : "v"(k));
}}"""


def kernel(kname, a, b):
    """waves whose hardware wave slot is odd run body b, even ones body a"""
    return f"""
__global__ __launch_bounds__(64) void k_{kname}(uint32_t *out, uint32_t iters, uint64_t *clk) {{
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_{b}(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_{a}(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) {{ clk[0] = s1 - s0; clk[1] = w1 - w0; }}
}}"""


KERNELS = []
src = ["#include <hip/hip_runtime.h>\n#include <cstdio>\n#include <cstdlib>\n#include <cstring>\n"]
bodies = {}
for n, p in PATTERNS.items():
    assert len(p) == 64, (n, len(p))
    bodies[n] = seq(p)
    src.append(body(n, bodies[n]))
    KERNELS.append((n, n, n))
# the classes in different waves
KERNELS.append(("split_F_H", "F", "H"))
# bursts with odd wave slots half a period out of phase
for n in ["b4", "b8", "b16", "b32", "qr_b16"]:
    p = PATTERNS[n]
    half = {"b4": 4, "b8": 8, "b16": 16, "b32": 32, "qr_b16": 16}[n]
    rot = p[half:] + p[:half]
    pn = n + "_rot"
    bodies[pn] = seq(rot)
    src.append(body(pn, bodies[pn]))
    KERNELS.append((n + "_phase", n, pn))
# dependent chains (form 1 of the headline CID pass is one chain per wave
# with s_nop 0 between dependent instructions): QR order F F H, G order
# H F H F F H (add3, xor, rot, add, xor, rot)
DEP = {"qr": ["F", "F", "H"] * 21 + ["F"], "g": ["H", "F", "H", "F", "F", "H"] * 10 + ["F"] * 4}
for pn, p in DEP.items():
    for ch in (1, 2, 4):
        for nop in (False, True):
            bn = f"dep_{pn}_c{ch}{'_nop' if nop else ''}"
            bodies[bn] = seq(p)
            src.append(body(bn, bodies[bn], ch, nop))
            KERNELS.append((bn, bn, bn))
for kn, a, b in KERNELS:
    src.append(kernel(kn, a, b))
tbl = ",\n".join(f'  {{"{kn}", (void*)k_{kn}}}' for kn, _, _ in KERNELS)
src.append(f"""
struct K {{ const char *name; void *fn; }};
static K ks_[] = {{
{tbl}
}};
int main(int argc, char **argv) {{
  const uint32_t iters = 2048;
  const int simds = 1024;
  uint32_t *out; uint64_t *clk;
  hipMalloc(&out, size_t(1) << 26);
  hipMalloc(&clk, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int occ : {{2, 4, 6, 8}}) {{
    for (auto &k : ks_) {{
      if (argc > 1 && !strstr(k.name, argv[1])) continue;
      const int blocks = simds * occ;
      void *args[] = {{&out, (void *)&iters, &clk}};
      float best = 1e30f; double ghz = 0;
      for (int rep = 0; rep < 3; ++rep) {{
        hipEventRecord(e0);
        hipLaunchKernel(k.fn, dim3(blocks), dim3(64), args, 0, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        if (ms < best) {{ best = ms; ghz = double(c[0]) / (double(c[1]) * 10.0); }}
      }}
      const double per_simd = double(occ) * iters * 64;
      printf("%-14s occ %d  %8.3f ms  clk %.2f GHz  cyc/instr/SIMD %.2f\\n", k.name, occ, best,
             ghz, best * 1e6 * ghz / per_simd);
    }}
  }}
  return 0;
}}
""")
open("tools/burst.hip", "w").write("".join(src))
