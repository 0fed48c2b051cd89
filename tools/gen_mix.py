"""Generate tools/mix.hip: VALU issue-rate microbenchmarks for the ARX
instruction classes (DESIGN.md "Rooflines").  Each kernel runs 16
independent register chains; the loop body is 64 instructions."""
VARIANTS = {
    "xor":        ["x"] * 64,
    "alignbit":   ["r"] * 64,
    "lshr1":      ["s"] * 64,
    "lshr7":      ["s7"] * 64,
    "lshr16":     ["s16"] * 64,
    "lshl1":      ["l1"] * 64,
    "lshl7":      ["sl"] * 64,
    "lshl16":     ["l16"] * 64,
    "lshl_v":     ["lv"] * 64,
    "lshr_v":     ["rv"] * 64,
    "add_self":   ["aa"] * 64,
    "lshr_b64":   ["r64"] * 64,
    "lshl_b64":   ["l64"] * 64,
    "pk_mov":     ["pm"] * 64,
    "bfe":        ["be"] * 64,
    "mul24":      ["m24"] * 64,
    "mad24":      ["md24"] * 64,
    "mul_lo":     ["ml"] * 64,
    "add_sgpr":   ["as"] * 64,
    "add_sgpr_e64": ["ase"] * 64,
    "pk_lshl16":  ["pl"] * 64,
    "sub":        ["sb"] * 64,
    "not":        ["nt"] * 64,
    "cndmask":    ["cm"] * 64,
    "mov":        ["mv"] * 64,
    "split_fast_slow_dep": ["s7", "x"] * 32,
}
SPLIT = {"split_xor_alignbit": ("xor", "alignbit")}


def ins(op, i):
    r = f"%{i % 16}"
    return {
        "x": f"v_xor_b32 {r}, {r}, %16",
        "xe": f"v_xor_b32_e64 {r}, {r}, %16",
        "ae": f"v_add_u32_e64 {r}, {r}, %16",
        "xs": f"v_xor_b32 {r}, %17, {r}",
        "r": f"v_alignbit_b32 {r}, {r}, {r}, 7",
        "a3": f"v_add3_u32 {r}, {r}, %16, {r}",
        "b3": f"v_bitop3_b32 {r}, {r}, %16, {r} bitop3:0x96",
        "p": f"v_perm_b32 {r}, {r}, {r}, %16",
        "s": f"v_lshrrev_b32 {r}, 1, {r}",
        "s7": f"v_lshrrev_b32 {r}, 7, {r}",
        "s16": f"v_lshrrev_b32 {r}, 16, {r}",
        "l1": f"v_lshlrev_b32 {r}, 1, {r}",
        "l16": f"v_lshlrev_b32 {r}, 16, {r}",
        "lv": f"v_lshlrev_b32 {r}, %16, {r}",
        "rv": f"v_lshrrev_b32 {r}, %16, {r}",
        "aa": f"v_add_u32 {r}, {r}, {r}",
        "r64": f"v_lshrrev_b64 v[40:41], 7, v[42:43]",
        "l64": f"v_lshlrev_b64 v[40:41], 7, v[42:43]",
        "pm": f"v_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]",
        "be": f"v_bfe_u32 {r}, {r}, 3, 9",
        "m24": f"v_mul_u32_u24 {r}, 128, {r}",
        "md24": f"v_mad_u32_u24 {r}, %16, {r}, {r}",
        "ml": f"v_mul_lo_u32 {r}, {r}, %16",
        "as": f"v_add_u32 {r}, %17, {r}",
        "ase": f"v_add_u32_e64 {r}, {r}, %17",
        "pl": f"v_pk_lshlrev_b16 {r}, 3, {r}",
        "sb": f"v_sub_u32 {r}, {r}, %16",
        "nt": f"v_not_b32 {r}, {r}",
        "cm": f"v_cndmask_b32 {r}, {r}, %16, vcc",
        "mv": f"v_mov_b32 {r}, %16",
        "lo": f"v_lshl_or_b32 {r}, {r}, 7, {r}",
        "la": f"v_lshl_add_u32 {r}, {r}, 7, {r}",
        "al": f"v_add_lshl_u32 {r}, {r}, %16, 3",
        "ao": f"v_and_or_b32 {r}, {r}, %16, {r}",
        "o3": f"v_or3_b32 {r}, {r}, %16, {r}",
        "xd": f"v_xad_u32 {r}, {r}, %16, {r}",
        "pk": f"v_pk_add_u16 {r}, {r}, 0 op_sel:[1,0] op_sel_hi:[0,1]",
        "ab": f"v_alignbyte_b32 {r}, {r}, {r}, 1",
        "bf": f"v_bfi_b32 {r}, {r}, %16, {r}",
        "xl": f"v_xor_b32 {r}, 0x12345678, {r}",
        "ai": f"v_add_u32 {r}, 7, {r}",
        "sl": f"v_lshlrev_b32 {r}, 7, {r}",
        "or": f"v_or_b32 {r}, {r}, %16",
        "xr": f"v_xor_b32 {r}, {r}, %{(i + 1) % 16}",
    }[op]


def body(ops):
    return "\\n".join(ins(op, i) for i, op in enumerate(ops))


OUTS = ",".join(f'"+v"(r[{i}])' for i in range(16))


def kernel(name, ops):
    return f"""
__device__ __forceinline__ void body_{name}(uint32_t *r, uint32_t k, uint32_t ks) {{
  asm volatile("{body(ops)}" : {OUTS} : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}}
__global__ __launch_bounds__(256) void k_{name}(uint32_t *out, uint32_t iters) {{
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_{name}(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}}
"""


def split_kernel(name, a, b):
    return f"""
__global__ __launch_bounds__(512) void k_{name}(uint32_t *out, uint32_t iters) {{
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1)
    for (uint32_t it = 0; it < iters; ++it) body_{b}(r, k, ks);
  else
    for (uint32_t it = 0; it < iters; ++it) body_{a}(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}}
"""


src = ["#include <hip/hip_runtime.h>\n#include <cstdio>\n#include <cstdlib>\n#include <cstring>\n"]
for n, ops in VARIANTS.items():
    src.append(kernel(n, ops))
for n, (a, b) in SPLIT.items():
    src.append(split_kernel(n, a, b))
names = list(VARIANTS) + list(SPLIT)
tbl = ",\n".join(f'  {{"{n}", (void*)k_{n}, {512 if n in SPLIT else 256}}}' for n in names)
src.append(f"""
struct K {{ const char *name; void *fn; int threads; }};
static K ks_[] = {{
{tbl}
}};
int main(int argc, char **argv) {{
  const uint32_t iters = 4096;
  int cus = 256;
  uint32_t *out;
  hipMalloc(&out, size_t(1) << 28);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int occ : {{2, 4, 8}}) {{
    for (auto &k : ks_) {{
      if (argc > 1 && !strstr(k.name, argv[1])) continue;
      const int waves_per_block = k.threads / 64;
      const int blocks = cus * 4 * occ / waves_per_block;
      void *args[] = {{&out, (void *)&iters}};
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {{
        hipEventRecord(e0);
        hipLaunchKernel(k.fn, dim3(blocks), dim3(k.threads), args, 0, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }}
      // wave-instructions per SIMD = occ waves x iters x 64
      const double per_simd = double(occ) * iters * 64;
      printf("%-20s occ %d  %8.3f ms  %6.3f ns/instr/SIMD  (= %.2f cyc at 2.1 GHz)\\n", k.name, occ,
             best, best * 1e6 / per_simd, best * 1e6 / per_simd * 2.1);
    }}
  }}
  return 0;
}}
""")
open("tools/mix.hip", "w").write("".join(src))
