// valu_rates.hip — diagnostic (not part of the product): issue rate of the
// VALU instructions the integer kernels are made of, on this part, so that
// the VALU rooflines in bench.py / DESIGN.md use measured per-instruction
// costs instead of guesses.  Each kernel runs 8 independent dependency chains
// per lane (enough ILP to hide latency at 8 waves/SIMD) of one instruction.
//
// build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;

#define BODY(OP)                                                   \
  for (int it = 0; it < kIters; ++it) {                            \
    _Pragma("unroll") for (int c = 0; c < kChains; ++c) { OP; }    \
  }

__global__ void k_add(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_xor(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_alignbit(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_mul_lo(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_mul_hi(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_mad64(uint32_t* out, uint32_t s) {
  uint64_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v[c]) : "v"(s) : "vcc"));
  uint64_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = static_cast<uint32_t>(r);
}

__global__ void k_fma64(uint32_t* out, uint32_t s) {
  double v[kChains];
  const double m = 1.0 + s * 1e-12;
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(v[c]) : "v"(m)));
  double r = 0;
  for (int c = 0; c < kChains; ++c) r += v[c];
  if (r == 1.2345) out[0] = 1;
}

__global__ void k_perm(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_lshl_or(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_lshl_or_b32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_add3(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(v[c]) : "v"(s)));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}

__global__ void k_addc(uint32_t* out, uint32_t s) {
  uint32_t v[kChains];
  for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;
  BODY(asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(v[c]) : "v"(s) : "vcc"));
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= v[c];
  if (r == 0x1234567u) out[0] = r;
}


// encodings: a VOP2 op in its 64-bit VOP3 form, SDWA and DPP forms, bitop3 / bfi
#define K1(NAME, INSN)                                                   \
  __global__ void NAME(uint32_t* out, uint32_t s) {                     \
    uint32_t v[kChains];                                                 \
    for (int c = 0; c < kChains; ++c) v[c] = threadIdx.x + c;            \
    BODY(asm volatile(INSN : "+v"(v[c]) : "v"(s)));                     \
    uint32_t r = 0;                                                      \
    for (int c = 0; c < kChains; ++c) r ^= v[c];                         \
    if (r == 0x1234567u) out[0] = r;                                     \
  }
K1(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
K1(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
K1(k_mov_sdwa, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2")
K1(k_add_dpp, "v_add_u32_dpp %0, %1, %0 row_shr:1 bound_ctrl:0")
K1(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
K1(k_bfi, "v_bfi_b32 %0, %1, %0, %1")
K1(k_pk_add, "v_pk_add_u16 %0, %0, %1")
K1(k_lshl_e32, "v_lshlrev_b32_e32 %0, %1, %0")

template <typename K>
static void run(const char* name, K k, int ops_per_body) {
  uint32_t* out;
  CHECK(hipMalloc(&out, 64));
  const int grid = 256 * 8, block = 256;  // 8 waves per SIMD on 256 CUs
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, out, 3u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, out, 3u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double lane_ops = 5.0 * grid * block * (double)kIters * kChains * ops_per_body;
  const double per_s = lane_ops / (ms * 1e-3);
  // wave-instructions per SIMD per cycle at 2.4 GHz on 1024 SIMDs
  const double ipc = per_s / 64.0 / 1024.0 / 2.4e9;
  std::printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4g, \"wave_instr_per_simd_cycle\": %.4f}\n", name, per_s, ipc);
  CHECK(hipFree(out));
}

int main() {
  run("v_add_u32", k_add, 1);
  run("v_xor_b32", k_xor, 1);
  run("v_alignbit_b32", k_alignbit, 1);
  run("v_mul_lo_u32", k_mul_lo, 1);
  run("v_mul_hi_u32", k_mul_hi, 1);
  run("v_mad_u64_u32", k_mad64, 1);
  run("v_fma_f64", k_fma64, 1);
  run("v_perm_b32", k_perm, 1);
  run("v_lshl_or_b32", k_lshl_or, 1);
  run("v_add3_u32", k_add3, 1);
  run("v_addc_co_u32", k_addc, 1);
  run("v_xor_b32_e64", k_xor_e64, 1);
  run("v_xor_b32_sdwa", k_xor_sdwa, 1);
  run("v_mov_b32_sdwa", k_mov_sdwa, 1);
  run("v_add_u32_dpp", k_add_dpp, 1);
  run("v_bitop3_b32", k_bitop3, 1);
  run("v_bfi_b32", k_bfi, 1);
  run("v_pk_add_u16", k_pk_add, 1);
  run("v_lshlrev_b32_e32", k_lshl_e32, 1);
  return 0;
}
