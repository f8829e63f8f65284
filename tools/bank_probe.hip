// Probe: VALU issue rate of v_min_u32/v_max_u32 when both source operands sit
// in the same VGPR bank (index mod 4) vs different banks.  Straight-line asm,
// 4 waves per SIMD, independent instructions.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bank_probe tools/bank_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// 16 independent min/max pairs per iteration on v[8..39]; operand distance D.
#define BODY(D)                                                             \
  "v_min_u32 v40, v8, v" #D "\n v_max_u32 v41, v9, v" #D "\n"             \
  "v_min_u32 v42, v10, v" #D "\n v_max_u32 v43, v11, v" #D "\n"           \
  "v_min_u32 v44, v12, v" #D "\n v_max_u32 v45, v13, v" #D "\n"           \
  "v_min_u32 v46, v14, v" #D "\n v_max_u32 v47, v15, v" #D "\n"

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, int reps) {
  uint32_t r = threadIdx.x;
  if (MODE >= 20 && (threadIdx.x & 63) >= (MODE == 20 ? 32 : 16)) return;  // half / quarter wave
  for (int i = 0; i < reps; ++i) {
    if constexpr (MODE == 0) {  // second operand v20 (bank 0) vs first operands v8..v15 (banks 0..3)
      asm volatile(BODY(20) BODY(20) BODY(20) BODY(20) ::: "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",
                   "v20", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    } else if constexpr (MODE == 1) {  // same-bank pairs only: v8 vs v12, ...
      asm volatile(
          "v_min_u32 v40, v8, v12\n v_max_u32 v41, v9, v13\n v_min_u32 v42, v10, v14\n v_max_u32 v43, v11, v15\n"
          "v_min_u32 v44, v8, v12\n v_max_u32 v45, v9, v13\n v_min_u32 v46, v10, v14\n v_max_u32 v47, v11, v15\n"
          "v_min_u32 v40, v8, v12\n v_max_u32 v41, v9, v13\n v_min_u32 v42, v10, v14\n v_max_u32 v43, v11, v15\n"
          "v_min_u32 v44, v8, v12\n v_max_u32 v45, v9, v13\n v_min_u32 v46, v10, v14\n v_max_u32 v47, v11, v15\n"
          "v_min_u32 v40, v8, v12\n v_max_u32 v41, v9, v13\n v_min_u32 v42, v10, v14\n v_max_u32 v43, v11, v15\n"
          "v_min_u32 v44, v8, v12\n v_max_u32 v45, v9, v13\n v_min_u32 v46, v10, v14\n v_max_u32 v47, v11, v15\n"
          "v_min_u32 v40, v8, v12\n v_max_u32 v41, v9, v13\n v_min_u32 v42, v10, v14\n v_max_u32 v43, v11, v15\n"
          "v_min_u32 v44, v8, v12\n v_max_u32 v45, v9, v13\n v_min_u32 v46, v10, v14\n v_max_u32 v47, v11, v15\n"
          ::: "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    } else if constexpr (MODE >= 3) {
#define OP3(OP) OP " v40, v8, v9, v13\n " OP " v41, v9, v10, v13\n " OP " v42, v10, v11, v13\n " OP " v43, v11, v12, v13\n " \
                OP " v44, v8, v9, v13\n " OP " v45, v9, v10, v13\n " OP " v46, v10, v11, v13\n " OP " v47, v11, v12, v13\n "
#define OPC "v_cmp_lt_u32_e64 s[20:21], v8, v9\n v_cmp_lt_u32_e64 s[22:23], v10, v11\n v_cndmask_b32_e64 v40, v8, v9, s[20:21]\n v_cndmask_b32_e64 v41, v9, v8, s[20:21]\n " \
            "v_cndmask_b32_e64 v42, v10, v11, s[22:23]\n v_cndmask_b32_e64 v43, v11, v10, s[22:23]\n v_cmp_lt_u32_e64 s[20:21], v12, v9\n v_cndmask_b32_e64 v44, v12, v9, s[22:23]\n "
#define OPD "v_mov_b32_dpp v40, v8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v41, v9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n " \
            "v_mov_b32_dpp v42, v10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v43, v11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n " \
            "v_mov_b32_dpp v44, v8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v45, v9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n " \
            "v_mov_b32_dpp v46, v10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v47, v11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n "
#define OPB(OP) OP " v40, v8, v9\n " OP " v41, v9, v10\n " OP " v42, v10, v11\n " OP " v43, v11, v12\n " \
                OP " v44, v8, v9\n " OP " v45, v9, v10\n " OP " v46, v10, v11\n " OP " v47, v11, v12\n "
      if constexpr (MODE >= 20)
        asm volatile(OPB("v_xor_b32") OPB("v_add_u32") OPB("v_xor_b32") OPB("v_add_u32") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 3)
        asm volatile(OPB("v_mul_f32") OPB("v_mul_f32") OPB("v_mul_f32") OPB("v_mul_f32") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 4)
        asm volatile(OPB("v_xor_b32") OPB("v_xor_b32") OPB("v_xor_b32") OPB("v_xor_b32") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 5)
        asm volatile(OPB("v_min_f32") OPB("v_min_f32") OPB("v_min_f32") OPB("v_min_f32") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 6)
        asm volatile(OP3("v_med3_u32") OP3("v_med3_u32") OP3("v_med3_u32") OP3("v_med3_u32") ::: "v8", "v9", "v10", "v11", "v12", "v13", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 7)
        asm volatile(OP3("v_max3_u32") OP3("v_max3_u32") OP3("v_max3_u32") OP3("v_max3_u32") ::: "v8", "v9", "v10", "v11", "v12", "v13", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 8)
        asm volatile(OPC OPC OPC OPC ::: "v8", "v9", "v10", "v11", "v12", "v13", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "s20", "s21", "s22", "s23");
      else if constexpr (MODE == 9)
        asm volatile(OPB("v_add_u32") OPB("v_add_u32") OPB("v_add_u32") OPB("v_add_u32") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 10)
        asm volatile(OP3("v_bitop3_b32") OP3("v_bitop3_b32") OP3("v_bitop3_b32") OP3("v_bitop3_b32") ::: "v8", "v9", "v10", "v11", "v12", "v13", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      // packed 16-bit compare-exchange halves (two 16-bit keys per VGPR): the
      // candidate for a two-pass hi16 / lo16 radix median
      else if constexpr (MODE == 12)
        asm volatile(OPB("v_pk_min_u16") OPB("v_pk_max_u16") OPB("v_pk_min_u16") OPB("v_pk_max_u16") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 13)
        asm volatile(OPB("v_min_u16") OPB("v_max_u16") OPB("v_min_u16") OPB("v_max_u16") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 14)
        asm volatile(OPB("v_pk_add_u16") OPB("v_pk_add_u16") OPB("v_pk_add_u16") OPB("v_pk_add_u16") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else if constexpr (MODE == 15)
        asm volatile(OPB("v_pk_min_f16") OPB("v_pk_max_f16") OPB("v_pk_min_f16") OPB("v_pk_max_f16") ::: "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
      else
        asm volatile(OPD OPD OPD OPD ::: "v8", "v9", "v10", "v11", "v12", "v13", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    } else {  // different-bank pairs only: v8 vs v9, ...
      asm volatile(
          "v_min_u32 v40, v8, v9\n v_max_u32 v41, v9, v10\n v_min_u32 v42, v10, v11\n v_max_u32 v43, v11, v12\n"
          "v_min_u32 v44, v8, v9\n v_max_u32 v45, v9, v10\n v_min_u32 v46, v10, v11\n v_max_u32 v47, v11, v12\n"
          "v_min_u32 v40, v8, v9\n v_max_u32 v41, v9, v10\n v_min_u32 v42, v10, v11\n v_max_u32 v43, v11, v12\n"
          "v_min_u32 v44, v8, v9\n v_max_u32 v45, v9, v10\n v_min_u32 v46, v10, v11\n v_max_u32 v47, v11, v12\n"
          "v_min_u32 v40, v8, v9\n v_max_u32 v41, v9, v10\n v_min_u32 v42, v10, v11\n v_max_u32 v43, v11, v12\n"
          "v_min_u32 v44, v8, v9\n v_max_u32 v45, v9, v10\n v_min_u32 v46, v10, v11\n v_max_u32 v47, v11, v12\n"
          "v_min_u32 v40, v8, v9\n v_max_u32 v41, v9, v10\n v_min_u32 v42, v10, v11\n v_max_u32 v43, v11, v12\n"
          "v_min_u32 v44, v8, v9\n v_max_u32 v45, v9, v10\n v_min_u32 v46, v10, v11\n v_max_u32 v47, v11, v12\n"
          ::: "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    }
    r += i;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
static void run(const char* tag, uint32_t* out, int waves_per_simd) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * waves_per_simd, reps = 20000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, 10);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, reps);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double instr_per_simd = (double)waves_per_simd * reps * 32;
  printf("%-22s waves/SIMD %d: %.3f ms  %.3f ns per VALU instr per SIMD (%.2f cyc @2.4GHz)\n", tag, waves_per_simd, ms,
         ms * 1e6 / instr_per_simd, ms * 1e-3 / instr_per_simd * 2.4e9);
}

int main() {
  uint32_t* out;
  CHECK(hipMalloc(&out, 256 * 1024 * 8 * 4));
  for (int w : {1, 2}) {
    run<4>("xor/add full wave", out, w);
    run<20>("xor/add 32 lanes", out, w);
    run<21>("xor/add 16 lanes", out, w);
  }
  for (int w : {2, 4}) {
    run<2>("min/max u32", out, w);
    run<3>("v_mul_f32", out, w);
    run<4>("v_xor_b32", out, w);
    run<9>("v_add_u32", out, w);
    run<6>("v_med3_u32", out, w);
    run<7>("v_max3_u32", out, w);
    run<10>("v_bitop3_b32", out, w);
    run<8>("v_cmp(e64)+cndmask mix", out, w);
    run<11>("v_mov_b32_dpp", out, w);
    run<12>("v_pk_min/max_u16", out, w);
    run<13>("v_min/max_u16", out, w);
    run<14>("v_pk_add_u16", out, w);
    run<15>("v_pk_min/max_f16", out, w);
  }
  return 0;
}
