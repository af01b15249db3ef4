// Shared device helpers for the MI355X (gfx950) QMIX/VDN learner kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MQ_DEV __device__ __forceinline__

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace mq {

// Two f32 FMAs in one v_pk_fma_f32 (half the issue slots of two v_fma_f32 at the same FLOP rate).
#ifdef MQ_SCALAR_FMA
MQ_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return f32x2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
#else
MQ_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
#endif

constexpr float kNegMask = -9999999.0f;   // q_learner.py:68,74

// Unsigned 32-bit division by a runtime-invariant divisor: q = (umulhi(x, mul) + x) >> shift, valid for
// x < 2^31 (row/step indices here are far below that). Host computes (mul, shift) once per launch.
struct FastDiv {
  uint32_t d, mul, shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shift = l;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  if (d == 1) { f.mul = 0; f.shift = 0; }
  return f;
}

MQ_DEV uint32_t fdiv(uint32_t x, const FastDiv& f) {
  uint32_t t = __umulhi(x, f.mul);
  return (t + x) >> f.shift;
}

// Global access as a wave-uniform base plus a 32-bit per-lane ELEMENT offset: the byte offset is formed in 32 bits
// and zero-extended, which is the pattern the backend lowers to one saddr load / store (SGPR base + VGPR offset)
// instead of 64-bit VALU address math. The caller guarantees elem * 4 < 2^32.
MQ_DEV float ld_u32(const float* base, uint32_t elem) { return *(const float*)((const char*)base + (elem << 2)); }
MQ_DEV void st_u32(float* base, uint32_t elem, float v) { *(float*)((char*)base + (elem << 2)) = v; }

// Raw buffer stores through a wave-uniform descriptor with a 32-bit per-lane byte offset. An offset of kDrop lies
// past num_records, so the hardware range check drops that lane's store: predicated stores without exec-mask
// branches (which split live ranges and cost register shuffles in the register-capped fused kernels).
constexpr uint32_t kDrop = 0xFFFFFFF0u;
MQ_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7FFFFFF0, 0x00020000);
}
MQ_DEV void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 0);
}
MQ_DEV void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, f32x4 v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 0);
}

// Lane exchange inside an aligned group of 4 lanes (DPP quad_perm, no LDS round trip).
MQ_DEV float quad_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}
MQ_DEV float quad_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
}
// Within each 16-lane DPP row: the value of lane (c + 8) mod 16 (row_ror:8, i.e. lane c ^ 8), and of lane 7 - c
// within each 8-lane half (row_half_mirror; pairs lanes whose bit 2 differs).
MQ_DEV float row_ror8(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, true));
}
MQ_DEV float row_half_mirror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
}
// Broadcast lane L of each quad to the whole quad.
template <int L>
MQ_DEV float quad_bcast(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), L * 0x55, 0xF, 0xF, true));
}
// Sum over the 4 lanes of a quad; every lane of the quad receives the same total ((a+b)+(c+d) order).
MQ_DEV float quad_sum(float v) {
  v = v + quad_xor1(v);
  return v + quad_xor2(v);
}

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup-scope release, which on gfx950 also
// drains every outstanding global load/store (s_waitcnt vmcnt(0)) at each barrier: in the persistent T loops that
// serialised every step behind its own output stores and the next step's prefetch. Nothing in those loops
// communicates through global memory inside the workgroup, so an LDS-only barrier is sufficient.
// s_waitcnt vmcnt(0) as a real instruction (visible to the compiler's wait-count pass). Issued once after a
// kernel's prologue loads so the loop header does not inherit them: otherwise the loop's first use of a
// prologue register is guarded by a vmcnt(N) that, in steady state, also waits for the previous step's stores.
MQ_DEV void drain_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

MQ_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

MQ_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

MQ_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
MQ_DEV float tanhf_(float x) { return tanhf(x); }

}  // namespace mq
