// Common CDNA4 (gfx950) helpers for the rdp kernels.
//
// Every global access in the hot kernels goes through a buffer resource (SRD): reads outside
// `num_records` return 0 and writes outside it are dropped, so a wrong index can corrupt an
// output but never fault the GPU (and zero-padding of convolution halos is free: an out-of-range
// voffset reads zeros, also for the LDS-DMA form `buffer_load ... lds`).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RDP_DEV __device__ __forceinline__

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

typedef __attribute__((address_space(3))) void lds_void;

// Offset used for "this lane reads zeros": >= num_records of every descriptor we build (<2 GiB).
#define RDP_OOB 0x80000000u

RDP_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  // wave-uniform by construction: only kernel arguments feed it (cdna_hip_programming.md T8/T20)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// ---- bf16 <-> f32 (round-to-nearest-even; NaN-preserving via the compiler's cvt) ----
RDP_DEV float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }
RDP_DEV u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 at -O3 (keeps NaN a NaN)
  return __builtin_bit_cast(u16, b);
}
// one v_cvt_pk_bf16_f32 (lo, hi) per pair: composing two scalar f2bf conversions let the SLP vectorizer
// pair the wrong operands (two converts + four shuffle ops per two pairs)
typedef __bf16 rdp_bf16x2 __attribute__((ext_vector_type(2)));
typedef float rdp_f32x2 __attribute__((ext_vector_type(2)));
RDP_DEV uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((rdp_f32x2){lo, hi}, rdp_bf16x2));
}

// ---- 16/8-byte buffer loads/stores ----
RDP_DEV uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}
RDP_DEV uint2 bload8(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
  return *reinterpret_cast<uint2*>(&v);
}
RDP_DEV uint32_t bload4(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0);
}
RDP_DEV void bstore16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<__attribute__((ext_vector_type(4))) uint32_t*>(&v), r, voff, 0, 0);
}
RDP_DEV void bstore8(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<__attribute__((ext_vector_type(2))) uint32_t*>(&v), r, voff, 0, 0);
}
RDP_DEV void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
}

// LDS-DMA: 16 bytes per lane, LDS destination = wave-uniform base + lane*16.
RDP_DEV void dma16(__amdgpu_buffer_rsrc_t r, lds_void* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_base, 16, voff, 0, 0, 0);
}

// The same LDS-DMA issued from inline asm. hipcc neither counts it nor orders later LDS reads
// behind it: after the builtin form, hipcc puts `s_waitcnt vmcnt(0)` in front of every
// ds_read_b64_tr_b16 (the transposed-read intrinsic may alias any DMA destination), which drains
// the NEXT stage's DMA before the current stage computes and serialises a double-buffered loop.
// Callers own the bookkeeping: `s_waitcnt vmcnt(N)` + barrier before reading a staged buffer.
// M0 is saved/restored inside the statement (cdna_hip_programming.md §5.7 LDS-DMA recipe).
RDP_DEV void dma16_async(__amdgpu_buffer_rsrc_t r, lds_void* lds_base, uint32_t voff) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_base);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(dst), "s"(r)
      : "memory");
}

RDP_DEV void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
RDP_DEV void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
RDP_DEV void raw_barrier() { __builtin_amdgcn_s_barrier(); }

// ---- XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective") ----
// Blocks are dealt round-robin over 8 XCDs; remap so each XCD gets a contiguous range of logical ids.
RDP_DEV uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  const uint32_t q = nwg >> 3, r = nwg & 7, xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ---- fast unsigned division by a runtime-invariant divisor (magic multiply) ----
struct FastDiv {
  uint32_t d, m, s;  // n / d = (umulhi(n, m) + n) >> s   for n < 2^31
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << s) - d)) / d + 1);
  return f;
}
RDP_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// branch-free 0 <= v < n (no short-circuit control flow around LDS-DMA issue)
RDP_DEV bool inb(int v, int n) { return (unsigned)v < (unsigned)n; }

// Sum over each 16-lane DPP row with 4 VALU DPP ops (no LDS): quad xor1, quad xor2,
// row_half_mirror (8-lane), row_mirror (16-lane). Every lane of the row receives the row sum.
template <int CTRL>
RDP_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
RDP_DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

RDP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
RDP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
