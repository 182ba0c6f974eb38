// Collective emulation for single-GPU boxes: a stand-in for one RCCL all-reduce kernel.
//
// The DDP bucket all-reduces (parallel/ddp.py) can only be measured at world > 1 on a multi-GPU node.
// To choose WHERE they are issued (the weight-gradient side stream vs a dedicated collective stream,
// SURVEY.md §7.4) on a one-GPU box, RDP_DDP_EMULATE replaces each natively issued ncclAllReduce by this
// kernel on the same stream: `blocks` workgroups of 256 threads (RCCL's channels each hold one
// workgroup on a CU) that stay resident for the modelled collective time, 2 (n - 1) / n x bytes / bw
// + alpha. Like the real collective it occupies CUs and blocks every later kernel of its stream until
// it completes. The spin reads the constant-rate wall clock (s_memrealtime) and sleeps between reads
// so the waves issue almost nothing.
#include "common.h"

__global__ __launch_bounds__(256) void comm_emulate_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// Traffic mode: the same residency, but the blocks also stream `n4` float4 elements from the scratch's first
// half into its second half (a read + a write each) -- the HBM traffic of a real ring all-reduce
// (reading the send buffer, writing what the peers deliver, reading both to reduce, writing the sum: about
// 3x the bucket through HBM) paced evenly over the modelled time, so it competes with the step's
// memory-bound passes the way RCCL's copies do. Chunk c of a block is issued once the clock passes
// c / chunks of the duration; the last wait runs to the end.
__global__ __launch_bounds__(256) void comm_emulate_traffic_kernel(uint64_t ticks, float4* __restrict__ buf,
                                                                   long n4) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = (long)blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  // 16 loads in flight per lane (64 KiB read + 64 KiB written per chunk and block): a few resident blocks
  // sustain the modelled rate (scripts/comm_emulate_check.py: the kernel must not outlast its modelled time)
  constexpr int U = 16, kChunk = 256 * U;
  const long chunks = hi > lo ? (hi - lo + kChunk - 1) / kChunk : 0;
  for (long c = 0; c < chunks; ++c) {
    const uint64_t due = (uint64_t)((double)ticks * c / chunks);
    while (__builtin_amdgcn_s_memrealtime() - t0 < due) __builtin_amdgcn_s_sleep(2);
    const long base = lo + c * kChunk;
    float4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long i = base + k * 256 + threadIdx.x;
      if (i < hi) v[k] = buf[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long i = base + k * 256 + threadIdx.x;
      if (i < hi) {
        v[k].x += 1.0f;
        buf[n4 + i] = v[k];
      }
    }
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// wall-clock ticks per microsecond of this device (hipDeviceAttributeWallClockRate is in kHz)
static double ticks_per_us() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 100.0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) return 100.0;
  return khz / 1000.0;
}

extern "C" int rdp_comm_emulate(double us, int blocks, hipStream_t s) {
  if (us < 0 || blocks < 1 || blocks > 4096) return -1;
  static thread_local double tpu = ticks_per_us();
  const uint64_t ticks = (uint64_t)(us * tpu);
  hipLaunchKernelGGL(comm_emulate_kernel, dim3(blocks), dim3(256), 0, s, ticks);
  return 0;
}

// scratch: >= 2 * traffic_bytes (16-byte aligned); traffic_bytes: bytes read (and as many written)
extern "C" int rdp_comm_emulate_traffic(double us, int blocks, void* scratch, long scratch_bytes, long traffic_bytes,
                                        hipStream_t s) {
  if (us < 0 || blocks < 1 || blocks > 4096 || traffic_bytes < 0 || (uintptr_t)scratch % 16 ||
      2 * traffic_bytes > scratch_bytes)
    return -1;
  static thread_local double tpu = ticks_per_us();
  const uint64_t ticks = (uint64_t)(us * tpu);
  hipLaunchKernelGGL(comm_emulate_traffic_kernel, dim3(blocks), dim3(256), 0, s, ticks, (float4*)scratch,
                     traffic_bytes / 16);
  return 0;
}
