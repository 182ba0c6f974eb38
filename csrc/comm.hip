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
