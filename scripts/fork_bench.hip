// Cost of forking work to a second stream, on the forking (main) queue.
//
// The training step forks every weight gradient to a side stream (models/unet.py _on_side): the main stream
// records an event after the kernel that produced dY and the side stream waits for it. At bs 4 the main
// queue shows a ~5 us gap before the next kernel at every fork (profiles/train_step_bs4.md). This measures
// the main queue's time per [work -> fork -> work] iteration for several fork mechanisms:
//   0  no fork (baseline)
//   1  hipEventRecord (timing off, no system fence) on main + hipStreamWaitEvent on side (the shipped form)
//   2  the same with a default event
//   3  hipStreamWriteValue32 on main + hipStreamWaitValue32 on side (signal memory)
//   4  a one-wave flag kernel on main (plain store, released at kernel end) + hipStreamWaitValue32 on side
// The side stream runs one small kernel per fork. Prints us per iteration (median of 5 runs of 200).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/fork_bench scripts/fork_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// stores over 256 blocks: a short memory-bound kernel like the bs-4 BN passes
__global__ __launch_bounds__(256) void work(float4* __restrict__ p, int n4, float v) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) p[i] = make_float4(v, v, v, (float)i);
}

__global__ void side_work(float* q) {
  if (threadIdx.x == 0) q[blockIdx.x] += 1.f;
}

__global__ void flag_kernel(volatile unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) *flag = v;
}

int main(int argc, char** argv) {
  // work size in MB (argv[1], default 32: each work kernel ~6 us, so the host stays ahead of the GPU and the
  // difference to variant 0 is the fork's cost on the main queue, not host issue time)
  const int mb = argc > 1 ? atoi(argv[1]) : 32;
  const int n4 = (mb << 20) / 16;
  float4* buf;
  float* q;
  CHECK(hipMalloc(&buf, (size_t)n4 * 16));
  CHECK(hipMalloc(&q, 4096));
  CHECK(hipMemset(q, 0, 4096));
  unsigned* flag = nullptr;
  // signal memory (one 8-byte signal) for the wait-value operations; plain device memory if refused
  if (hipExtMallocWithFlags((void**)&flag, 8, hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    printf("(signal memory refused: plain device memory)\n");
    CHECK(hipMalloc((void**)&flag, 64));
  }
  CHECK(hipMemset(flag, 0, 8));
  hipStream_t a, b;
  CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t e0, e1, evf, evd;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreateWithFlags(&evf, hipEventDisableTiming | hipEventDisableSystemFence));
  CHECK(hipEventCreateWithFlags(&evd, hipEventDisableTiming));
  unsigned seq = 0;
  const int iters = 200;
  const char* names[5] = {"no fork", "event (no timing, no system fence)", "event (default)",
                          "stream write / wait value", "flag kernel + wait value"};
  for (int variant = 0; variant < 5; ++variant) {
    std::vector<float> runs;
    for (int rep = 0; rep < 6; ++rep) {
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0, a));
      for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, a, buf, n4, (float)i);
        if (variant == 1 || variant == 2) {
          hipEvent_t ev = variant == 1 ? evf : evd;
          CHECK(hipEventRecord(ev, a));
          CHECK(hipStreamWaitEvent(b, ev, 0));
        } else if (variant == 3) {
          ++seq;
          CHECK(hipStreamWriteValue32(a, flag, seq, 0));
          CHECK(hipStreamWaitValue32(b, flag, seq, hipStreamWaitValueGte, 0xffffffffu));
        } else if (variant == 4) {
          ++seq;
          hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, a, (volatile unsigned*)flag, seq);
          CHECK(hipStreamWaitValue32(b, flag, seq, hipStreamWaitValueGte, 0xffffffffu));
        }
        if (variant != 0) hipLaunchKernelGGL(side_work, dim3(4), dim3(64), 0, b, q);
        hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, a, buf, n4, (float)i + 0.5f);
      }
      CHECK(hipEventRecord(e1, a));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipDeviceSynchronize());
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0) runs.push_back(ms * 1e3f / iters);  // rep 0: warm-up
    }
    std::sort(runs.begin(), runs.end());
    printf("%3d MB  %d  %-38s %7.2f us per [work, fork, work] (min %.2f, max %.2f)\n",
           mb, variant, names[variant], runs[runs.size() / 2], runs.front(), runs.back());
    fflush(stdout);
  }
  return 0;
}
