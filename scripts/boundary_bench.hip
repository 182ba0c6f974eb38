// Kernel-boundary cost vs the bytes the previous kernel left dirty in L2, plain vs write-through stores.
//
// Hypothesis under test (reference-batch step, profiles/train_step_bs4.md): a dependent launch after a
// kernel that wrote a few MB pays the end-of-kernel L2 writeback of those lines (every XCD's L2 is
// written back at the release), so small-batch kernels cost several us more than their work. Stores
// with the write-through policy (aux 16 = sc1 on gfx950) leave no dirty lines behind.
//
// For each size S: 200 x [writer(S bytes) -> tiny dependent kernel] on one stream, timed with events;
// the same with sc1 stores; and a baseline of tiny -> tiny pairs. Prints us per pair.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/boundary_bench scripts/boundary_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int AUX>
__global__ __launch_bounds__(256) void writer(uint4* __restrict__ p, long n16, uint32_t v) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(n16 * 16), 0x00020000);
  for (long i = blockIdx.x * 256l + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 d = {v, v + 1, v + 2, (uint32_t)i};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (uint32_t)(i * 16), 0, AUX);
  }
}

__global__ void tiny(int* q) {
  if (threadIdx.x == 0) q[blockIdx.x] += 1;
}

int main() {
  const long maxb = 64l << 20;
  uint4* buf;
  int* q;
  CHECK(hipMalloc(&buf, maxb));
  CHECK(hipMalloc(&q, 4096));
  CHECK(hipMemset(q, 0, 4096));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 200;
  auto timeit = [&](auto&& body) -> float {
    for (int i = 0; i < 20; ++i) body(i);
    hipEventRecord(e0, s);
    for (int i = 0; i < reps; ++i) body(i);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / reps;
  };
  const float base = timeit([&](int) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, q);
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, q);
  });
  printf("tiny -> tiny: %.2f us per pair\n", base);
  const long sizes[] = {256l << 10, 1l << 20, 4l << 20, 16l << 20, 32l << 20, 64l << 20};
  for (long bytes : sizes) {
    const long n16 = bytes / 16;
    const int grid = (int)((n16 + 255) / 256 < 2048 ? (n16 + 255) / 256 : 2048);
    const float w0 = timeit([&](int i) { hipLaunchKernelGGL(writer<0>, dim3(grid), dim3(256), 0, s, buf, n16, (uint32_t)i); });
    const float w16 = timeit([&](int i) { hipLaunchKernelGGL(writer<16>, dim3(grid), dim3(256), 0, s, buf, n16, (uint32_t)i); });
    const float p0 = timeit([&](int i) {
      hipLaunchKernelGGL(writer<0>, dim3(grid), dim3(256), 0, s, buf, n16, (uint32_t)i);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, q);
    });
    const float p16 = timeit([&](int i) {
      hipLaunchKernelGGL(writer<16>, dim3(grid), dim3(256), 0, s, buf, n16, (uint32_t)i);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, q);
    });
    const float p2 = timeit([&](int i) {
      hipLaunchKernelGGL(writer<2>, dim3(grid), dim3(256), 0, s, buf, n16, (uint32_t)i);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, q);
    });
    printf("%6ld KB: writer alone plain %.2f / sc1 %.2f us; writer+tiny plain %.2f / nt %.2f / sc1 %.2f us\n",
           bytes >> 10, w0, w16, p0, p2, p16);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
