// launchbench.hip — dev micro-benchmark (not part of the product): the per-kernel floor of
// back-to-back dependent launches on one stream, which bounds the latency-bound phase kernels.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launchbench tools/launchbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big { const unsigned* p[96]; unsigned n[64]; };

__global__ void k_empty() {}
__global__ void k_touch(unsigned* out, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += 1;
}
__global__ void k_params(const Big* P, unsigned* out, unsigned n) {
  const Big b = *P;
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && b.n[i & 63] == 12345u) out[i] = b.p[i % 96][0];
}
__global__ void k_stream(const uint4* in, size_t n4, unsigned* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = in[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0xdeadbeefu) sink[0] = 1;
}

template <class F>
static float timeit(hipStream_t s, int reps, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  const unsigned n = 65536;
  unsigned* out;
  Big* P;
  uint4* big;
  const size_t bytes = 128ull << 20;
  hipMalloc(&out, n * 4);
  hipMalloc(&P, sizeof(Big));
  hipMalloc(&big, bytes);
  hipMemset(out, 0, n * 4);
  hipMemset(big, 1, bytes);
  Big h{};
  for (int i = 0; i < 96; ++i) h.p[i] = out;
  hipMemcpy(P, &h, sizeof h, hipMemcpyHostToDevice);
  const int R = 2000;
  printf("empty <<<1,64>>>         %.2f us/launch\n", timeit(s, R, [&] { k_empty<<<1, 64, 0, s>>>(); }));
  printf("empty <<<256,256>>>      %.2f us/launch\n", timeit(s, R, [&] { k_empty<<<256, 256, 0, s>>>(); }));
  printf("touch <<<256,256>>>      %.2f us/launch\n", timeit(s, R, [&] { k_touch<<<256, 256, 0, s>>>(out, n); }));
  printf("params <<<256,256>>>     %.2f us/launch\n", timeit(s, R, [&] { k_params<<<256, 256, 0, s>>>(P, out, n); }));
  printf("params <<<1,256>>>       %.2f us/launch\n", timeit(s, R, [&] { k_params<<<1, 256, 0, s>>>(P, out, n); }));
  const float st = timeit(s, 200, [&] { k_stream<<<2048, 256, 0, s>>>(big, bytes / 16, out); });
  printf("stream 128 MiB           %.2f us/launch (%.0f GB/s)\n", st, bytes / st / 1e3);
  const float st2 = timeit(s, 200, [&] {
    k_stream<<<2048, 256, 0, s>>>(big, bytes / 16, out);
    for (int j = 0; j < 8; ++j) k_params<<<256, 256, 0, s>>>(P, out, n);
  });
  printf("stream + 8 params        %.2f us -> %.2f us per params launch after a stream\n", st2, (st2 - st) / 8);
  return 0;
}
