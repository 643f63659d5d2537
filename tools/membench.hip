// membench.hip — dev micro-benchmark for the SYNC classify access pattern (not part of the product).
// Streams `pairs` (content row, receiver row) pairs of N u64 cells from a rows x N matrix, with the
// classify kernel's work decomposition, for several row strides / layouts, and reports GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int CHUNK = 4096, BLOCK = 256, CPT = CHUNK / BLOCK;

__global__ void __launch_bounds__(BLOCK) stream_pairs(const unsigned long long* base, size_t stride, const uint2* pairs,
                                                      uint32_t npairs, uint32_t n, unsigned long long* sink) {
  const uint32_t chunks = n / CHUNK;
  unsigned long long acc = 0;
  for (uint32_t w = blockIdx.x; w < npairs * chunks; w += gridDim.x) {
    const uint32_t i = w / chunks, ch = w % chunks;
    const uint2 p = pairs[i];
    const unsigned long long* a = base + (size_t)p.x * stride + (size_t)ch * CHUNK;
    const unsigned long long* o = base + (size_t)p.y * stride + (size_t)ch * CHUNK;
    ulonglong2 va[CPT / 2], vo[CPT / 2];
#pragma unroll
    for (int j = 0; j < CPT / 2; ++j) va[j] = *reinterpret_cast<const ulonglong2*>(a + j * 2 * BLOCK + 2 * threadIdx.x);
#pragma unroll
    for (int j = 0; j < CPT / 2; ++j) vo[j] = *reinterpret_cast<const ulonglong2*>(o + j * 2 * BLOCK + 2 * threadIdx.x);
#pragma unroll
    for (int j = 0; j < CPT / 2; ++j) acc += (va[j].x ^ vo[j].x) + (va[j].y ^ vo[j].y);
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint32_t n = 65536, rows = 65536;
  const uint32_t npairs = argc > 1 ? atoi(argv[1]) : 218;
  const size_t pad_cells[] = {0, 512, 4096 + 64};
  unsigned long long* sink;
  hipMalloc(&sink, 8);
  for (size_t pad : pad_cells) {
    const size_t stride = n + pad;
    unsigned long long* m = nullptr;
    if (hipMalloc(&m, sizeof(unsigned long long) * stride * rows) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(m, 1, sizeof(unsigned long long) * stride * rows);
    for (int mode = 0; mode < 2; ++mode) {
      const int sets = 21;  // a fresh set of rows per launch: nothing stays in the 256 MiB MALL
      std::vector<uint2> hp(npairs * sets);
      srand(7);
      for (uint32_t i = 0; i < npairs * sets; ++i) {
        if (mode == 0) hp[i] = make_uint2(rand() % rows, rand() % rows);           // random rows
        else hp[i] = make_uint2((2 * i) % rows, (2 * i + 1) % rows);               // adjacent rows
      }
      uint2* dp;
      hipMalloc(&dp, sizeof(uint2) * npairs * sets);
      hipMemcpy(dp, hp.data(), sizeof(uint2) * npairs * sets, hipMemcpyHostToDevice);
      for (int grid : {1024, 2048, 4096}) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        stream_pairs<<<grid, BLOCK>>>(m, stride, dp, npairs, n, sink);
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) stream_pairs<<<grid, BLOCK>>>(m, stride, dp + (size_t)(r + 1) * npairs, npairs, n, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 2.0 * npairs * n * 8;
        printf("pad=%zu mode=%s grid=%d: %.1f us/launch, %.0f GB/s\n", pad, mode ? "adjacent" : "random", grid,
               ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
      }
      hipFree(dp);
    }
    hipFree(m);
  }
  return 0;
}
