// clsbench.hip — dev micro-benchmark for k_sync_classify's access pattern (not part of the product).
// Streams `pairs` (content row, receiver row) pairs of N u32 record words out of an N x N matrix
// (fresh random rows per launch so nothing stays in the 256 MiB MALL) with several work
// decompositions and reports GB/s of algorithmic bytes (2 x 4 B x N per pair).
//   hipcc --offload-arch=gfx950 -O3 -o tools/clsbench tools/clsbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr uint32_t N = 65536;

__device__ __forceinline__ uint32_t mix(uint4 a, uint4 o) { return (a.x ^ o.x) + (a.y ^ o.y) + (a.z ^ o.z) + (a.w ^ o.w); }

// V0: block per (pair, 4096-subject chunk), 16 subjects / thread, static grid-stride (old design)
__global__ void __launch_bounds__(256) v0(const uint32_t* m, const uint2* pairs, uint32_t np, uint32_t* sink) {
  constexpr uint32_t CH = 4096;
  const uint32_t chunks = N / CH;
  uint32_t acc = 0;
  for (uint32_t w = blockIdx.x; w < np * chunks; w += gridDim.x) {
    const uint2 p = pairs[w / chunks];
    const uint32_t base = (w % chunks) * CH;
    const uint32_t* a = m + (size_t)p.x * N + base;
    const uint32_t* o = m + (size_t)p.y * N + base;
    uint4 va[4], vo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) va[j] = *reinterpret_cast<const uint4*>(a + j * 1024 + 4 * threadIdx.x);
#pragma unroll
    for (int j = 0; j < 4; ++j) vo[j] = *reinterpret_cast<const uint4*>(o + j * 1024 + 4 * threadIdx.x);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += mix(va[j], vo[j]);
    if (__syncthreads_or(acc == 0x7fffffffu)) sink[1] = 1;
  }
  if (acc == 0x12345u) sink[0] = acc;
}

// V1: wave per (pair, 1024-subject chunk), interleaved grid-stride, no pipelining, CPW loads/row
template <int CPW>
__global__ void __launch_bounds__(256) v1(const uint32_t* m, const uint2* pairs, uint32_t np, uint32_t* sink) {
  constexpr uint32_t CH = CPW * 256;
  const uint32_t chunks = N / CH, lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  uint32_t acc = 0;
  for (uint32_t w = wid; w < np * chunks; w += nw) {
    const uint2 p = pairs[w / chunks];
    const uint32_t base = (w % chunks) * CH;
    const uint32_t* a = m + (size_t)p.x * N + base;
    const uint32_t* o = m + (size_t)p.y * N + base;
    uint4 va[CPW], vo[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j) va[j] = *reinterpret_cast<const uint4*>(a + j * 256 + 4 * lane);
#pragma unroll
    for (int j = 0; j < CPW; ++j) vo[j] = *reinterpret_cast<const uint4*>(o + j * 256 + 4 * lane);
#pragma unroll
    for (int j = 0; j < CPW; ++j) acc += mix(va[j], vo[j]);
    if (__ballot(acc == 0x7fffffffu)) sink[1] = 1;
  }
  if (acc == 0x12345u) sink[0] = acc;
}

// V2: as V1 with a one-deep software pipeline (next unit's loads issued before processing)
__global__ void __launch_bounds__(256) v2(const uint32_t* m, const uint2* pairs, uint32_t np, uint32_t* sink) {
  constexpr uint32_t CH = 1024;
  const uint32_t chunks = N / CH, lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  const uint32_t total = np * chunks;
  uint32_t acc = 0;
  if (wid >= total) return;
  uint4 va[4], vo[4], na[4], no[4];
  auto load = [&](uint32_t w, uint4* x, uint4* y) {
    const uint2 p = pairs[w / chunks];
    const uint32_t base = (w % chunks) * CH;
    const uint32_t* a = m + (size_t)p.x * N + base;
    const uint32_t* o = m + (size_t)p.y * N + base;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = *reinterpret_cast<const uint4*>(a + j * 256 + 4 * lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = *reinterpret_cast<const uint4*>(o + j * 256 + 4 * lane);
  };
  load(wid, va, vo);
  for (uint32_t w = wid; w < total; w += nw) {
    const bool more = w + nw < total;
    if (more) load(w + nw, na, no);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += mix(va[j], vo[j]);
    if (__ballot(acc == 0x7fffffffu)) sink[1] = 1;
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { va[j] = na[j]; vo[j] = no[j]; }
    }
  }
  if (acc == 0x12345u) sink[0] = acc;
}

// V3: pure contiguous streaming read of the same byte count (roofline reference)
__global__ void __launch_bounds__(256) v3(const uint4* m, size_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = m[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint32_t np = argc > 1 ? atoi(argv[1]) : 218;
  const int sets = 24;
  uint32_t* m = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&m, sizeof(uint32_t) * (size_t)N * N) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&sink, 8);
  hipMemset(m, 1, sizeof(uint32_t) * (size_t)N * N);
  std::vector<uint2> hp((size_t)np * sets);
  srand(7);
  for (auto& x : hp) x = make_uint2(rand() % N, rand() % N);
  uint2* dp = nullptr;
  hipMalloc(&dp, sizeof(uint2) * hp.size());
  hipMemcpy(dp, hp.data(), sizeof(uint2) * hp.size(), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 2.0 * 4.0 * N * np;
  auto run = [&](const char* name, auto launch) {
    for (int s = 0; s < 2; ++s) launch(dp + (size_t)s * np);  // warm-up
    float best = 1e9f, sum = 0.f;
    for (int s = 2; s < sets; ++s) {
      hipEventRecord(e0);
      launch(dp + (size_t)s * np);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
      sum += ms;
    }
    const float avg = sum / (sets - 2);
    printf("%-36s avg %7.2f us  best %7.2f us  %7.0f GB/s (avg)\n", name, avg * 1e3, best * 1e3, bytes / (avg * 1e-3) / 1e9);
  };
  for (int g : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "v0 block/4096 grid %d", g);
    run(nm, [&](const uint2* p) { v0<<<g, 256>>>(m, p, np, sink); });
  }
  for (int g : {512, 1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "v1<4> wave/1024 grid %d", g);
    run(nm, [&](const uint2* p) { v1<4><<<g, 256>>>(m, p, np, sink); });
    snprintf(nm, sizeof nm, "v1<8> wave/2048 grid %d", g);
    run(nm, [&](const uint2* p) { v1<8><<<g, 256>>>(m, p, np, sink); });
    snprintf(nm, sizeof nm, "v1<2> wave/512 grid %d", g);
    run(nm, [&](const uint2* p) { v1<2><<<g, 256>>>(m, p, np, sink); });
    snprintf(nm, sizeof nm, "v2 wave/1024 pipelined grid %d", g);
    run(nm, [&](const uint2* p) { v2<<<g, 256>>>(m, p, np, sink); });
  }
  const size_t n16 = (size_t)bytes / 16;
  for (int g : {1024, 4096, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "v3 contiguous stream grid %d", g);
    run(nm, [&](const uint2* p) { v3<<<g, 256>>>(reinterpret_cast<const uint4*>(m) + (size_t)(p - dp) * n16 % ((size_t)N * N / 4 - n16), n16, sink); });
  }
  return 0;
}
