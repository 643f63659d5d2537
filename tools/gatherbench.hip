// gatherbench.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE for the access shapes of the
// storm kernels (not part of the product).  Every kernel touches a KNOWN number of distinct lines
// with no reuse (a permutation of 128-B lines of an 8 GiB buffer: nothing stays in the 256 MiB MALL),
// so counter bytes / access is the counters' tally per access shape:
//   k_cal_stream16    coalesced 16 B / lane streaming read of 1 GiB (the guide's calibration: x2)
//   k_cal_gather4     one random 4-B load per distinct 128-B line
//   k_cal_gather8     one random 8-B load per distinct 128-B line
//   k_cal_gather16    one random 16-B load per distinct 128-B line
//   k_cal_wave256     a wave reads 256 contiguous bytes (4 B / lane) at a random 256-B-aligned offset
//   k_cal_atomic4     one random 4-B atomicOr per distinct 128-B line
//   k_cal_store4      one random 4-B store per distinct 128-B line
//   k_cal_store32     one random 32-B (8 lanes x 4 B) store per distinct 128-B line
// Prints accesses per kernel; tools/gatherbench_summary.py turns the PMC passes into bytes / access.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint64_t BUF_BYTES = 8ull << 30;
constexpr uint64_t NLINES = BUF_BYTES / 128;  // 2^26
constexpr uint32_t COUNT = 1u << 24;          // accesses per random kernel (16 M distinct lines = 2 GiB)
constexpr uint64_t PERM = 2654435761ull;      // odd: i * PERM mod 2^k is a permutation

__device__ __forceinline__ uint64_t line_of(uint32_t i, uint64_t nl) { return ((uint64_t)i * PERM) & (nl - 1); }
__device__ __forceinline__ uint32_t word_of(uint32_t i) { return (i * 0x9E3779B9u) >> 27; }  // 0..31

__global__ void k_cal_stream16(const uint4* p, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x9abcdef1u) sink[0] = acc;
}

__global__ void k_cal_gather4(const uint32_t* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  const uint32_t v = p[line_of(i, NLINES) * 32 + word_of(i)];
  if (v == 0x9abcdef1u) sink[0] = v;
}

__global__ void k_cal_gather8(const uint2* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  const uint2 v = p[line_of(i, NLINES) * 16 + (word_of(i) & 15)];
  if (v.x + v.y == 0x9abcdef1u) sink[0] = v.x;
}

__global__ void k_cal_gather16(const uint4* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  const uint4 v = p[line_of(i, NLINES) * 8 + (word_of(i) & 7)];
  if (v.x + v.y + v.z + v.w == 0x9abcdef1u) sink[0] = v.x;
}

__global__ void k_cal_wave256(const uint32_t* p, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  const uint32_t w = i >> 6, lane = i & 63;
  const uint64_t blk = ((uint64_t)w * PERM) & (NLINES / 2 - 1);  // 256-B blocks
  const uint32_t v = p[blk * 64 + lane];
  if (v == 0x9abcdef1u) sink[0] = v;
}

__global__ void k_cal_atomic4(uint32_t* p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  atomicOr(&p[line_of(i, NLINES) * 32 + word_of(i)], 1u << (i & 31));
}

__global__ void k_cal_store4(uint32_t* p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT) return;
  p[line_of(i, NLINES) * 32 + word_of(i)] = i;
}

__global__ void k_cal_store32(uint32_t* p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= COUNT * 8u) return;
  const uint32_t a = i >> 3, lane = i & 7;
  p[line_of(a, NLINES) * 32 + (word_of(a) & 24) + lane] = i;
}

int main() {
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, BUF_BYTES) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(buf, 1, BUF_BYTES);
  hipDeviceSynchronize();
  const uint32_t blocks = COUNT / 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timed = [&](const char* name, double accesses, auto launch) {
    for (int r = 0; r < 3; ++r) launch();  // three launches each: the summary takes the median
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%s accesses=%.0f us=%.1f accesses_per_s=%.3e\n", name, accesses, ms * 1e3, accesses / (ms * 1e-3));
  };
  const uint64_t n16 = (1ull << 30) / 16;
  timed("k_cal_stream16", (double)(1ull << 30), [&] { k_cal_stream16<<<4096, 256>>>((const uint4*)buf, n16, sink); });
  timed("k_cal_gather4", COUNT, [&] { k_cal_gather4<<<blocks, 256>>>((const uint32_t*)buf, sink); });
  timed("k_cal_gather8", COUNT, [&] { k_cal_gather8<<<blocks, 256>>>((const uint2*)buf, sink); });
  timed("k_cal_gather16", COUNT, [&] { k_cal_gather16<<<blocks, 256>>>((const uint4*)buf, sink); });
  timed("k_cal_wave256", COUNT / 64, [&] { k_cal_wave256<<<blocks, 256>>>((const uint32_t*)buf, sink); });
  timed("k_cal_atomic4", COUNT, [&] { k_cal_atomic4<<<blocks, 256>>>((uint32_t*)buf); });
  timed("k_cal_store4", COUNT, [&] { k_cal_store4<<<blocks, 256>>>((uint32_t*)buf); });
  timed("k_cal_store32", COUNT, [&] { k_cal_store32<<<blocks * 8, 256>>>((uint32_t*)buf); });
  hipDeviceSynchronize();
  hipFree(buf);
  hipFree(sink);
  return 0;
}
