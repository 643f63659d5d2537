// clsbench_engine.hip — times the engine's own k_sync_classify in isolation (dev tool, not product).
// Builds a converged N x N record matrix (every subject ALIVE inc 0 in every row), queues `np`
// SYNC messages between random (sender, receiver) pairs per launch, and launches the real kernel
// from swim_phases.h with the engine's launch shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/clsbench_engine tools/clsbench_engine.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../scalecube-cluster_amd/csrc/swim_phases.h"

using namespace swimdev;

int main(int argc, char** argv) {
  const uint32_t n = 65536, np = argc > 1 ? atoi(argv[1]) : 218;
  const int sets = 24;
  const int grids[] = {512, 1024, 2048};
  Ctx c{};
  Bufs b{};
  c.n = n; c.lo = 0; c.nl = n; c.sz = n; c.world = 1;
  hipMalloc(&c.recs, sizeof(uint32_t) * (size_t)n * n);
  hipMemset(c.recs, 0, sizeof(uint32_t) * (size_t)n * n);
  // REC_IN_TABLE in every word: fill the high byte of each u32 with 0x80
  hipMemset2D(reinterpret_cast<char*>(c.recs) + 3, 4, 0x80, 1, (size_t)n * n);
  hipMalloc(&c.stats, 8 * ST_COUNT * ST_REPL);
  hipMalloc(&c.err, 4);
  hipMalloc(&b.k, sizeof(Counters));
  b.chunks = n / SYNC_CHUNK;
  b.snap_cap = 64;
  hipMalloc(&b.snap, sizeof(uint32_t) * b.snap_cap * n);
  hipMalloc(&b.snap_idx, 4 * n);
  hipMemset(b.snap_idx, 0xff, 4 * n);
  const uint32_t cap = np * sets;
  hipMalloc(&b.reqs_out, sizeof(SyncReq) * cap);
  hipMalloc(&b.item_chunk, sizeof(uint2) * (size_t)cap * b.chunks);
  hipMalloc(&b.item_total, 4 * cap);
  b.pool_cap = 1 << 22;
  hipMalloc(&b.pool, 4 * b.pool_cap);
  std::vector<SyncReq> hq(cap);
  srand(11);
  for (auto& q : hq) {
    q = SyncReq{};
    q.from = rand() % n; q.to = rand() % n; q.flags = 4; q.content = NONE; q.snap = NONE;
  }
  hipMemcpy(b.reqs_out, hq.data(), sizeof(SyncReq) * cap, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 2.0 * 4.0 * n * np;
  for (int g : grids) {
    float sum = 0.f, best = 1e9f;
    for (int s = 0; s < sets; ++s) {
      Counters k{};
      k.req_cursor = np;
      hipMemcpy(b.k, &k, sizeof k, hipMemcpyHostToDevice);
      Bufs bs = b;
      bs.reqs_out = b.reqs_out + (size_t)s * np;
      bs.item_chunk = b.item_chunk + (size_t)s * np * b.chunks;
      bs.item_total = b.item_total + (size_t)s * np;
      hipEventRecord(e0);
      k_sync_classify<<<g, CLS_BLOCK>>>(c, bs, 0, nullptr);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (s >= 2) { sum += ms; best = ms < best ? ms : best; }
    }
    const float avg = sum / (sets - 2);
    printf("engine k_sync_classify grid %5d: avg %7.2f us best %7.2f us  %6.0f GB/s\n", g, avg * 1e3, best * 1e3,
           bytes / (avg * 1e-3) / 1e9);
  }
  uint32_t err = 0;
  hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost);
  printf("err %u  (%s)\n", err, hipGetErrorString(hipGetLastError()));
  return 0;
}
