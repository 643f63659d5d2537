// ipc_check.hip — hardware check of the RCCL transport's memory mapping (tools only): the exchange
// region of a rank is allocated uncached (hipExtMallocWithFlags(hipDeviceMallocUncached), engine.hip
// xreg_alloc) and mapped into the other ranks' processes with hipIpcGetMemHandle /
// hipIpcOpenMemHandle (setup_peers_rccl).  The one-rank RCCL engine exercises the handle export only;
// this program exercises the OTHER process's side on one GPU: the parent allocates the region, fills
// it on the device, exports the handle and starts itself again as a child process (never exec: the
// parent has touched the GPU), which opens the handle, checks the parent's words with a kernel
// (system-scope loads, as k_pull_rows does) and writes its own; the parent then checks those.
//   ./tools/ipc_check            -> prints "ipc_check ok: ..." or a failure, exit 0 / 1
#include <hip/hip_runtime.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

extern char** environ;

constexpr size_t WORDS = 1u << 22;  // 16 MiB

__global__ void fill(uint32_t* p, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < WORDS; i += (size_t)gridDim.x * blockDim.x)
    __hip_atomic_store(p + i, (uint32_t)(i * 2654435761u) ^ salt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void check(const uint32_t* p, uint32_t salt, uint32_t* bad) {
  uint32_t n = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < WORDS; i += (size_t)gridDim.x * blockDim.x)
    n += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != ((uint32_t)(i * 2654435761u) ^ salt);
  if (n) atomicAdd(bad, n);
}

static int fail(const char* what, hipError_t e) {
  std::printf("ipc_check FAILED: %s: %s\n", what, hipGetErrorString(e));
  return 1;
}

static int count_bad(const uint32_t* p, uint32_t salt, uint32_t* out) {
  uint32_t* bad = nullptr;
  hipError_t e;
  if ((e = hipMalloc(&bad, 4)) != hipSuccess) return fail("hipMalloc", e);
  hipMemset(bad, 0, 4);
  check<<<1024, 256>>>(p, salt, bad);
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("check kernel", e);
  hipMemcpy(out, bad, 4, hipMemcpyDeviceToHost);
  hipFree(bad);
  return 0;
}

int main(int argc, char** argv) {
  hipError_t e;
  if (argc == 3 && std::strcmp(argv[1], "child") == 0) {
    hipIpcMemHandle_t h;
    FILE* f = std::fopen(argv[2], "rb");
    if (!f || std::fread(&h, sizeof h, 1, f) != 1) { std::printf("ipc_check FAILED: child cannot read the handle\n"); return 1; }
    std::fclose(f);
    void* q = nullptr;
    if ((e = hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess)) != hipSuccess) return fail("hipIpcOpenMemHandle", e);
    uint32_t bad = 0;
    if (count_bad(static_cast<uint32_t*>(q), 0x5a5a5a5au, &bad)) return 1;
    if (bad) { std::printf("ipc_check FAILED: child read %u wrong words of the parent's\n", bad); return 1; }
    fill<<<1024, 256>>>(static_cast<uint32_t*>(q), 0xc3c3c3c3u);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("child fill", e);
    if ((e = hipIpcCloseMemHandle(q)) != hipSuccess) return fail("hipIpcCloseMemHandle", e);
    return 0;
  }
  void* p = nullptr;
  bool uncached = true;
  if (hipExtMallocWithFlags(&p, WORDS * 4, hipDeviceMallocUncached) != hipSuccess) {
    uncached = false;
    if ((e = hipMalloc(&p, WORDS * 4)) != hipSuccess) return fail("hipMalloc", e);
  }
  fill<<<1024, 256>>>(static_cast<uint32_t*>(p), 0x5a5a5a5au);
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("parent fill", e);
  hipIpcMemHandle_t h;
  if ((e = hipIpcGetMemHandle(&h, p)) != hipSuccess) return fail(uncached ? "hipIpcGetMemHandle (uncached)" : "hipIpcGetMemHandle", e);
  char path[] = "/tmp/ipc_check_XXXXXX";
  const int fd = mkstemp(path);
  if (fd < 0 || write(fd, &h, sizeof h) != (ssize_t)sizeof h) { std::printf("ipc_check FAILED: handle file\n"); return 1; }
  close(fd);
  char self[4096];
  const ssize_t ln = readlink("/proc/self/exe", self, sizeof self - 1);
  if (ln <= 0) { std::printf("ipc_check FAILED: readlink\n"); return 1; }
  self[ln] = 0;
  char* cargv[] = {self, const_cast<char*>("child"), path, nullptr};
  pid_t pid;
  if (posix_spawn(&pid, self, nullptr, nullptr, cargv, environ) != 0) { std::printf("ipc_check FAILED: spawn\n"); return 1; }
  int st = 0;
  waitpid(pid, &st, 0);
  unlink(path);
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) { std::printf("ipc_check FAILED: child status %d\n", st); return 1; }
  uint32_t bad = 0;
  if (count_bad(static_cast<uint32_t*>(p), 0xc3c3c3c3u, &bad)) return 1;
  if (bad) { std::printf("ipc_check FAILED: parent read %u wrong words of the child's\n", bad); return 1; }
  std::printf("ipc_check ok: %s region of %zu MiB exported by hipIpcGetMemHandle, opened in another process "
              "(hipIpcOpenMemHandle), words written by each side read back by the other with system-scope loads\n",
              uncached ? "uncached (hipDeviceMallocUncached)" : "cached", WORDS * 4 >> 20);
  hipFree(p);
  return 0;
}
