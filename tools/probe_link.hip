// probe_link.hip - the host link's ceilings for the host path (diagnostic,
// NOT product code; DESIGN.md 4.7, "Round 6: the link"). Prints one JSON
// object per measurement:
//   direct  kernels reading pinned host memory (16-byte loads, all CUs) and
//           writing 16-byte records back to pinned host memory, at the host
//           path's byte ratio (44 B read : 16 B written per frame) and
//           read-only / write-only
//   copy    copy-engine transfers (hipMemcpyAsync) H2D, D2H and both at once,
//           one stream per direction, transfer sizes 64 KiB .. 64 MiB
//   copyT   T host threads, each with its own stream, each issuing transfers
//           of one size (the per-context pattern of direct=0) against one
//           thread issuing the same bytes as transfers T times as large (the
//           pattern a per-process submitter would produce)
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/probe_link.hip -o tools/probe_link -lpthread
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <thread>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

// frames of `rd` 16-byte pieces read per lane-frame, one 16-byte record
// written per frame (wr 0: none); grid-stride over nf frames
__global__ void __launch_bounds__(256) k_direct(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nf,
                                                int rd, int wr, u32x4* __restrict__ sink) {
  u32x4 acc = {0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x; f < nf; f += stride) {
    u32x4 a = {0, 0, 0, 0};
    for (int k = 0; k < rd; k++) a += src[f * (uint64_t)rd + k];
    if (wr) dst[f] = a;
    acc += a;
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[0] = acc;  // keeps the loads
}

static void direct(int ncu) {
  const uint64_t nf = 16ull << 20;  // frames
  const int rds[] = {3, 3, 0};      // 48 B per frame read (the staged 44 B, 16-B pieces) / none
  const int wrs[] = {1, 0, 1};
  const char* names[] = {"read48_write16", "read48", "write16"};
  u32x4 *h_src, *h_dst, *d_sink;
  CK(hipHostMalloc((void**)&h_src, nf * 48, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&h_dst, nf * 16, hipHostMallocDefault));
  CK(hipMalloc((void**)&d_sink, 64));
  memset(h_src, 1, nf * 48);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < 3; v++) {
    for (int gm : {1, 4, 16}) {
      const uint64_t nfv = rds[v] ? nf : nf;
      const int grid = ncu * gm;
      for (int w = 0; w < 2; w++) hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, h_src, h_dst, nfv, rds[v], wrs[v], d_sink);
      CK(hipDeviceSynchronize());
      const int K = 5;
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < K; k++)
        hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, h_src, h_dst, nfv, rds[v], wrs[v], d_sink);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double s = ms / 1e3 / K;
      const double rb = (double)nfv * 16 * rds[v], wb = (double)nfv * 16 * wrs[v];
      printf("{\"probe\": \"direct\", \"pattern\": \"%s\", \"grid\": %d, \"ms\": %.3f, \"read_GBps\": %.2f, "
             "\"write_GBps\": %.2f, \"Mframes_per_s\": %.1f}\n",
             names[v], grid, s * 1e3, rb / s / 1e9, wb / s / 1e9, nfv / s / 1e6);
      fflush(stdout);
    }
  }
  CK(hipHostFree(h_src));
  CK(hipHostFree(h_dst));
  CK(hipFree(d_sink));
}

static void copies() {
  const size_t big = 256ull << 20;
  uint8_t *h_a, *h_b, *d_a, *d_b;
  CK(hipHostMalloc((void**)&h_a, big, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&h_b, big, hipHostMallocDefault));
  CK(hipMalloc((void**)&d_a, big));
  CK(hipMalloc((void**)&d_b, big));
  memset(h_a, 1, big);
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (size_t sz = 64 << 10; sz <= (64u << 20); sz *= 4) {
    const int n = (int)(big / sz);
    for (int mode = 0; mode < 3; mode++) {  // H2D, D2H, both
      for (int w = 0; w < 2; w++) {
        const double t0 = now_s();
        for (int k = 0; k < n; k++) {
          if (mode != 1) CK(hipMemcpyAsync(d_a + k * sz, h_a + k * sz, sz, hipMemcpyHostToDevice, s1));
          if (mode != 0) CK(hipMemcpyAsync(h_b + k * sz, d_b + k * sz, sz, hipMemcpyDeviceToHost, s2));
        }
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        const double s = now_s() - t0;
        if (w == 1) {
          const char* m = mode == 0 ? "h2d" : mode == 1 ? "d2h" : "both";
          printf("{\"probe\": \"copy\", \"dir\": \"%s\", \"bytes\": %zu, \"transfers\": %d, \"GBps_per_dir\": %.2f, "
                 "\"us_per_transfer\": %.2f}\n",
                 m, sz, n, (double)big / s / 1e9, s * 1e6 / n);
          fflush(stdout);
        }
      }
    }
  }
  CK(hipStreamDestroy(s1));
  CK(hipStreamDestroy(s2));
  CK(hipHostFree(h_a));
  CK(hipHostFree(h_b));
  CK(hipFree(d_a));
  CK(hipFree(d_b));
}

// T threads x transfers of sz (own stream each) vs one thread x transfers of T*sz
static void copy_threads(int T, size_t sz, double secs) {
  const size_t per = 64ull << 20;  // each thread's region
  std::vector<uint8_t*> h(T), d(T);
  std::vector<hipStream_t> st(T);
  for (int t = 0; t < T; t++) {
    CK(hipHostMalloc((void**)&h[t], per, hipHostMallocDefault));
    CK(hipMalloc((void**)&d[t], per));
    CK(hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking));
  }
  std::atomic<uint64_t> bytes{0};
  std::atomic<int> go{0};
  auto worker = [&](int t, size_t tsz) {
    while (!go.load()) {
    }
    const double t0 = now_s();
    uint64_t b = 0;
    size_t off = 0;
    int inflight = 0;
    while (now_s() - t0 < secs) {
      CK(hipMemcpyAsync(d[t] + off, h[t] + off, tsz, hipMemcpyHostToDevice, st[t]));
      b += tsz;
      off = off + 2 * tsz <= per ? off + tsz : 0;
      if (++inflight == 8) {
        CK(hipStreamSynchronize(st[t]));
        inflight = 0;
      }
    }
    CK(hipStreamSynchronize(st[t]));
    bytes += b;
  };
  for (int pass = 0; pass < 2; pass++) {
    const int nt = pass == 0 ? T : 1;
    const size_t tsz = pass == 0 ? sz : sz * T;
    bytes = 0;
    go = 0;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(worker, t, tsz);
    const double t0 = now_s();
    go = 1;
    for (auto& x : th) x.join();
    const double s = now_s() - t0;
    printf("{\"probe\": \"copyT\", \"threads\": %d, \"transfer_bytes\": %zu, \"GBps\": %.2f, \"transfers_per_s\": %.0f}\n",
           nt, tsz, bytes.load() / s / 1e9, bytes.load() / (double)tsz / s);
    fflush(stdout);
  }
  for (int t = 0; t < T; t++) {
    CK(hipHostFree(h[t]));
    CK(hipFree(d[t]));
    CK(hipStreamDestroy(st[t]));
  }
}

int main(int argc, char** argv) {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const char* what = argc > 1 ? argv[1] : "all";
  if (!strcmp(what, "all") || !strcmp(what, "direct")) direct(ncu);
  if (!strcmp(what, "all") || !strcmp(what, "copy")) copies();
  if (!strcmp(what, "all") || !strcmp(what, "copyT")) {
    // a C2 batch closed on the 50-us timer at 16 threads holds ~5000 frames:
    // 220 KB staged, 80 KB of records
    copy_threads(16, 220u << 10, 1.0);
    copy_threads(16, 1u << 20, 1.0);
  }
  return 0;
}
