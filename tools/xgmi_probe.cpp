// xgmi_probe: is this MI355X node wired the way the data-parallel engine assumes?
//
// The MI355X-native counterpart of the reference's cluster smoke test
// (/root/reference/mingpt/slurm/mpi_hello_world.c:6-19, which only printed rank + hostname).
// Single process, all local GPUs:
//   1. enumerate devices: name, gfx arch, PCI bus id, CUs, HBM size;
//   2. peer matrix: hipDeviceCanAccessPeer + hipExtGetLinkTypeAndHopCount (expect XGMI, 1 hop,
//      7 peers per GPU on an 8-GPU node);
//   3. per-pair P2P copy bandwidth with hipMemcpyPeerAsync (one xGMI link ~ 150 GB/s);
//   4. local HBM copy bandwidth per GPU;
//   5. an RCCL all-reduce over all local GPUs (ncclCommInitAll): correctness check, then a size
//      sweep printing algorithm / bus bandwidth -- the numbers that size the gradient buckets;
//   6. "hello from rank r on GPU g (bus id)" per rank.
// Links the HIP runtime and RCCL that torch ships (build_ext._torch_runtime_dir), i.e. the RCCL the
// training processes load, and reports its version and path.  With one visible GPU there is no
// link to measure: the P2P and all-reduce bandwidth sections print "n/a" instead of timing no-ops.
// Build: python build_ext.py --tools  ->  build/bin/xgmi_probe [--max-mb N] [--no-p2p]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#define HIPCHECK(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)
#define NCCLCHECK(x)                                                                         \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) {                                                                 \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

static const char* link_name(uint32_t t) {
  switch (t) {
    case HSA_AMD_LINK_INFO_TYPE_HYPERTRANSPORT: return "HT";
    case HSA_AMD_LINK_INFO_TYPE_QPI: return "QPI";
    case HSA_AMD_LINK_INFO_TYPE_PCIE: return "PCIE";
    case HSA_AMD_LINK_INFO_TYPE_INFINBAND: return "IB";
    case HSA_AMD_LINK_INFO_TYPE_XGMI: return "XGMI";
    default: return "?";
  }
}

static double time_copy(int dst, int src, void* d, void* s, size_t bytes, int iters) {
  HIPCHECK(hipSetDevice(src));
  hipStream_t st;
  HIPCHECK(hipStreamCreate(&st));
  hipEvent_t a, b;
  HIPCHECK(hipEventCreate(&a));
  HIPCHECK(hipEventCreate(&b));
  HIPCHECK(hipMemcpyPeerAsync(d, dst, s, src, bytes, st));  // warm
  HIPCHECK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i) HIPCHECK(hipMemcpyPeerAsync(d, dst, s, src, bytes, st));
  HIPCHECK(hipEventRecord(b, st));
  HIPCHECK(hipEventSynchronize(b));
  float ms = 0.f;
  HIPCHECK(hipEventElapsedTime(&ms, a, b));
  HIPCHECK(hipEventDestroy(a));
  HIPCHECK(hipEventDestroy(b));
  HIPCHECK(hipStreamDestroy(st));
  return (double)bytes * iters / (ms * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
  size_t max_mb = 256;
  bool p2p = true;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--max-mb") && i + 1 < argc) max_mb = strtoul(argv[++i], nullptr, 10);
    else if (!strcmp(argv[i], "--no-p2p")) p2p = false;
  }
  int n = 0;
  HIPCHECK(hipGetDeviceCount(&n));
  int ver = 0;
  NCCLCHECK(ncclGetVersion(&ver));
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  const char* node = getenv("SLURM_NODEID");
  Dl_info di{};
  const char* rpath = dladdr((void*)&ncclGetVersion, &di) && di.dli_fname ? di.dli_fname : "?";
  printf("xgmi_probe on %s (node %s): %d GPU(s), RCCL %d.%d.%d (%s)\n", host, node ? node : "0", n,
         ver / 10000, (ver / 100) % 100, ver % 100, rpath);
  std::vector<std::string> bus(n);
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t p;
    HIPCHECK(hipGetDeviceProperties(&p, d));
    char b[64];
    HIPCHECK(hipDeviceGetPCIBusId(b, sizeof(b), d));
    bus[d] = b;
    printf("  GPU %d: %s (%s) bus %s, %d CUs, %.1f GiB HBM, LDS/block %zu KiB\n", d, p.name, p.gcnArchName,
           b, p.multiProcessorCount, p.totalGlobalMem / 1073741824.0, p.sharedMemPerBlock / 1024);
  }
  // ---- peer matrix
  if (n > 1) {
    printf("peer matrix (link type / hops):\n      ");
    for (int j = 0; j < n; ++j) printf("   GPU%-4d", j);
    printf("\n");
    for (int i = 0; i < n; ++i) {
      printf("GPU%-3d", i);
      int peers = 0;
      for (int j = 0; j < n; ++j) {
        if (i == j) {
          printf("   %-7s", "-");
          continue;
        }
        int can = 0;
        HIPCHECK(hipDeviceCanAccessPeer(&can, i, j));
        uint32_t lt = 0, hops = 0;
        if (hipExtGetLinkTypeAndHopCount(i, j, &lt, &hops) != hipSuccess) lt = 0;
        printf("   %s/%u%s", link_name(lt), hops, can ? " " : "!");
        peers += can;
      }
      printf("   (%d peers)\n", peers);
    }
  }
  const size_t bytes = 256ull << 20;
  std::vector<void*> buf(n), buf2(n);
  for (int d = 0; d < n; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMalloc(&buf[d], bytes));
    HIPCHECK(hipMalloc(&buf2[d], bytes));
    HIPCHECK(hipMemset(buf[d], 1, bytes));
  }
  // ---- local HBM copy bandwidth (read + write)
  for (int d = 0; d < n; ++d) {
    double gbs = time_copy(d, d, buf2[d], buf[d], bytes, 10);
    printf("  GPU %d device-local copy: %.0f GB/s (read+write %.0f GB/s)\n", d, gbs, 2 * gbs);
  }
  // ---- P2P bandwidth
  if (n == 1) printf("P2P copy bandwidth: n/a (1 GPU visible: no xGMI link to measure)\n");
  if (p2p && n > 1) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (i != j) {
          HIPCHECK(hipSetDevice(i));
          hipError_t e = hipDeviceEnablePeerAccess(j, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
          (void)hipGetLastError();
        }
    printf("P2P copy bandwidth GB/s (row = src, col = dst):\n");
    for (int i = 0; i < n; ++i) {
      printf("  GPU%-2d", i);
      for (int j = 0; j < n; ++j) {
        if (i == j) {
          printf("  %6s", "-");
          continue;
        }
        printf("  %6.1f", time_copy(j, i, buf2[j], buf[i], 64ull << 20, 5));
      }
      printf("\n");
    }
  }
  // ---- RCCL all-reduce over all local GPUs
  std::vector<ncclComm_t> comms(n);
  std::vector<int> devs(n);
  for (int d = 0; d < n; ++d) devs[d] = d;
  NCCLCHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  std::vector<hipStream_t> streams(n);
  for (int d = 0; d < n; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamCreate(&streams[d]));
    int rank = 0;
    NCCLCHECK(ncclCommUserRank(comms[d], &rank));
    printf("hello from rank %d on GPU %d (%s) of %s\n", rank, d, bus[d].c_str(), host);
  }
  // correctness: rank r contributes (r + 1); expect n(n+1)/2 everywhere
  const size_t cnt = 1 << 20;
  for (int d = 0; d < n; ++d) {
    HIPCHECK(hipSetDevice(d));
    fill_kernel<<<256, 256, 0, streams[d]>>>((float*)buf[d], cnt, (float)(d + 1));
  }
  NCCLCHECK(ncclGroupStart());
  for (int d = 0; d < n; ++d)
    NCCLCHECK(ncclAllReduce(buf[d], buf[d], cnt, ncclFloat, ncclSum, comms[d], streams[d]));
  NCCLCHECK(ncclGroupEnd());
  bool ok = true;
  for (int d = 0; d < n; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamSynchronize(streams[d]));
    float host[4];
    HIPCHECK(hipMemcpy(host, (float*)buf[d] + cnt - 4, sizeof(host), hipMemcpyDeviceToHost));
    for (float v : host) ok &= v == (float)(n * (n + 1) / 2);
  }
  printf("all-reduce correctness: %s\n", ok ? "OK" : "FAILED");
  if (n == 1)
    printf("all-reduce bandwidth: n/a (1 rank: the collective moves no data; run on a multi-GPU node)\n");
  else
    printf("all-reduce sweep (fp32 sum, %d ranks):\n  %10s %10s %12s %12s\n", n, "bytes", "time_us", "algbw_GB/s",
           "busbw_GB/s");
  for (size_t b = 1 << 20; n > 1 && b <= (max_mb << 20) && b <= bytes; b <<= 1) {
    const size_t c = b / 4;
    const int iters = 10;
    for (int w = 0; w < 2; ++w) {  // warm + timed
      auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < iters; ++it) {
        NCCLCHECK(ncclGroupStart());
        for (int d = 0; d < n; ++d)
          NCCLCHECK(ncclAllReduce(buf[d], buf[d], c, ncclFloat, ncclSum, comms[d], streams[d]));
        NCCLCHECK(ncclGroupEnd());
      }
      for (int d = 0; d < n; ++d) {
        HIPCHECK(hipSetDevice(d));
        HIPCHECK(hipStreamSynchronize(streams[d]));
      }
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
      if (w == 1) {
        double alg = b / (us * 1e-6) / 1e9;
        double busf = n > 1 ? 2.0 * (n - 1) / n : 1.0;
        printf("  %10zu %10.1f %12.1f %12.1f\n", b, us, alg, alg * busf);
      }
    }
  }
  for (int d = 0; d < n; ++d) {
    NCCLCHECK(ncclCommDestroy(comms[d]));
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipFree(buf[d]));
    HIPCHECK(hipFree(buf2[d]));
    HIPCHECK(hipStreamDestroy(streams[d]));
  }
  return ok ? 0 : 1;
}
