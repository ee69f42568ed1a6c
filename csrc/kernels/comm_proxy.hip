// One-GPU stand-in for a gradient bucket's ring all-reduce (parallel/comm_proxy.py).
//
// On one MI355X there is no second rank to talk to, but the question an 8-GPU run asks of the
// collectives -- do they progress beside the step's compute kernels or queue behind them? -- is a
// question about CU slots, not links.  A ring all-reduce over N ranks moves 2 (N - 1) / N x the
// bucket's bytes through each rank, on a fixed number of workgroups ("channels") that hold their
// CUs for the whole collective while they wait on the links.  This kernel does the same on one
// GPU: `channels` workgroups move `total16` 16-byte units (read the bucket, write a scratch copy),
// each paced to rate / channels with the 100 MHz constant clock, so the kernel takes as long as
// the collective would at that bus bandwidth and occupies as many CUs.  rate 0: unpaced (an HBM
// copy on `channels` CUs).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace {

constexpr int kChunk = 4;  // 16-byte units per thread per chunk: 16 KiB per workgroup chunk

__global__ __launch_bounds__(256) void comm_proxy_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, long n16,
                                                         long total16, long ticks_per_chunk) {
  const long per = (total16 + gridDim.x - 1) / gridDim.x;
  const long i0 = (long)blockIdx.x * per;
  const long i1 = i0 + per < total16 ? i0 + per : total16;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long c = i0; c < i1; c += 256 * kChunk) {
    uint4 v[kChunk];
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      long i = c + k * 256 + threadIdx.x;
      if (i >= n16) i -= n16;  // total16 < 2 n16: the second pass re-reads the bucket
      if (c + k * 256 + threadIdx.x < i1) v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      long i = c + k * 256 + threadIdx.x;
      if (i >= n16) i -= n16;
      if (c + k * 256 + threadIdx.x < i1) dst[i] = v[k];
    }
    if (ticks_per_chunk > 0) {  // hold the CU until the link time of the units moved so far is spent
      const long done = (c + 256 * kChunk < i1 ? c + 256 * kChunk : i1) - i0;  // a partial last chunk: its share
      const unsigned long long due = t0 + (((unsigned long long)done * ticks_per_chunk) >> 10);
      while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(4);
    }
  }
}

}  // namespace

namespace mg {

void comm_proxy(const void* src, void* dst, long n16, long total16, int channels, double gbps,
                hipStream_t stream) {
  if (total16 <= 0 || n16 <= 0) return;
  // per-workgroup chunk of 256 x kChunk x 16 bytes at gbps / channels, in 100 MHz ticks
  const long ticks = gbps > 0 ? (long)(256.0 * kChunk * 16 * channels / (gbps * 1e9) * 1e8 + 0.5) : 0;
  comm_proxy_kernel<<<channels, 256, 0, stream>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst),
                                                   n16, total16, ticks);
}

}  // namespace mg
