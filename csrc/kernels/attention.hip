// Decode attention for gfx950 (CDNA4, MI355X): one new query per sequence against the KV cache.
//
// The reference re-runs the full forward over the whole prefix for every generated token
// (/root/reference/mingpt/model.py:322-356); models/generation.py keeps each layer's qkv rows as a
// cache instead and this kernel attends the new token's query to them (training attention:
// attention_train.hip).  Tried and measured slower at GPT-2 decode shapes (B=1, L <= 288): all of
// a key row's chunks requested at once (registers), and a 256-thread fold of the key groups
// (extra barriers) -- 5.3 -> 5.8 us per call.
#include "attn_common.h"
#include "kernels.h"

using namespace mg;
using mg::attn::fexp2;

namespace {

// =============================================================================== decode
// One new query per sequence attending to a KV cache held as qkv rows [B, Tmax, 3D] (the prefill
// writes its qkv GEMM output straight into it).  Split-key ("flash-decoding") form: grid =
// B*H*S, workgroup (b, h, s) takes keys [s*CH, (s+1)*CH) of 0..pos, writes its partial softmax
// state (max, sum, sum p v) and the last of the S workgroups of (b, h) to finish combines them --
// a (b, h) per workgroup left the chip nearly idle (12 workgroups at B = 1) with each key's row a
// serial latency.  The hand-off between workgroups uses agent-scope atomic stores / loads for the
// partials (sc1: no cache of another CU or XCD is involved), each wave draining its stores before
// the workgroup's counter increment (MI355X_MICROARCH 'Correctness boundaries').  The last
// workgroup resets the counter, so the kernel can be replayed inside a hipGraph.
constexpr int kDecSplitsMax = 16;  // combine handles up to this many partials per (b, h)

__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16_t* __restrict__ qkv_new,
                                                          bf16_t* __restrict__ cache,
                                                          bf16_t* __restrict__ out, int H, int hd,
                                                          int D, long Tmax, int pos,
                                                          const int* __restrict__ pos_dev,
                                                          float scale_log2, int S, int CH,  // CH: set below
                                                          int KPS,
                                                          float* __restrict__ part,
                                                          unsigned* __restrict__ counters) {
  if (pos_dev) pos = min(max(*pos_dev, 0), (int)Tmax - 1);  // hipGraph decode: position in device memory
  __shared__ float qs[128];
  __shared__ float sc[256];
  __shared__ float red[16];
  __shared__ float acc[256 * 8];
  __shared__ int last_flag;
  const int bh = blockIdx.x / S, sp = blockIdx.x % S;
  const int b = bh / H, hh = bh % H;
  const long ld = 3L * D;
  const bf16_t* qrow = qkv_new + (long)b * ld + hh * hd;
  bf16_t* cb = cache + (long)b * Tmax * ld;
  if (sp == 0) {  // append this step's K/V at row pos (readers take row pos from qkv_new)
    for (int i = threadIdx.x; i < 2 * hd; i += 256) {
      const int which = i / hd, d = i % hd;
      cb[(long)pos * ld + (long)D * (1 + which) + hh * hd + d] = qrow[(long)D * (1 + which) + d];
    }
  }
  for (int d = threadIdx.x; d < hd; d += 256) qs[d] = bf2f(qrow[d]);
  __syncthreads();
  const int L = pos + 1;
  // splits actually used at this position: KPS (128 or 256) keys each (a short context is one workgroup and
  // skips the hand-off); the grid is sized for Tmax so a captured graph replays at any position
  const int Se = min(S, (L + KPS - 1) / KPS);
  if (sp >= Se) return;  // never counted: the last arrival is the Se-th
  CH = (L + Se - 1) / Se;
  const int k0 = sp * CH, k1 = min(k0 + CH, L);
  const int nk = max(k1 - k0, 0);
  // scores: one key per thread (CH <= 256)
  float s = -INFINITY;
  if (threadIdx.x < nk) {
    const int j = k0 + threadIdx.x;
    const bf16_t* kr = (j == pos) ? qrow + D : cb + (long)j * ld + D + hh * hd;
    float a = 0.f;
    for (int d = 0; d < hd; d += 8) {
      float k8[8];
      unpack8(ld16(kr + d), k8);
#pragma unroll
      for (int e = 0; e < 8; ++e) a += qs[d + e] * k8[e];
    }
    s = a * scale_log2;
  }
  const float mx = block_max<4>(s, red);
  const float p = threadIdx.x < nk ? fexp2(s - mx) : 0.f;
  sc[threadIdx.x] = p;
  const float sm = block_sum<4>(p, red + 4);
  __syncthreads();
  // P V: DCH = hd/8 lanes of 8 dims per key group, 256/DCH key groups, loads issued 4 at a time
  const int dch = hd >> 3;
  const int ngrp = 256 / dch;
  const int grp = threadIdx.x / dch, d8 = (threadIdx.x % dch) * 8;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (grp < ngrp) {
    int jj = grp;
    for (; jj + 3 * ngrp < nk; jj += 4 * ngrp) {
      uint4 vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = k0 + jj + u * ngrp;
        const bf16_t* vr = (j == pos) ? qrow + 2 * D : cb + (long)j * ld + 2 * D + hh * hd;
        vv[u] = ld16(vr + d8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v8[8];
        unpack8(vv[u], v8);
        const float pj = sc[jj + u * ngrp];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += pj * v8[e];
      }
    }
    for (; jj < nk; jj += ngrp) {
      const int j = k0 + jj;
      const bf16_t* vr = (j == pos) ? qrow + 2 * D : cb + (long)j * ld + 2 * D + hh * hd;
      float v8[8];
      unpack8(ld16(vr + d8), v8);
      const float pj = sc[jj];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pj * v8[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[threadIdx.x * 8 + e] = o[e];
  __syncthreads();
  if (Se == 1) {  // the whole context in this workgroup: normalise and write
    if (threadIdx.x < hd) {
      const int c = threadIdx.x / 8, e = threadIdx.x % 8;
      float v = 0.f;
      for (int g = 0; g < ngrp; ++g) v += acc[(g * dch + c) * 8 + e];
      out[(long)b * D + hh * hd + threadIdx.x] = f2bf(v / sm);
    }
    return;
  }
  // partial state of this split: {max, sum, o[hd]} (fp32)
  float* mine = part + (long)blockIdx.x * (hd + 2);
  if (threadIdx.x < hd) {
    const int c = threadIdx.x / 8, e = threadIdx.x % 8;
    float v = 0.f;
    for (int g = 0; g < ngrp; ++g) v += acc[(g * dch + c) * 8 + e];
    __hip_atomic_store(mine + 2 + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(mine, nk ? mx : -INFINITY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, sm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counters + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = prev == (unsigned)(Se - 1);
  }
  __syncthreads();
  if (!last_flag) return;
  // last split of (b, h): combine the S partial states (agent-scope loads: never a stale line),
  // every load issued before any is used
  const float* pb = part + (long)bh * S * (hd + 2);
  if (threadIdx.x < Se) {
    red[threadIdx.x] = __hip_atomic_load(pb + threadIdx.x * (hd + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sc[threadIdx.x] = __hip_atomic_load(pb + threadIdx.x * (hd + 2) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x < hd) {
    float ov[kDecSplitsMax];
#pragma unroll
    for (int t = 0; t < kDecSplitsMax; ++t)
      ov[t] = t < Se ? __hip_atomic_load(pb + t * (hd + 2) + 2 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
    float M = -INFINITY;
    for (int t = 0; t < Se; ++t) M = fmaxf(M, red[t]);
    float Ls = 0.f, Os = 0.f;
#pragma unroll
    for (int t = 0; t < kDecSplitsMax; ++t) {
      if (t < Se && red[t] != -INFINITY) {
        const float w = fexp2(red[t] - M);
        Ls += w * sc[t];
        Os += w * ov[t];
      }
    }
    out[(long)b * D + hh * hd + threadIdx.x] = f2bf(Os / Ls);
  }
  if (threadIdx.x == 0) __hip_atomic_store(counters + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

namespace mg {

size_t attention_decode_part_floats(int B, int H, int hd) {
  return (size_t)B * H * kDecSplitsMax * (hd + 2);
}

// part / counters: the caller's workspace (kernels.h).  They used to be one process-wide buffer
// grown on demand, which a decode hipGraph captured at a smaller size then replayed into freed
// memory once another batch size had re-allocated it.
void attention_decode(const bf16_t* qkv_new, bf16_t* cache, bf16_t* out, int B, int H, int hd,
                      long Tmax, int pos, hipStream_t stream, float* part, unsigned* counters,
                      const int* pos_dev) {
  // fixed grid (graph replays move pos only); the kernel uses ceil(L / 128) of the S splits, so
  // each holds <= 256 keys for Tmax <= 4096 (checked by the binding)
  const int S = kDecSplitsMax;
  const int CH = 0;
  // keys per split: a split hands its partial state to the last arrival (store drain + returning
  // atomic, ~5 us measured when 48 workgroups meet on one counter); with few (b, h) pairs a single
  // workgroup up to 256 keys beats splitting (B = 1 greedy: 3,167 -> 3,289 tok/s), with many the
  // extra parallelism pays (B = 8: 14.3k vs 13.9k)
  const int kps = B * H <= 32 ? 256 : 128;
  attn_decode_kernel<<<B * H * S, 256, 0, stream>>>(qkv_new, cache, out, H, hd, H * hd, Tmax, pos, pos_dev,
                                                    1.4426950408889634f / sqrtf((float)hd), S, CH, kps,
                                                    part, counters);
}

}  // namespace mg
