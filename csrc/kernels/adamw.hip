// Fused AdamW + global-norm gradient clipping over flat buffers (gfx950).
//
// Replaces torch.optim.AdamW (/root/reference/mingpt/model.py:117-121) and
// clip_grad_norm (/root/reference/mingpt/trainer.py:129-130).  The framework keeps every
// parameter as a view into ONE flat buffer per dtype (bf16 compute params, fp32 master
// weights, fp32 grads, fp32 exp_avg / exp_avg_sq), so a whole optimizer step is 3 launches:
//   1. grad_sumsq_partial: per-block sum of squares of the (scaled) grads,
//   2. grad_sumsq_final:   one block folds the partials -> {sumsq, norm} on the device,
//   3. adamw_kernel:       multi-tensor-apply style: block b owns chunk b of a host-built chunk
//                          table (chunks never straddle parameters, so weight decay is a
//                          per-chunk constant).  The clip coefficient is computed on device from
//                          step 2's output: no host sync, graph-capturable.
// Numerics match torch.optim.AdamW (decoupled decay p *= 1 - lr*wd, bias corrections, eps
// added after dividing sqrt(v) by sqrt(bc2)).
#include "common.h"
#include "kernels.h"

using namespace mg;

namespace {

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ g, long n,
                                                            float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = g4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = (n4 << 2) + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    s += g[i] * g[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sumsq_final_kernel(const float* __restrict__ part, int G,
                                                          float grad_scale, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < G; i += 256) s += part[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) {
    out[0] = s;
    out[1] = sqrtf(s) * grad_scale;
  }
}

typedef float f32v4 __attribute__((ext_vector_type(4)));
MG_DEVICE void ld4_nt(const float* p, float (&o)[4]) {
  const f32v4 v = __builtin_nontemporal_load(reinterpret_cast<const f32v4*>(p));
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
MG_DEVICE void st4_nt(float* p, const float (&a)[4]) {
  __builtin_nontemporal_store(f32v4{a[0], a[1], a[2], a[3]}, reinterpret_cast<f32v4*>(p));
}

// Gradient loads: fp32 main grads, or the bf16 buffer a bf16 all-reduce / reduce-scatter left.
MG_DEVICE void load_grad4(const float* g, long e, float (&o)[4]) {
  const float4 v = *reinterpret_cast<const float4*>(g + e);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
MG_DEVICE void load_grad4(const bf16_t* g, long e, float (&o)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(g + e);
  o[0] = bf2f(u.x & 0xffffu); o[1] = bf2f(u.x >> 16);
  o[2] = bf2f(u.y & 0xffffu); o[3] = bf2f(u.y >> 16);
}
MG_DEVICE float load_grad1(const float* g, long e) { return g[e]; }
MG_DEVICE float load_grad1(const bf16_t* g, long e) { return bf2f(g[e]); }

// Sum of squares over the chunks of a chunk table (block b -> chunk b): the global grad norm of
// exactly the elements the optimizer updates (a ZeRO shard is a set of pieces, not one range).
template <typename G>
__global__ __launch_bounds__(256) void sumsq_chunks_kernel(const int64_t* __restrict__ chunk_start,
                                                           const int* __restrict__ chunk_len,
                                                           const G* __restrict__ g,
                                                           float* __restrict__ part) {
  __shared__ float red[4];
  const long s0 = chunk_start[blockIdx.x];
  const int len = chunk_len[blockIdx.x];
  float s = 0.f;
  for (int i = threadIdx.x * 4; i < len; i += 256 * 4) {
    if (i + 4 <= len) {
      float v[4];
      load_grad4(g, s0 + i, v);
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    } else {
      for (int j = i; j < len; ++j) {
        const float v = load_grad1(g, s0 + j);
        s += v * v;
      }
    }
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

#ifndef MG_ADAMW_U
#define MG_ADAMW_U 2
#endif
constexpr int kAdamwU = MG_ADAMW_U;  // float4 groups per thread per iteration: 1 / 4 measured no faster (PERF.md)

// chunk b updates master/param/grad[chunk_start[b] ...] and the moments at
// m/v[moment_start[b] ...] (moment_start == nullptr: the same index).  Replicated DP keeps
// moments for the whole flat buffer; ZeRO-1 keeps them only for the rank's pieces, packed.
// zg (optional): the fp32 main-grad buffer, zeroed at each updated element once read (the
// separate zero-fill pass fused in: the same bytes, one launch fewer).
template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(
    const int64_t* __restrict__ chunk_start, const int* __restrict__ chunk_len,
    const float* __restrict__ chunk_wd, const int64_t* __restrict__ moment_start,
    float* __restrict__ master, bf16_t* __restrict__ param, const G* __restrict__ grad,
    float* __restrict__ m, float* __restrict__ v, const float* __restrict__ norm, float lr, float b1,
    float b2, float eps, float bc1, float bc2_sqrt, float grad_scale, float clip,
    const float* __restrict__ hp, int n_chunks, float* __restrict__ zg) {
  if (hp) {  // graph mode: {lr, step} from device memory (the host values were captured once)
    lr = hp[0];
    bc1 = 1.f - powf(b1, hp[1]);
    bc2_sqrt = sqrtf(1.f - powf(b2, hp[1]));
  }
  float gs = grad_scale;
  if (clip > 0.f) {
    const float tn = sqrtf(norm[0]) * grad_scale;
    const float coef = clip / (tn + 1e-6f);
    if (coef < 1.f) gs *= coef;
  }
  const float step = lr / bc1;
  const float z4[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = blockIdx.x; c < n_chunks; c += gridDim.x) {
  const long s0 = chunk_start[c];
  const long ms0 = moment_start ? moment_start[c] : s0;
  const int len = chunk_len[c];
  const float decay = 1.f - lr * chunk_wd[c];
  // every operand is touched once per step: non-temporal loads / stores (no L2 / MALL pollution),
  // and kAdamwU float4 groups per thread per iteration so 4 kAdamwU loads are in flight before any use
  auto upd = [&](float (&pa)[4], const float (&ga)[4], float (&ma)[4], float (&va)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gg = ga[j] * gs;
      ma[j] = b1 * ma[j] + (1.f - b1) * gg;
      va[j] = b2 * va[j] + (1.f - b2) * gg * gg;
      pa[j] = pa[j] * decay - step * ma[j] / (sqrtf(va[j]) / bc2_sqrt + eps);
    }
  };
  int i = threadIdx.x * 4;
  for (; i + (kAdamwU - 1) * 1024 + 4 <= len; i += kAdamwU * 1024) {
    float pa[kAdamwU][4], ga[kAdamwU][4], ma[kAdamwU][4], va[kAdamwU][4];
#pragma unroll
    for (int u = 0; u < kAdamwU; ++u) {
      const long e = s0 + i + u * 1024, me = ms0 + i + u * 1024;
      ld4_nt(master + e, pa[u]);
      load_grad4(grad, e, ga[u]);
      ld4_nt(m + me, ma[u]);
      ld4_nt(v + me, va[u]);
    }
#pragma unroll
    for (int u = 0; u < kAdamwU; ++u) {
      const long e = s0 + i + u * 1024, me = ms0 + i + u * 1024;
      upd(pa[u], ga[u], ma[u], va[u]);
      if (zg) st4_nt(zg + e, z4);  // after the grad's use: its load has returned
      st4_nt(master + e, pa[u]);
      st4_nt(m + me, ma[u]);
      st4_nt(v + me, va[u]);
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(v2u{pack2(pa[u][0], pa[u][1]), pack2(pa[u][2], pa[u][3])},
                                  reinterpret_cast<v2u*>(param + e));
    }
  }
  for (; i < len; i += 1024) {
    const long e = s0 + i, me = ms0 + i;
    if (i + 4 <= len) {
      float pa[4], ga[4], ma[4], va[4];
      ld4_nt(master + e, pa);
      load_grad4(grad, e, ga);
      ld4_nt(m + me, ma);
      ld4_nt(v + me, va);
      upd(pa, ga, ma, va);
      if (zg) st4_nt(zg + e, z4);
      st4_nt(master + e, pa);
      st4_nt(m + me, ma);
      st4_nt(v + me, va);
      *reinterpret_cast<uint2*>(param + e) = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
    } else {
      for (int j = 0; j < 4 && i + j < len; ++j) {
        const long k = e + j, mk = me + j;
        const float gg = load_grad1(grad, k) * gs;
        if (zg) zg[k] = 0.f;
        const float mj = b1 * m[mk] + (1.f - b1) * gg;
        const float vj = b2 * v[mk] + (1.f - b2) * gg * gg;
        const float pj = master[k] * decay - step * mj / (sqrtf(vj) / bc2_sqrt + eps);
        m[mk] = mj;
        v[mk] = vj;
        master[k] = pj;
        param[k] = f2bf(pj);
      }
    }
  }
  }
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ src,
                                                          bf16_t* __restrict__ dst, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dst[i] = f2bf(src[i]);
}

}  // namespace

namespace mg {

static const uint64_t* g_seed_ofs = nullptr;
static const float* g_opt_hp = nullptr;
void set_graph_state(const uint64_t* seed_ofs, const float* opt_hp) {
  g_seed_ofs = seed_ofs;
  g_opt_hp = opt_hp;
}
const uint64_t* graph_seed_ofs() { return g_seed_ofs; }
const float* graph_opt_hp() { return g_opt_hp; }

constexpr int kNormBlocks = 1024;

size_t grad_norm_workspace() { return sizeof(float) * kNormBlocks; }

void grad_sumsq(const float* grad, long n, float grad_scale, float* workspace, float* out,
                hipStream_t stream) {
  sumsq_partial_kernel<<<kNormBlocks, 256, 0, stream>>>(grad, n, workspace);
  sumsq_final_kernel<<<1, 256, 0, stream>>>(workspace, kNormBlocks, grad_scale, out);
}

void grad_sumsq_chunks(const int64_t* chunk_start, const int* chunk_len, int n_chunks,
                       const void* grad, bool grad_bf16, float grad_scale, float* workspace,
                       float* out, hipStream_t stream) {
  if (grad_bf16)
    sumsq_chunks_kernel<bf16_t><<<n_chunks, 256, 0, stream>>>(
        chunk_start, chunk_len, static_cast<const bf16_t*>(grad), workspace);
  else
    sumsq_chunks_kernel<float><<<n_chunks, 256, 0, stream>>>(
        chunk_start, chunk_len, static_cast<const float*>(grad), workspace);
  sumsq_final_kernel<<<1, 256, 0, stream>>>(workspace, n_chunks, grad_scale, out);
}

void adamw_step(const int64_t* chunk_start, const int* chunk_len, const float* chunk_wd,
                const int64_t* moment_start, int n_chunks, float* master, bf16_t* param,
                const void* grad, bool grad_bf16, float* m, float* v, const float* norm, float lr,
                float b1, float b2, float eps, int step, float grad_scale, float clip,
                hipStream_t stream, float* zero_grad) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, (float)step));
  const int grid = n_chunks;  // one workgroup per chunk
  if (grad_bf16)
    adamw_kernel<bf16_t><<<grid, 256, 0, stream>>>(
        chunk_start, chunk_len, chunk_wd, moment_start, master, param,
        static_cast<const bf16_t*>(grad), m, v, norm, lr, b1, b2, eps, bc1, bc2_sqrt, grad_scale,
        clip, g_opt_hp, n_chunks, zero_grad);
  else
    adamw_kernel<float><<<grid, 256, 0, stream>>>(
        chunk_start, chunk_len, chunk_wd, moment_start, master, param,
        static_cast<const float*>(grad), m, v, norm, lr, b1, b2, eps, bc1, bc2_sqrt, grad_scale,
        clip, g_opt_hp, n_chunks, zero_grad);
}

void f32_to_bf16(const float* src, bf16_t* dst, long n, hipStream_t stream) {
  const int grid = (int)std::min<long>(4096, (n + 255) / 256);
  f32_to_bf16_kernel<<<grid, 256, 0, stream>>>(src, dst, n);
}

}  // namespace mg
