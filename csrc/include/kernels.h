// Host-side launch API of every gfx950 kernel in csrc/kernels.  Pure HIP: no torch headers,
// raw device pointers + an explicit stream, so the kernels can be driven by the torch binding
// (csrc/bindings.cpp), by native tools, or captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mg {
typedef uint16_t bf16_t;

// layernorm.hip
void layernorm_fwd(const bf16_t* x, const bf16_t* w, const bf16_t* b, bf16_t* y, float* mean,
                   float* rstd, int M, int D, float eps, hipStream_t stream);
// dz (optional): also dz = residual-dropout backward of the stored dx (probability p, the forward's
// seed), its fp32 column sums added into dzb (the bias gradient of the branch that produced x)
void layernorm_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* w, const float* mean,
                   const float* rstd, const bf16_t* dres, bf16_t* dx, float* dw, float* db,
                   float* workspace, int M, int D, hipStream_t stream, bf16_t* dz = nullptr,
                   float* dzb = nullptr, float p = 0.f, uint64_t seed = 0);
size_t layernorm_bwd_workspace(int M, int D, bool drop);

// embedding.hip
void embedding_fwd(const int64_t* idx, const bf16_t* wte, const bf16_t* wpe, bf16_t* out, int M,
                   int T, int D, int V, float p, uint64_t seed, hipStream_t stream,
                   const int* pos_dev = nullptr,  // pos_dev: decode, position read on the device
                   const unsigned long long* am_part = nullptr,  // greedy decode: the token of row m
                   int am_groups = 0,             //   = argmax over the LM-head GEMV's keys
                   int64_t* tok = nullptr,        //   am_part[m][0 .. am_groups), written to tok[m]
                   int64_t* seq = nullptr,        //   and seq[m * seq_ld + *pos_dev]
                   long seq_ld = 0);
unsigned int debug_error_bits();  // MG_DEBUG builds: device range-check bits, cleared on read
void embedding_bwd(const int64_t* idx, const bf16_t* dout, float* dwte, float* dwpe, int M, int T,
                   int D, int V, float p, uint64_t seed, hipStream_t stream);

// xent.hip
void xent_fwd(const bf16_t* logits, const int64_t* targets, float* loss_row, float* lse, float* out,
              int M, int V, int ld, hipStream_t stream);
void xent_bwd(const bf16_t* logits, const int64_t* targets, const float* lse, const float* gscale,
              const float* inv_n, bf16_t* dlogits, int M, int V, int ld, hipStream_t stream);
int xent_fused_nv(int ld);
void xent_fused(const bf16_t* logits, const int64_t* targets, float* loss_row, float* out,
                bf16_t* dlogits, int M, int V, int ld, hipStream_t stream);
void xent_scale(bf16_t* dlogits, const float* gscale, long n, hipStream_t stream);

// adamw.hip (also holds the hipGraph-mode device state; see common.h eff_seed)
void set_graph_state(const uint64_t* seed_ofs, const float* opt_hp);
const uint64_t* graph_seed_ofs();
const float* graph_opt_hp();
size_t grad_norm_workspace();
void grad_sumsq(const float* grad, long n, float grad_scale, float* workspace, float* out,
                hipStream_t stream);
void grad_sumsq_chunks(const int64_t* chunk_start, const int* chunk_len, int n_chunks,
                       const void* grad, bool grad_bf16, float grad_scale, float* workspace,
                       float* out, hipStream_t stream);
void adamw_step(const int64_t* chunk_start, const int* chunk_len, const float* chunk_wd,
                const int64_t* moment_start, int n_chunks, float* master, bf16_t* param,
                const void* grad, bool grad_bf16, float* m, float* v, const float* norm, float lr,
                float b1, float b2, float eps, int step, float grad_scale, float clip,
                hipStream_t stream, float* zero_grad = nullptr);
void f32_to_bf16(const float* src, bf16_t* dst, long n, hipStream_t stream);
// one-GPU stand-in for a ring all-reduce's CU occupancy and duration (comm_proxy.hip)
void comm_proxy(const void* src, void* dst, long n16, long total16, int channels, double gbps,
                hipStream_t stream);

// gemv.hip (decode-time skinny GEMM, B <= 8 rows; epi 0 none, 1 bias, 2 bias+GELU, 3 bias+residual)
bool gemv_supported(int B, int K);
// greedy-decode epilogue of the LM-head GEMV: each workgroup's best (ordered bf16 logit << 32 |
// ~index) key per row into part[b][workgroup]; workgroup 0 advances *pos.  The argmax over the
// workgroups (first index on ties) is taken by the next step's embedding kernel (embedding_fwd
// with am_part) or on the host after the last step.
struct GemvArgmax {
  unsigned long long* part;  // [B][gemv_grid(N, B)]
  int* pos;                  // device position of the step (+1)
};
int gemv_grid(int N, int B);  // workgroups of gemv() for N outputs at B rows (argmax key groups)
void gemv(const bf16_t* x, const bf16_t* W, bf16_t* y, int B, int N, int K, long ldy, const bf16_t* bias,
          const bf16_t* resid, int epi, hipStream_t stream, const bf16_t* lnw = nullptr,
          const bf16_t* lnb = nullptr, float eps = 1e-5f, const GemvArgmax* am = nullptr);

// elementwise.hip
void bias_act_fwd(const bf16_t* x, const bf16_t* b, bf16_t* pre, bf16_t* y, long M, int N, int act,
                  hipStream_t stream);
void bias_dropout_residual(const bf16_t* x, const bf16_t* b, const bf16_t* r, bf16_t* y, long M,
                           int N, float p, uint64_t seed, hipStream_t stream);
void gelu_bwd(const bf16_t* dy, const bf16_t* pre, bf16_t* dx, long n, hipStream_t stream);
void dropout_bwd(const bf16_t* dy, bf16_t* dx, long M, int N, float p, uint64_t seed, hipStream_t stream);
void transpose(const bf16_t* src, bf16_t* dst, int R, int C, int ldd, hipStream_t stream);
void bias_grad(const bf16_t* dy, float* db, long M, int N, hipStream_t stream, long ld = 0);  // row stride ld (0: N)
void dropout_bias_grad(const bf16_t* dy, bf16_t* dx, float* db, long M, int N, float p, uint64_t seed,
                       hipStream_t stream);

// gemm.hip -- layout 0 NT (fwd), 1 NN (dgrad), 2 TN (wgrad, fp32 accumulate)
// epi: 0 none, 1 bias, 2 bias+gelu (gelu'(z) -> aux), 3 resid + dropout(acc + bias), 4 acc*gelu'(aux);
// 6 / 7: 2 / 4 with aux in the fragment order of the W4 256 x 256 tiles (gemm_frag_aux_elems)
void gemm(int layout, int epi, const bf16_t* A, const bf16_t* B, void* C, long lda, long ldb,
          long ldc, int M, int N, int K, int a_ext, int b_ext, int ka, int kb, const bf16_t* bias,
          bf16_t* aux, const bf16_t* resid, float p, uint64_t seed, hipStream_t stream,
          size_t a_bytes, size_t b_bytes,  // operand sizes in bytes (< 4 GiB for the DMA path)
          float* dbias = nullptr);         // EPI 4 only: += column sums of C (bias gradient)
void gemm_set_variant(int v);  // tile config override: 0 auto (per shape), 1 T128, 5 W4, 6 W4-192
void gemm_set_debug_buffer(unsigned long long* p);  // MG_GEMM_STAMPS diagnostic builds
int gemm_get_variant();
int gemm_pick(int M, int N, int K, int layout);  // tile config the dispatcher picks (gemm_set_variant codes)

// attention_train.hip / attention.hip -- causal flash attention; qkv [B*T, 3D], out [B*T, D],
// lse [B*H*T]; dmask: dropout keep-bits generated by attention_fwd when p > 0
// (attention_dropout_mask_words u32), read by attention_bwd
size_t attention_dropout_mask_words(int B, int T, int H);
// 16-bit dropout keep threshold of probability p (keep iff a 16-bit uniform >= thr; 0: no dropout)
// and the matching keep scale 65536 / (65536 - thr)
int attention_dropout_threshold(float p);
float attention_dropout_scale(int thr);
void attention_fwd(const bf16_t* qkv, bf16_t* out, float* lse, uint32_t* dmask, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream);
// delta [B*H*T] and dq [attention_bwd_workspace_floats] fp32 are workspaces; writes all three
// slots of dqkv
size_t attention_bwd_workspace_floats(int B, int T, int H, int hd);
void attention_set_bwd_mode(int mode);
void attention_set_bwd64(int on);
#ifdef MG_BWD64_STAMPS
void attention_bwd64_stamps(unsigned long long* host);  // diagnostic build only
#endif  // 1 (default): hd = 64 key-block backward attn_bwd64_kernel; 0: the general kernel  // 0 auto, 1 persistent (b, h) workgroups, 2 key-block partials
// dbias (fp32 [3D] or null): += the column sums of dqkv (the qkv bias gradient), fused into the
// backward kernels where the schedule allows
void attention_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse,
                   const uint32_t* dmask, float* delta, float* dq, bf16_t* dqkv, int B, int T, int H,
                   int hd, float p, uint64_t seed, hipStream_t stream, float* dbias = nullptr);

// one decode step: appends K/V of qkv_new [B, 3D] at row pos of cache [B, Tmax, 3D]; out [B, D].
// part (attention_decode_part_floats(B, H, hd) floats) and counters (B * H, zero; the kernel leaves
// them zero) are the caller's workspace: one per decode state, so a captured hipGraph never sees
// another state's (possibly freed) buffers.
size_t attention_decode_part_floats(int B, int H, int hd);
void attention_decode(const bf16_t* qkv_new, bf16_t* cache, bf16_t* out, int B, int H, int hd,
                      long Tmax, int pos, hipStream_t stream, float* part, unsigned* counters,
                      const int* pos_dev = nullptr);

}  // namespace mg
