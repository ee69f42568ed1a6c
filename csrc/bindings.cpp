// torch <-> gfx950 kernel bindings.  Every op validates shapes/dtypes on the host BEFORE
// launching (a mis-shaped launch can fault the GPU for the whole node), then launches on the
// caller's current HIP stream.  Built into mingpt_distributed_amd/_C.so by build_ext.py.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "comm.h"
#include "kernels.h"

namespace {

using mg::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) \
  CHECK_DEV(t);       \
  TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) \
  CHECK_DEV(t);      \
  TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be fp32")
#define CHECK_I64(t) \
  CHECK_DEV(t);      \
  TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")

inline bf16_t* bp(const at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
inline float* fp(const at::Tensor& t) { return t.data_ptr<float>(); }
inline float* fp_opt(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
inline bf16_t* bp_opt(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<bf16_t*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------------------- layernorm
std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                      double eps) {
  CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(b); CHECK_CONTIG(x);
  const int64_t D = x.size(-1), M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "layernorm: D must be a multiple of 8 and <= 4096");
  TORCH_CHECK(w.numel() == D && b.numel() == D, "layernorm: weight/bias size mismatch");
  DevGuard g(x.device());
  auto y = at::empty_like(x);
  auto mean = at::empty({M}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  mg::layernorm_fwd(bp(x), bp(w), bp(b), bp(y), fp(mean), fp(rstd), (int)M, (int)D, (float)eps,
                    cur_stream());
  return {y, mean, rstd};
}

// drop_p > 0 with dz_bias (fp32 [D]): returns (dx, dz), dz = the residual-dropout backward of dx
// (seed: the forward's) and dz's column sums added into dz_bias (layernorm.hip, fused)
std::vector<at::Tensor> layernorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                      const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& dw,
                                      const at::Tensor& db, const c10::optional<at::Tensor>& dres,
                                      const c10::optional<at::Tensor>& dz_bias, double drop_p, int64_t drop_seed) {
  CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(w); CHECK_F32(mean); CHECK_F32(rstd);
  CHECK_F32(dw); CHECK_F32(db); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  const int64_t D = x.size(-1), M = x.numel() / D;
  TORCH_CHECK(dy.numel() == x.numel() && dw.numel() == D && db.numel() == D && mean.numel() == M,
              "layernorm_bwd: shape mismatch");
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "layernorm_bwd: D must be a multiple of 8, at most 4096");
  DevGuard g(x.device());
  auto dx = at::empty_like(x);
  if (dres.has_value() && dres->defined()) {
    CHECK_BF16(*dres); CHECK_CONTIG(*dres);
    TORCH_CHECK(dres->numel() == x.numel(), "layernorm_bwd: dres shape");
  }
  const bool drop = dz_bias.has_value() && dz_bias->defined();
  at::Tensor dz;
  if (drop) {
    CHECK_F32(*dz_bias); CHECK_CONTIG(*dz_bias);
    TORCH_CHECK(dz_bias->numel() == D && D % 8 == 0, "layernorm_bwd: dz_bias must be fp32 [D]");
    dz = at::empty_like(x);
  }
  auto ws = at::empty({(int64_t)mg::layernorm_bwd_workspace((int)M, (int)D, drop)}, mean.options());
  mg::layernorm_bwd(bp(dy), bp(x), bp(w), fp(mean), fp(rstd), bp_opt(dres), bp(dx), fp(dw), fp(db), fp(ws),
                    (int)M, (int)D, cur_stream(), drop ? bp(dz) : nullptr, drop ? fp(*dz_bias) : nullptr,
                    (float)drop_p, (uint64_t)drop_seed);
  if (drop) return {dx, dz};
  return {dx};
}

at::Tensor layernorm_bwd_plain(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                               const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& dw,
                               const at::Tensor& db, const c10::optional<at::Tensor>& dres) {
  return layernorm_bwd(dy, x, w, mean, rstd, dw, db, dres, c10::nullopt, 0.0, 0)[0];
}

// ------------------------------------------------------------------------------- embedding
// pos_dev (int32 [1], optional; decode with T == 1): the position row of wpe is read on the device.
// am_part (int64 [B, G], optional, with pos_dev): greedy decode -- the token of row b is the argmax
// of the previous step's LM-head keys am_part[b] (gemv with am_part), written to tok[b] (idx may
// be that same buffer) and to seq[b, pos] when given.
at::Tensor embedding_fwd(const at::Tensor& idx, const at::Tensor& wte, const at::Tensor& wpe,
                         double p, int64_t seed, const c10::optional<at::Tensor>& pos_dev,
                         const c10::optional<at::Tensor>& am_part, const c10::optional<at::Tensor>& seq) {
  CHECK_I64(idx); CHECK_BF16(wte); CHECK_BF16(wpe); CHECK_CONTIG(idx);
  CHECK_CONTIG(wte); CHECK_CONTIG(wpe);
  TORCH_CHECK(idx.dim() == 2, "idx must be [B, T]");
  const int64_t B = idx.size(0), T = idx.size(1), D = wte.size(1);
  TORCH_CHECK(D % 8 == 0 && wpe.size(1) == D && T <= wpe.size(0), "embedding: shape mismatch");
  const int* pd = nullptr;
  if (pos_dev.has_value()) {
    TORCH_CHECK(T == 1 && pos_dev->scalar_type() == at::kInt && pos_dev->is_cuda(),
                "embedding_fwd: pos_dev (int32 cuda) is for one-token decode steps");
    pd = pos_dev->data_ptr<int>();
  }
  const unsigned long long* ap = nullptr;
  int groups = 0;
  int64_t* seqp = nullptr;
  long seq_ld = 0;
  if (am_part.has_value()) {
    TORCH_CHECK(pd && am_part->scalar_type() == at::kLong && am_part->is_contiguous() && am_part->dim() == 2 &&
                am_part->size(0) == B, "embedding_fwd: am_part int64 [B, G] with pos_dev");
    ap = reinterpret_cast<const unsigned long long*>(am_part->data_ptr<int64_t>());
    groups = (int)am_part->size(1);
    if (seq.has_value()) {
      TORCH_CHECK(seq->scalar_type() == at::kLong && seq->is_contiguous() && seq->dim() == 2 && seq->size(0) == B,
                  "embedding_fwd: seq int64 [B, L]");
      seqp = seq->data_ptr<int64_t>();
      seq_ld = seq->size(1);
    }
  }
  DevGuard g(idx.device());
  auto out = at::empty({B, T, D}, wte.options());
  mg::embedding_fwd(idx.data_ptr<int64_t>(), bp(wte), bp(wpe), bp(out), (int)(B * T), (int)T,
                    (int)D, (int)wte.size(0), (float)p, (uint64_t)seed, cur_stream(), pd, ap, groups,
                    ap ? idx.data_ptr<int64_t>() : nullptr, seqp, seq_ld);
  return out;
}

void embedding_bwd(const at::Tensor& idx, const at::Tensor& dout,
                   const c10::optional<at::Tensor>& dwte, const c10::optional<at::Tensor>& dwpe,
                   double p, int64_t seed) {
  CHECK_I64(idx); CHECK_BF16(dout); CHECK_CONTIG(dout); CHECK_CONTIG(idx);
  const int64_t B = idx.size(0), T = idx.size(1), D = dout.size(-1);
  TORCH_CHECK(dout.numel() == B * T * D, "embedding_bwd: shape mismatch");
  if (dwte.has_value()) { CHECK_F32(*dwte); TORCH_CHECK(dwte->size(-1) == D); }
  if (dwpe.has_value()) { CHECK_F32(*dwpe); TORCH_CHECK(dwpe->size(-1) == D && dwpe->size(0) >= T); }
  DevGuard g(idx.device());
  mg::embedding_bwd(idx.data_ptr<int64_t>(), bp(dout), fp_opt(dwte), fp_opt(dwpe), (int)(B * T),
                    (int)T, (int)D, dwte.has_value() ? (int)(dwte->numel() / D) : 0, (float)p, (uint64_t)seed, cur_stream());
}

// ------------------------------------------------------------------------------- cross entropy
// logits [M, ld] with V valid columns; returns (out[2] = {loss, 1/n_valid}, lse[M])
std::vector<at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& targets, int64_t V) {
  CHECK_BF16(logits); CHECK_I64(targets); CHECK_CONTIG(logits); CHECK_CONTIG(targets);
  const int64_t ld = logits.size(-1), M = logits.numel() / ld;
  TORCH_CHECK(targets.numel() == M && V <= ld && ld % 8 == 0, "xent: shape mismatch");
  DevGuard g(logits.device());
  auto opts = logits.options().dtype(at::kFloat);
  auto loss_row = at::empty({M}, opts);
  auto lse = at::empty({M}, opts);
  auto out = at::empty({2}, opts);
  mg::xent_fwd(bp(logits), targets.data_ptr<int64_t>(), fp(loss_row), fp(lse), fp(out), (int)M,
               (int)V, (int)ld, cur_stream());
  return {out, lse};
}

at::Tensor xent_bwd(const at::Tensor& logits, const at::Tensor& targets, const at::Tensor& lse,
                    const at::Tensor& gscale, const at::Tensor& out, int64_t V) {
  CHECK_BF16(logits); CHECK_I64(targets); CHECK_F32(lse); CHECK_F32(gscale); CHECK_F32(out);
  const int64_t ld = logits.size(-1), M = logits.numel() / ld;
  TORCH_CHECK(targets.numel() == M && lse.numel() == M, "xent_bwd: shape mismatch");
  DevGuard g(logits.device());
  auto dl = at::empty_like(logits);
  mg::xent_bwd(bp(logits), targets.data_ptr<int64_t>(), fp(lse), fp(gscale), fp(out) + 1, bp(dl),
               (int)M, (int)V, (int)ld, cur_stream());
  return dl;
}

// one-pass training cross-entropy: returns (out[2] = {loss, 1/n_valid}, dlogits = (softmax -
// onehot) / n_valid); empty list when the row width is outside the fused kernel's range
std::vector<at::Tensor> xent_fused(const at::Tensor& logits, const at::Tensor& targets, int64_t V) {
  CHECK_BF16(logits); CHECK_I64(targets); CHECK_CONTIG(logits); CHECK_CONTIG(targets);
  const int64_t ld = logits.size(-1), M = logits.numel() / ld;
  TORCH_CHECK(targets.numel() == M && V <= ld && ld % 8 == 0, "xent_fused: shape mismatch");
  if (mg::xent_fused_nv((int)ld) == 0) return {};
  DevGuard g(logits.device());
  auto opts = logits.options().dtype(at::kFloat);
  auto loss_row = at::empty({M}, opts);
  auto out = at::empty({2}, opts);
  auto dl = at::empty_like(logits);
  mg::xent_fused(bp(logits), targets.data_ptr<int64_t>(), fp(loss_row), fp(out), bp(dl), (int)M,
                 (int)V, (int)ld, cur_stream());
  return {out, dl};
}

void xent_scale_(const at::Tensor& dlogits, const at::Tensor& gscale) {
  CHECK_BF16(dlogits); CHECK_CONTIG(dlogits); CHECK_F32(gscale);
  TORCH_CHECK(dlogits.numel() % 8 == 0, "xent_scale_: numel must be a multiple of 8");
  DevGuard g(dlogits.device());
  mg::xent_scale(bp(dlogits), fp(gscale), dlogits.numel(), cur_stream());
}

// ------------------------------------------------------------------------------- hipGraph mode
// While set, launches read dropout-seed offsets from seed_ofs[0] (uint64, bumped inside the graph
// each replay) and AdamW reads {lr, step} from opt_hp (fp32[2], written before each replay).
void set_graph_state(const c10::optional<at::Tensor>& seed_ofs, const c10::optional<at::Tensor>& opt_hp) {
  if (seed_ofs.has_value()) {
    TORCH_CHECK(seed_ofs->scalar_type() == at::kLong && seed_ofs->is_cuda() && seed_ofs->numel() >= 1);
  }
  if (opt_hp.has_value()) { CHECK_F32(*opt_hp); TORCH_CHECK(opt_hp->numel() >= 2); }
  mg::set_graph_state(seed_ofs.has_value() ? reinterpret_cast<const uint64_t*>(seed_ofs->data_ptr<int64_t>()) : nullptr,
                      opt_hp.has_value() ? fp(*opt_hp) : nullptr);
}

// ------------------------------------------------------------------------------- optimizer
void grad_sumsq(const at::Tensor& grad, double grad_scale, const at::Tensor& out) {
  CHECK_F32(grad); CHECK_F32(out); CHECK_CONTIG(grad);
  TORCH_CHECK(out.numel() >= 2);
  DevGuard g(grad.device());
  auto ws = at::empty({(int64_t)(mg::grad_norm_workspace() / 4)}, grad.options());
  mg::grad_sumsq(fp(grad), grad.numel(), (float)grad_scale, fp(ws), fp(out), cur_stream());
}

// The chunk tables are built and range-checked on the host by optim.make_chunk_table, which
// also returns the bounds it checked against (table_end: one past the last flat element any
// chunk touches; moment_end: the same for the packed moments).  The kernels index through the
// tables unchecked, so every buffer handed in here must cover those bounds: a table built for
// another store (e.g. before a re-layout) fails here instead of reading or writing out of bounds.
void grad_sumsq_chunks(const at::Tensor& chunk_start, const at::Tensor& chunk_len,
                       const at::Tensor& grad, double grad_scale, const at::Tensor& out,
                       int64_t table_end) {
  CHECK_I64(chunk_start); CHECK_DEV(chunk_len); CHECK_CONTIG(grad); CHECK_F32(out);
  TORCH_CHECK(chunk_len.scalar_type() == at::kInt, "chunk_len must be int32");
  TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16,
              "grad must be fp32 or bf16");
  TORCH_CHECK(chunk_start.numel() == chunk_len.numel() && out.numel() >= 2);
  TORCH_CHECK(table_end >= 0 && grad.numel() >= table_end, "grad_sumsq_chunks: chunk table reaches element ",
              table_end, " of a ", grad.numel(), "-element gradient buffer");
  const int64_t nc = chunk_len.numel();
  if (nc == 0) { out.zero_(); return; }
  DevGuard g(grad.device());
  auto ws = at::empty({nc}, out.options());
  mg::grad_sumsq_chunks(chunk_start.data_ptr<int64_t>(), chunk_len.data_ptr<int>(), (int)nc,
                        grad.data_ptr(), grad.scalar_type() == at::kBFloat16, (float)grad_scale,
                        fp(ws), fp(out), cur_stream());
}

void adamw_step(const at::Tensor& chunk_start, const at::Tensor& chunk_len,
                const at::Tensor& chunk_wd, const c10::optional<at::Tensor>& moment_start,
                const at::Tensor& master, const at::Tensor& param, const at::Tensor& grad,
                const at::Tensor& m, const at::Tensor& v, const at::Tensor& norm, double lr,
                double b1, double b2, double eps, int64_t step, double grad_scale, double clip,
                int64_t table_end, int64_t moment_end, const c10::optional<at::Tensor>& zero_grad) {
  CHECK_I64(chunk_start); CHECK_DEV(chunk_len); CHECK_F32(chunk_wd);
  TORCH_CHECK(chunk_len.scalar_type() == at::kInt, "chunk_len must be int32");
  CHECK_F32(master); CHECK_BF16(param); CHECK_F32(m); CHECK_F32(v); CHECK_F32(norm);
  CHECK_DEV(grad);
  TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16,
              "grad must be fp32 or bf16");
  const int64_t n = master.numel();
  TORCH_CHECK(param.numel() == n && grad.numel() == n, "adamw: flat buffer size mismatch");
  TORCH_CHECK(table_end >= 0 && n >= table_end, "adamw: chunk table reaches element ", table_end,
              " of ", n, "-element flat buffers");
  TORCH_CHECK(moment_end >= 0 && m.numel() >= moment_end && v.numel() >= moment_end,
              "adamw: chunk table reaches moment ", moment_end, " of ", m.numel());
  const int64_t* ms = nullptr;
  if (moment_start.has_value() && moment_start->defined()) {
    CHECK_I64(*moment_start);
    TORCH_CHECK(moment_start->numel() == chunk_start.numel(), "adamw: moment table length");
    TORCH_CHECK(m.numel() == v.numel(), "adamw: moment buffer size mismatch");
    ms = moment_start->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(m.numel() == n && v.numel() == n, "adamw: moment buffer size mismatch");
  }
  TORCH_CHECK(chunk_start.numel() == chunk_len.numel() && chunk_wd.numel() == chunk_len.numel());
  float* zg = nullptr;  // fp32 main grads zeroed as they are consumed (same flat indexing)
  if (zero_grad.has_value() && zero_grad->defined()) {
    CHECK_F32(*zero_grad);
    TORCH_CHECK(zero_grad->numel() >= table_end, "adamw: zero_grad buffer shorter than the chunk table");
    zg = fp(*zero_grad);
  }
  if (chunk_len.numel() == 0) return;
  DevGuard g(master.device());
  mg::adamw_step(chunk_start.data_ptr<int64_t>(), chunk_len.data_ptr<int>(), fp(chunk_wd), ms,
                 (int)chunk_len.numel(), fp(master), bp(param), grad.data_ptr(),
                 grad.scalar_type() == at::kBFloat16, fp(m), fp(v), fp(norm), (float)lr, (float)b1,
                 (float)b2, (float)eps, (int)step, (float)grad_scale, (float)clip, cur_stream(),
                 zg);
}

void f32_to_bf16(const at::Tensor& src, const at::Tensor& dst) {
  CHECK_F32(src); CHECK_BF16(dst);
  TORCH_CHECK(src.numel() == dst.numel() && src.is_contiguous() && dst.is_contiguous());
  DevGuard g(src.device());
  mg::f32_to_bf16(fp(src), bp(dst), src.numel(), cur_stream());
}

void comm_proxy(const at::Tensor& src, const at::Tensor& scratch, double factor, int64_t channels,
                double gbps) {
  TORCH_CHECK(src.is_cuda() && scratch.is_cuda() && src.is_contiguous() && scratch.is_contiguous());
  const int64_t bytes = src.numel() * src.element_size();
  TORCH_CHECK(scratch.numel() * scratch.element_size() >= bytes, "comm_proxy: scratch too small");
  TORCH_CHECK(factor >= 0 && factor < 2 && channels > 0 && channels <= 1024 && gbps >= 0);
  // a timing model: the bucket's 16-byte-aligned interior is moved, < 32 edge bytes are not
  const uintptr_t p0 = reinterpret_cast<uintptr_t>(src.data_ptr()), pa = (p0 + 15) & ~uintptr_t(15);
  const long n16 = bytes >= (int64_t)(pa - p0) ? (long)((bytes - (int64_t)(pa - p0)) / 16) : 0;
  DevGuard g(src.device());
  mg::comm_proxy(reinterpret_cast<const void*>(pa), scratch.data_ptr(), n16, (long)(factor * n16),
                 (int)channels, gbps, cur_stream());
}

// ------------------------------------------------------------------------------- elementwise
at::Tensor bias_act(const at::Tensor& x, const c10::optional<at::Tensor>& b,
                    const c10::optional<at::Tensor>& pre, int64_t act) {
  CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(N % 8 == 0, "bias_act: N % 8 != 0");
  if (b.has_value()) { CHECK_BF16(*b); TORCH_CHECK(b->numel() == N); }
  if (pre.has_value()) { CHECK_BF16(*pre); TORCH_CHECK(pre->numel() == x.numel()); }
  DevGuard g(x.device());
  auto y = at::empty_like(x);
  mg::bias_act_fwd(bp(x), bp_opt(b), bp_opt(pre), bp(y), M, (int)N, (int)act, cur_stream());
  return y;
}

at::Tensor bias_dropout_residual(const at::Tensor& x, const c10::optional<at::Tensor>& b,
                                 const at::Tensor& r, double p, int64_t seed) {
  CHECK_BF16(x); CHECK_BF16(r); CHECK_CONTIG(x); CHECK_CONTIG(r);
  const int64_t N = x.size(-1), M = x.numel() / N;
  TORCH_CHECK(N % 8 == 0 && r.numel() == x.numel(), "bias_dropout_residual: shape mismatch");
  if (b.has_value()) { CHECK_BF16(*b); TORCH_CHECK(b->numel() == N); }
  DevGuard g(x.device());
  auto y = at::empty_like(x);
  mg::bias_dropout_residual(bp(x), bp_opt(b), bp(r), bp(y), M, (int)N, (float)p, (uint64_t)seed,
                            cur_stream());
  return y;
}

at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& pre) {
  CHECK_BF16(dy); CHECK_BF16(pre); CHECK_CONTIG(dy); CHECK_CONTIG(pre);
  TORCH_CHECK(dy.numel() == pre.numel() && dy.numel() % 8 == 0);
  DevGuard g(dy.device());
  auto dx = at::empty_like(dy);
  mg::gelu_bwd(bp(dy), bp(pre), bp(dx), dy.numel(), cur_stream());
  return dx;
}

// dst[C, ldd] = src[R, C]^T with columns R..ldd-1 zero (ldd = 0 -> R)
at::Tensor transpose(const at::Tensor& src, int64_t ldd) {
  CHECK_BF16(src); CHECK_CONTIG(src);
  TORCH_CHECK(src.dim() == 2, "transpose: 2-D input");
  const int64_t R = src.size(0), C = src.size(1);
  if (ldd <= 0) ldd = R;
  TORCH_CHECK(ldd >= R, "transpose: ldd < rows");
  DevGuard g(src.device());
  auto dst = at::empty({C, ldd}, src.options());
  mg::transpose(bp(src), bp(dst), (int)R, (int)C, (int)ldd, cur_stream());
  return dst;
}

// residual-stream dropout backward: the mask is keyed on (row, column) of the [.., N] tensor
at::Tensor dropout_bwd(const at::Tensor& dy, double p, int64_t seed) {
  CHECK_BF16(dy); CHECK_CONTIG(dy);
  const int64_t N = dy.size(-1), M = dy.numel() / N;
  TORCH_CHECK(N % 8 == 0, "dropout_bwd: last dim must be a multiple of 8");
  DevGuard g(dy.device());
  auto dx = at::empty_like(dy);
  mg::dropout_bwd(bp(dy), bp(dx), M, (int)N, (float)p, (uint64_t)seed, cur_stream());
  return dx;
}

// dx = dropout_bwd(dy) and db += colsum(dx) in one pass
at::Tensor dropout_bias_grad(const at::Tensor& dy, const at::Tensor& db, double p, int64_t seed) {
  CHECK_BF16(dy); CHECK_F32(db); CHECK_CONTIG(dy);
  const int64_t N = dy.size(-1), M = dy.numel() / N;
  TORCH_CHECK(N % 8 == 0 && db.numel() == N, "dropout_bias_grad: shape mismatch");
  DevGuard g(dy.device());
  auto dx = at::empty_like(dy);
  mg::dropout_bias_grad(bp(dy), bp(dx), fp(db), M, (int)N, (float)p, (uint64_t)seed, cur_stream());
  return dx;
}

void bias_grad(const at::Tensor& dy, const at::Tensor& db) {
  CHECK_BF16(dy); CHECK_F32(db); CHECK_CONTIG(dy);
  const int64_t N = dy.size(-1), M = dy.numel() / N;
  TORCH_CHECK(N % 8 == 0 && db.numel() == N, "bias_grad: shape mismatch");
  DevGuard g(dy.device());
  mg::bias_grad(bp(dy), fp(db), M, (int)N, cur_stream());
}

// ------------------------------------------------------------------------------- gemm
// layout 0 (NT): c[M, ldc] = a[M, K] @ b[N, K]^T           (+ epilogue)
// layout 1 (NN): c[M, N]   = a[M, K] @ b[Kb, N]            (b rows >= Kb read as zero)
// layout 2 (TN): c[M, N]  += a[K, Ma]^T @ b[K, N]   fp32 c (M <= Ma store rows)
void gemm(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, int64_t layout, int64_t epi,
          const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux,
          const c10::optional<at::Tensor>& resid, double p, int64_t seed, int64_t M, int64_t N,
          const c10::optional<at::Tensor>& dbias) {
  CHECK_BF16(a); CHECK_BF16(b); CHECK_DEV(c);
  CHECK_CONTIG(a); CHECK_CONTIG(b); CHECK_CONTIG(c);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm: 2-D operands required");
  TORCH_CHECK(layout >= 0 && layout <= 2 && epi >= 0 && epi <= 7 && epi != 5, "gemm: bad layout/epilogue");
  TORCH_CHECK((epi != 6 || layout == 0) && (epi != 7 || layout == 1), "gemm: fragment-ordered GELU' epilogues: 6 NT, 7 NN");
  const int64_t lda = a.size(1), ldb = b.size(1), ldc = c.size(1);
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0, "gemm: row strides must be multiples of 8");
  TORCH_CHECK(M > 0 && N > 0 && M <= c.size(0) && N <= ldc, "gemm: output bounds");
  int64_t K, a_ext, b_ext, ka, kb;
  if (layout == 0) {
    K = lda; ka = lda; kb = ldb; a_ext = a.size(0); b_ext = b.size(0);
    TORCH_CHECK(lda == ldb, "gemm NT: K mismatch");
    TORCH_CHECK(M <= a_ext && N <= (epi == 0 ? ldc : b_ext), "gemm NT: shape mismatch");
    TORCH_CHECK(c.scalar_type() == at::kBFloat16, "gemm NT: bf16 output");
  } else if (layout == 1) {
    K = lda; ka = lda; kb = b.size(0); a_ext = a.size(0); b_ext = ldb;
    TORCH_CHECK(kb <= K && M <= a_ext && N <= ldb && (epi == 0 || epi == 4 || epi == 7), "gemm NN: shape mismatch");
    TORCH_CHECK(c.scalar_type() == at::kBFloat16, "gemm NN: bf16 output");
  } else {
    K = a.size(0); ka = K; kb = b.size(0); a_ext = lda; b_ext = ldb;
    TORCH_CHECK(kb == K && M <= lda && N <= ldb && epi == 0, "gemm TN: shape mismatch");
    TORCH_CHECK(c.scalar_type() == at::kFloat, "gemm TN: fp32 accumulate output");
  }
  TORCH_CHECK(K % 8 == 0, "gemm: K must be a multiple of 8");
  const bf16_t* bias_p = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() >= N, "gemm: bias too short");
    bias_p = bp(*bias);
  }
  bf16_t* aux_p = nullptr;
  if (epi == 2 || epi == 4 || epi == 6 || epi == 7) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "gemm: epilogue needs aux");
    CHECK_BF16(*aux); CHECK_CONTIG(*aux);
    if (epi >= 6) {  // fragment order: whole 256 x 256 tiles
      TORCH_CHECK(aux->numel() == ((M + 255) / 256) * ((N + 255) / 256) * 65536 && ldc == N,
                  "gemm: fragment-ordered aux must hold ceil(M/256) * ceil(N/256) * 65536 elements");
    } else {
      TORCH_CHECK(aux->numel() == c.numel(), "gemm: aux shape");
    }
    aux_p = bp(*aux);
  }
  const bf16_t* res_p = nullptr;
  if (epi == 3) {
    TORCH_CHECK(resid.has_value() && resid->defined(), "gemm: epilogue needs resid");
    CHECK_BF16(*resid); CHECK_CONTIG(*resid);
    TORCH_CHECK(resid->numel() == c.numel() && ldc == N, "gemm: resid shape");
    res_p = bp(*resid);
  }
  // operands past 4 GiB are fine: every block's buffer descriptor starts at its own tile / split
  // origin (gemm.hip Stager::retarget; split-K ranges are capped below 4 GiB by set_split)
  float* dbias_p = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    CHECK_F32(*dbias);
    TORCH_CHECK((epi == 4 || epi == 7) && dbias->numel() >= N, "gemm: dbias only with the gelu_bwd epilogue");
    dbias_p = fp(*dbias);
  }
  DevGuard g(a.device());
  mg::gemm((int)layout, (int)epi, bp(a), bp(b), c.data_ptr(), lda, ldb, ldc, (int)M, (int)N, (int)K,
           (int)a_ext, (int)b_ext, (int)ka, (int)kb, bias_p, aux_p, res_p, (float)p, (uint64_t)seed,
           cur_stream(), (size_t)a.numel() * 2, (size_t)b.numel() * 2, dbias_p);
}

// ------------------------------------------------------------------------------- attention
std::vector<at::Tensor> attention_fwd(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H,
                                      double p, int64_t seed) {
  CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  const int64_t D3 = qkv.size(-1), D = D3 / 3, hd = D / H;
  TORCH_CHECK(D3 == 3 * D && D == H * hd && qkv.numel() == B * T * D3, "attention: qkv shape");
  TORCH_CHECK(hd % 8 == 0 && hd <= 128, "attention: head dim must be a multiple of 8 and <= 128");
  DevGuard g(qkv.device());
  auto out = at::empty({B * T, D}, qkv.options());
  auto lse = at::empty({B * H * T}, qkv.options().dtype(at::kFloat));
  at::Tensor mask = p > 0 ? at::empty({(int64_t)mg::attention_dropout_mask_words((int)B, (int)T, (int)H)},
                                      qkv.options().dtype(at::kInt))
                          : at::empty({0}, qkv.options().dtype(at::kInt));
  mg::attention_fwd(bp(qkv), bp(out), fp(lse),
                    p > 0 ? reinterpret_cast<uint32_t*>(mask.data_ptr<int>()) : nullptr, (int)B, (int)T,
                    (int)H, (int)hd, (float)p, (uint64_t)seed, cur_stream());
  return {out, lse, mask};
}

at::Tensor attention_bwd(const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& dout,
                         const at::Tensor& lse, const at::Tensor& mask, int64_t B, int64_t T,
                         int64_t H, double p, int64_t seed, const c10::optional<at::Tensor>& dbias) {
  CHECK_BF16(qkv); CHECK_BF16(out); CHECK_BF16(dout); CHECK_F32(lse);
  CHECK_CONTIG(qkv); CHECK_CONTIG(out); CHECK_CONTIG(dout);
  const int64_t D3 = qkv.size(-1), D = D3 / 3, hd = D / H;
  TORCH_CHECK(qkv.numel() == B * T * D3 && out.numel() == B * T * D && dout.numel() == B * T * D &&
              lse.numel() == B * H * T && hd % 8 == 0 && hd <= 128 && D <= 4096, "attention_bwd: shape mismatch");
  TORCH_CHECK(B * T * H * 16 < (int64_t)1 << 31, "attention_bwd: B*T*H too large");
  DevGuard g(qkv.device());
  auto dqkv = at::empty_like(qkv);
  auto opts = qkv.options().dtype(at::kFloat);
  auto delta = at::empty({B * H * T}, opts);  // rowsum(dO * O) per (b, h, t), attn_bwd_pre_kernel
  // fp32 dQ accumulator (persistent mode) or per-key-block partials (attention_train.hip)
  auto dq = at::empty({(int64_t)mg::attention_bwd_workspace_floats((int)B, (int)T, (int)H, (int)hd)}, opts);
  const uint32_t* mp = nullptr;
  if (p > 0) {
    CHECK_DEV(mask);
    TORCH_CHECK(mask.scalar_type() == at::kInt &&
                    mask.numel() == (int64_t)mg::attention_dropout_mask_words((int)B, (int)T, (int)H),
                "attention_bwd: dropout mask from attention_fwd required when p > 0");
    mp = reinterpret_cast<const uint32_t*>(mask.data_ptr<int>());
  }
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    CHECK_F32(*dbias); CHECK_CONTIG(*dbias);
    TORCH_CHECK(dbias->numel() == D3, "attention_bwd: dbias must be fp32 [3D]");
    db = fp(*dbias);
  }
  mg::attention_bwd(bp(qkv), bp(out), bp(dout), fp(lse), mp, fp(delta), fp(dq), bp(dqkv), (int)B,
                    (int)T, (int)H, (int)hd, (float)p, (uint64_t)seed, cur_stream(), db);
  return dqkv;
}

// y[B, ldy] (ldy >= N) = epi(x[B, K] @ W[N, K]^T): the decode-time projection (gemv.hip)
at::Tensor gemv(const at::Tensor& x, const at::Tensor& W, int64_t epi, const c10::optional<at::Tensor>& bias,
                const c10::optional<at::Tensor>& resid, int64_t ldy, const c10::optional<at::Tensor>& lnw,
                const c10::optional<at::Tensor>& lnb, double eps, const c10::optional<at::Tensor>& am_part,
                const c10::optional<at::Tensor>& am_pos) {
  CHECK_BF16(x); CHECK_BF16(W); CHECK_CONTIG(x); CHECK_CONTIG(W);
  const int64_t K = W.size(1), N = W.size(0), B = x.numel() / K;
  TORCH_CHECK(x.size(-1) == K && mg::gemv_supported((int)B, (int)K), "gemv: B <= 8, K % 8 == 0, K <= 4096");
  if (ldy <= 0) ldy = N;
  TORCH_CHECK(ldy >= N && epi >= 0 && epi <= 3, "gemv: ldy / epi");
  if (bias.has_value()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N); }
  if (epi == 3) {
    TORCH_CHECK(resid.has_value(), "gemv: residual epilogue needs resid");
    CHECK_BF16(*resid); CHECK_CONTIG(*resid);
    TORCH_CHECK(resid->numel() == B * ldy, "gemv: resid shape");
  }
  TORCH_CHECK(lnw.has_value() == lnb.has_value(), "gemv: LayerNorm needs weight and bias");
  if (lnw.has_value()) {
    CHECK_BF16(*lnw); CHECK_BF16(*lnb);
    TORCH_CHECK(lnw->numel() == K && lnb->numel() == K, "gemv: LayerNorm size");
  }
  DevGuard g(x.device());
  mg::GemvArgmax am{};
  if (am_part.has_value()) {
    // greedy decode: the LM-head GEMV (N > 8192 rows) also leaves one argmax key per (row,
    // workgroup) in am_part [B, gemv_grid(N, B)] (int64 storage of the unsigned keys) and advances
    // *am_pos; the next step's embedding_fwd(am_part=...) reduces the keys into the token
    TORCH_CHECK(N > 8192 && epi == 0, "gemv argmax: LM-head shape (N > 8192, no epilogue)");
    TORCH_CHECK(am_part->scalar_type() == at::kLong && am_part->is_cuda() && am_part->is_contiguous() &&
                am_part->numel() == B * mg::gemv_grid((int)N, (int)B), "gemv argmax: am_part int64 [B, gemv_argmax_groups(N, B)]");
    TORCH_CHECK(am_pos.has_value() && am_pos->scalar_type() == at::kInt && am_pos->is_cuda(),
                "gemv argmax: am_pos int32 [1]");
    am.part = reinterpret_cast<unsigned long long*>(am_part->data_ptr<int64_t>());
    am.pos = am_pos->data_ptr<int>();
  }
  auto y = at::empty({B, ldy}, x.options());
  mg::gemv(bp(x), bp(W), bp(y), (int)B, (int)N, (int)K, ldy, bias.has_value() ? bp(*bias) : nullptr,
           epi == 3 ? bp(*resid) : nullptr, (int)epi, cur_stream(), bp_opt(lnw), bp_opt(lnb), (float)eps,
           am_part.has_value() ? &am : nullptr);
  return y;
}

// pos_dev (int32 [1] on the device, optional): the position is read by the kernel (hipGraph decode)
// part / counters (optional): the decode state's own workspace (kernels.h); without them a
// temporary pair is allocated for this call (tests; not for captured graphs)
at::Tensor attention_decode(const at::Tensor& qkv_new, const at::Tensor& cache, int64_t H,
                            int64_t pos, const c10::optional<at::Tensor>& pos_dev,
                            const c10::optional<at::Tensor>& part,
                            const c10::optional<at::Tensor>& counters) {
  CHECK_BF16(qkv_new); CHECK_BF16(cache); CHECK_CONTIG(qkv_new); CHECK_CONTIG(cache);
  TORCH_CHECK(cache.dim() == 3, "cache must be [B, Tmax, 3D]");
  const int64_t B = cache.size(0), Tmax = cache.size(1), D3 = cache.size(2), D = D3 / 3;
  TORCH_CHECK(qkv_new.numel() == B * D3 && D % H == 0, "attention_decode: shape mismatch");
  TORCH_CHECK(pos >= 0 && pos < Tmax && (D / H) % 8 == 0 && D / H <= 128, "attention_decode: pos / head dim");
  TORCH_CHECK(Tmax <= 4096, "attention_decode: KV cache longer than 4096 positions");
  DevGuard g(cache.device());
  auto out = at::empty({B, D}, cache.options());
  const int* pd = nullptr;
  if (pos_dev.has_value()) {
    TORCH_CHECK(pos_dev->scalar_type() == at::kInt && pos_dev->is_cuda(), "pos_dev must be int32 cuda");
    pd = pos_dev->data_ptr<int>();
  }
  const int64_t np = (int64_t)mg::attention_decode_part_floats((int)B, (int)H, (int)(D / H));
  at::Tensor pt, ct;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(counters.has_value() && counters->defined(), "attention_decode: part without counters");
    CHECK_F32(*part); CHECK_DEV(*counters);
    TORCH_CHECK(part->numel() >= np && part->device() == cache.device(), "attention_decode: part workspace too small");
    TORCH_CHECK(counters->scalar_type() == at::kInt && counters->numel() >= B * H &&
                counters->device() == cache.device(), "attention_decode: counters must be int32 [B * H]");
    pt = *part;
    ct = *counters;
  } else {
    pt = at::empty({np}, cache.options().dtype(at::kFloat));
    ct = at::zeros({B * H}, cache.options().dtype(at::kInt));
  }
  mg::attention_decode(bp(qkv_new), bp(cache), bp(out), (int)B, (int)H, (int)(D / H), Tmax, (int)pos,
                       cur_stream(), fp(pt), reinterpret_cast<unsigned*>(ct.data_ptr<int>()), pd);
  return out;
}

// ------------------------------------------------------------------------------- native RCCL
// csrc/comm/rccl_comm.cpp.  Every collective runs on the communicator's comm stream after the
// tensor's device's CURRENT stream (the producers); comm_wait makes that stream wait again.
mg::comm::DType comm_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return mg::comm::DType::F32;
    case at::kBFloat16: return mg::comm::DType::BF16;
    case at::kHalf: return mg::comm::DType::F16;
    case at::kLong: return mg::comm::DType::I64;
    case at::kByte: return mg::comm::DType::U8;
    default: TORCH_CHECK(false, "comm: unsupported dtype ", t.scalar_type());
  }
}

hipStream_t comm_cs(int64_t h, const at::Tensor& t) {
  CHECK_DEV(t);
  CHECK_CONTIG(t);
  TORCH_CHECK(t.device().index() == mg::comm::device(h), "comm: tensor on device ", t.device().index(),
              ", communicator on device ", mg::comm::device(h));
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

int64_t comm_all_reduce(int64_t h, const at::Tensor& t) {
  hipStream_t cs = comm_cs(h, t);
  return mg::comm::all_reduce(h, t.data_ptr(), (size_t)t.numel(), comm_dtype(t), cs);
}

int64_t comm_reduce_scatter(int64_t h, const at::Tensor& in, const at::Tensor& out) {
  hipStream_t cs = comm_cs(h, in);
  comm_cs(h, out);
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "comm_reduce_scatter: dtype mismatch");
  TORCH_CHECK(in.numel() == out.numel() * mg::comm::nranks(h), "comm_reduce_scatter: input must hold nranks x output");
  return mg::comm::reduce_scatter(h, in.data_ptr(), out.data_ptr(), (size_t)out.numel(), comm_dtype(in), cs);
}

int64_t comm_all_gather(int64_t h, const at::Tensor& in, const at::Tensor& out) {
  hipStream_t cs = comm_cs(h, in);
  comm_cs(h, out);
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "comm_all_gather: dtype mismatch");
  TORCH_CHECK(out.numel() == in.numel() * mg::comm::nranks(h), "comm_all_gather: output must hold nranks x input");
  return mg::comm::all_gather(h, in.data_ptr(), out.data_ptr(), (size_t)in.numel(), comm_dtype(in), cs);
}

int64_t comm_broadcast(int64_t h, const at::Tensor& t, int64_t root) {
  hipStream_t cs = comm_cs(h, t);
  TORCH_CHECK(root >= 0 && root < mg::comm::nranks(h), "comm_broadcast: bad root");
  return mg::comm::broadcast(h, t.data_ptr(), (size_t)t.numel(), comm_dtype(t), (int)root, cs);
}

void comm_wait(int64_t h, int64_t ticket) {
  const int d = mg::comm::device(h);
  mg::comm::wait(h, ticket, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(d).stream());
}

}  // namespace


PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("comm_load", [](const std::string& path) {
    mg::comm::load_rccl(path);
    return (int64_t)mg::comm::rccl_version();
  }, py::arg("path") = std::string());
  m.def("comm_unique_id", []() { return py::bytes(mg::comm::unique_id()); });
  m.def("comm_create", [](const py::bytes& uid, int64_t nranks, int64_t rank, int64_t device) {
    return mg::comm::create(std::string(uid), (int)nranks, (int)rank, (int)device);
  });
  m.def("comm_destroy", &mg::comm::destroy);
  m.def("comm_stream_ptr", [](int64_t h) { return (int64_t)(intptr_t)mg::comm::comm_stream(h); });
  m.def("comm_all_reduce", &comm_all_reduce);
  m.def("comm_reduce_scatter", &comm_reduce_scatter);
  m.def("comm_all_gather", &comm_all_gather);
  m.def("comm_broadcast", &comm_broadcast);
  m.def("comm_wait", &comm_wait);
  m.def("comm_pending", &mg::comm::pending);
  m.def("comm_retire", &mg::comm::retire);
  m.def("comm_query", &mg::comm::query);
  m.doc() = "mingpt_distributed_amd gfx950 kernels";
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd_plain);
  m.def("layernorm_bwd_dropout", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("dw"), py::arg("db"), py::arg("dres"), py::arg("dz_bias"),
        py::arg("drop_p"), py::arg("drop_seed"));
  m.def("embedding_fwd", &embedding_fwd, py::arg("idx"), py::arg("wte"), py::arg("wpe"), py::arg("p"),
        py::arg("seed"), py::arg("pos_dev") = py::none(), py::arg("am_part") = py::none(),
        py::arg("seq") = py::none());
  // debug builds: OR of the device error words (1/2 = token id out of range in embedding fwd/bwd,
  // 4 = cross-entropy target >= V), cleared on read; always 0 in release builds
  m.def("debug_error_bits", []() -> int64_t { return (int64_t)mg::debug_error_bits(); });
  m.def("debug_build", []() {
#ifdef MG_DEBUG
    return true;
#else
    return false;
#endif
  });
  m.def("embedding_bwd", &embedding_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("xent_fused", &xent_fused);
  m.def("xent_scale_", &xent_scale_);
  m.def("set_graph_state", &set_graph_state, py::arg("seed_ofs") = py::none(), py::arg("opt_hp") = py::none());
  m.def("grad_sumsq", &grad_sumsq);
  m.def("grad_sumsq_chunks", &grad_sumsq_chunks);
  m.def("adamw_step", &adamw_step, py::arg("chunk_start"), py::arg("chunk_len"), py::arg("chunk_wd"),
        py::arg("moment_start"), py::arg("master"), py::arg("param"), py::arg("grad"), py::arg("m"),
        py::arg("v"), py::arg("norm"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
        py::arg("step"), py::arg("grad_scale"), py::arg("clip"), py::arg("table_end"),
        py::arg("moment_end"), py::arg("zero_grad") = py::none());
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("comm_proxy", &comm_proxy);
  m.def("bias_act", &bias_act);
  m.def("bias_dropout_residual", &bias_dropout_residual);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("transpose", &transpose);
  m.def("bias_grad", &bias_grad);
  m.def("dropout_bias_grad", &dropout_bias_grad);
  m.def("gemm", &gemm, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("layout"), py::arg("epi"),
        py::arg("bias"), py::arg("aux"), py::arg("resid"), py::arg("p"), py::arg("seed"), py::arg("M"),
        py::arg("N"), py::arg("dbias") = py::none());
  m.def("gemm_set_variant", &mg::gemm_set_variant);
  m.def("gemm_get_variant", &mg::gemm_get_variant);
  m.def("gemm_pick", &mg::gemm_pick, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("layout"));
  m.def("attention_set_bwd_mode", &mg::attention_set_bwd_mode);
  m.def("attention_set_bwd64", &mg::attention_set_bwd64);
#ifdef MG_BWD64_STAMPS
  m.def("attention_bwd64_stamps", []() {
    auto t = at::empty({64 * 4 * 8 * 8 + 64 * 4 * 16}, at::kLong);
    mg::attention_bwd64_stamps(reinterpret_cast<unsigned long long*>(t.data_ptr<int64_t>()));
    return t;
  });
#endif
  m.def("attention_fwd", &attention_fwd);
  m.def("attention_bwd", &attention_bwd, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"),
        py::arg("mask"), py::arg("B"), py::arg("T"), py::arg("H"), py::arg("p"), py::arg("seed"),
        py::arg("dbias") = py::none());
  m.def("gemv", &gemv, py::arg("x"), py::arg("W"), py::arg("epi"), py::arg("bias") = py::none(),
        py::arg("resid") = py::none(), py::arg("ldy") = 0, py::arg("lnw") = py::none(),
        py::arg("lnb") = py::none(), py::arg("eps") = 1e-5, py::arg("am_part") = py::none(),
        py::arg("am_pos") = py::none());
  m.def("gemv_argmax_groups", [](int64_t N, int64_t B) { return (int64_t)mg::gemv_grid((int)N, (int)B); },
        py::arg("N"), py::arg("B"));
  m.def("gemv_supported", &mg::gemv_supported);
  m.def("attention_decode", &attention_decode, py::arg("qkv_new"), py::arg("cache"), py::arg("H"),
        py::arg("pos"), py::arg("pos_dev") = py::none(), py::arg("part") = py::none(),
        py::arg("counters") = py::none());
  m.def("attention_decode_part_floats", [](int64_t B, int64_t H, int64_t hd) {
    return (int64_t)mg::attention_decode_part_floats((int)B, (int)H, (int)hd);
  });
}
