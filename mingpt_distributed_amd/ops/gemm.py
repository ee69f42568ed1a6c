"""GEMM front-end for the GPU path: the three layouts a transformer step needs, each with the
epilogue fused where the data is produced.

* ``gemm_nt``      C[M,N] = A[M,K] @ B[N,K]^T   (forward; B is an nn.Linear weight [out, in])
                   epilogues: ``none`` | ``bias`` | ``gelu`` (bias + tanh-GELU, also stores
                   GELU'(z) for the backward) | ``resid`` (R + dropout(acc + bias)) |
                   ``gelu_bwd`` (acc * aux, aux = the stored GELU')
* ``gemm_nn``      C[M,N] = A[M,K] @ B[K,N]     (data gradient dX = dY @ W)
                   epilogue: ``none`` | ``gelu_bwd`` (multiply by aux = GELU'(z) from the forward)
* ``gemm_tn_acc``  C[N,K] += A[M,N]^T @ B[M,K] (weight gradient, fp32 accumulate into main_grad)

All three run on the hand-written MFMA kernels in ``csrc/kernels/gemm.hip`` (``_C.gemm``); the
training step (``ops/fused.py``) uses nothing else, and there is no runtime switch to a library
GEMM (hipBLASLt is only a reference point in ``bench/gemm_blas_shapes.py``).
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import ext

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_RESID, EPI_GELU_BWD = 0, 1, 2, 3, 4
EPI_GELU_FRAG, EPI_GELU_BWD_FRAG = 6, 7  # GELU' plane in the fragment order of the W4 256x256 tiles


def frag_aux_elems(M: int, N: int) -> int:
    """Elements of a fragment-ordered GELU' plane for an [M, N] output (whole 256x256 tiles)."""
    return -(-M // 256) * -(-N // 256) * 65536


def frag_plane_rowmajor(plane: torch.Tensor, M: int, N: int) -> torch.Tensor:
    """Row-major [M, N] view of a fragment-ordered plane (a copy; tests and debugging).  Order per
    256x256 tile: (wave row wm, wave col wn, fragment row i, fragment-column pair jp, lane, jj, 4);
    lane = 16 g + r holds row 16 i + r, columns 16 (2 jp + jj) + 4 g .. + 3 of its wave's 128^2
    quadrant (csrc/kernels/gemm.hip, epilogue_staged)."""
    tm, tn = -(-M // 256), -(-N // 256)
    v = plane[: tm * tn * 65536].view(tm, tn, 2, 2, 8, 4, 4, 16, 2, 4)
    # dims: tm tn wm wn i jp g r jj e -> rows (tm wm i r), cols (tn wn jp jj g e)
    v = v.permute(0, 2, 4, 7, 1, 3, 5, 8, 6, 9).reshape(tm * 256, tn * 256)
    return v[:M, :N].contiguous()


def frag_aux_ok(M: int, N: int, K: int) -> bool:
    """The fragment-ordered GELU' plane (epilogues 6 / 7) needs producer and consumer on the same
    256x256 tile grid: true when the dispatcher would pick W4-256 for both the forward [M, N, K]
    and the data gradient [M, N, K'] anyway (every GPT-2 / gpt2-xl training shape), so forcing
    them costs nothing."""
    C = ext()
    return C.gemm_get_variant() == 0 and C.gemm_pick(M, N, K, 0) == 5 and C.gemm_pick(M, N, K, 1) == 5


# Row-chunked launches are no longer needed for operands past 4 GiB (the GPT-2 logits beyond ~42k
# tokens): each block's buffer descriptor starts at its own tile / split origin and split-K ranges
# stay below 4 GiB (gemm.hip set_split).  The mechanism stays for tests (monkeypatch this cap).
_MAX_BYTES = 1 << 62


def _row_chunks(M: int, *row_bytes: int):
    """Row ranges [r0, r1) of an M-row operand such that no chunk of any operand whose rows are
    ``row_bytes`` wide reaches ``_MAX_BYTES``: the M-chunked launches are exact (the epilogues used
    here do not depend on the global row index)."""
    cap = max(256, (_MAX_BYTES // max(max(row_bytes), 1)) // 256 * 256)
    if M <= cap:
        return [(0, M)]
    n = -(-M // cap)
    step = min(cap, -(-(-(-M // n)) // 256) * 256)  # balanced: equal tile counts per launch
    return [(r0, min(M, r0 + step)) for r0 in range(0, M, step)]


def _check2d(t, name):
    if t.dim() != 2 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous 2-D tensor, got {tuple(t.shape)}")


def gemm_nt(a: torch.Tensor, b: torch.Tensor, *, bias: Optional[torch.Tensor] = None,
            epi: str = "none", resid: Optional[torch.Tensor] = None, p: float = 0.0, seed: int = 0,
            pre_out: Optional[torch.Tensor] = None, ld: Optional[int] = None,
            aux: Optional[torch.Tensor] = None, dbias: Optional[torch.Tensor] = None,
            frag: bool = False) -> torch.Tensor:
    """C = A @ B^T with a fused epilogue. ``ld`` pads the output row stride (logits).
    ``gelu`` writes GELU'(z) into ``pre_out``; ``gelu_bwd`` multiplies by ``aux`` (that GELU') and,
    with ``dbias`` (fp32 [N]), also adds the output's column sums into it (the bias gradient).
    ``frag=True`` (``gelu`` only): ``pre_out`` is a fragment-ordered plane of
    ``frag_aux_elems(M, N)`` elements for ``gemm_nn(..., aux_frag=True)``."""
    _check2d(a, "A")
    _check2d(b, "B")
    M, K = a.shape
    N = b.shape[0]
    ld = ld or N
    c = torch.empty((M, ld), dtype=torch.bfloat16, device=a.device)
    code = {"none": EPI_NONE, "bias": EPI_BIAS, "gelu": EPI_GELU, "resid": EPI_RESID,
            "gelu_bwd": EPI_GELU_BWD}[epi]
    if code == EPI_BIAS and bias is None:
        code = EPI_NONE
    if frag:
        if code != EPI_GELU:
            raise ValueError("gemm_nt: frag=True is the gelu epilogue's fragment-ordered GELU' plane")
        code = EPI_GELU_FRAG
    side = aux if code == EPI_GELU_BWD else pre_out
    chunks = _row_chunks(M, 2 * K, 2 * ld)
    if len(chunks) > 1 and code == EPI_GELU_FRAG:
        raise ValueError("gemm_nt: the fragment-ordered GELU' plane is one launch; operand too large")
    if len(chunks) > 1 and code == EPI_RESID and p > 0:
        raise ValueError("gemm_nt: residual dropout keys its mask on the global row; operand too large")
    for r0, r1 in chunks:
        sl = (lambda t: t if t is None or len(chunks) == 1 else t[r0:r1])
        ext().gemm(sl(a), b, sl(c), 0, code, bias, sl(side), sl(resid), float(p), int(seed), r1 - r0, N,
                   dbias)
    return c


def transpose(w: torch.Tensor, ld: Optional[int] = None) -> torch.Tensor:
    """W^T as a contiguous [cols, ld] bf16 tensor (columns >= rows zero): the B operand that turns a
    data gradient dX = dY @ W into the NT layout (both operands k-contiguous, the fast GEMM path)."""
    return ext().transpose(w, int(ld or 0))


def gemm_dgrad(dy: torch.Tensor, w: torch.Tensor, *, epi: str = "none",
               aux: Optional[torch.Tensor] = None, wt: Optional[torch.Tensor] = None,
               dbias: Optional[torch.Tensor] = None, aux_frag: bool = False) -> torch.Tensor:
    """dX = dY @ W (W [N_out, N_in] as stored by nn.Linear).  Block shapes run NN straight from the
    stored weight (the W4 kernel's transposing LDS reads; no per-step transposed copy:
    bench/dgrad_nn_vs_nt.py); a long reduction (the LM head's K = vocab) runs NT against W^T, where
    the 128x96-wave W4 tile applies.  With ``epi="gelu_bwd"`` and ``dbias`` (fp32 [N_in]), the
    column sums of the result (the next bias gradient) are accumulated in the epilogue."""
    if aux_frag or (wt is None and dy.shape[1] < 8192 and w.shape[0] == dy.shape[1]):
        return gemm_nn(dy, w, epi=epi, aux=aux, dbias=dbias, aux_frag=aux_frag)
    if wt is None:
        wt = transpose(w, dy.shape[1])
    return gemm_nt(dy, wt, epi=epi, aux=aux, dbias=dbias)


def gemm_nn(a: torch.Tensor, b: torch.Tensor, *, epi: str = "none",
            aux: Optional[torch.Tensor] = None, dbias: Optional[torch.Tensor] = None,
            aux_frag: bool = False) -> torch.Tensor:
    """C = A @ B (B row-major [K, N]); ``gelu_bwd`` multiplies by ``aux`` (a stored GELU') and,
    with ``dbias`` (fp32 [N]), adds the column sums of the fp32 C into it (staged epilogue).
    ``aux_frag``: ``aux`` is the fragment-ordered plane of ``gemm_nt(..., frag=True)``."""
    _check2d(a, "A")
    _check2d(b, "B")
    M, K = a.shape
    N = b.shape[1]
    c = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    code = {"none": EPI_NONE, "gelu_bwd": EPI_GELU_BWD}[epi]
    if dbias is not None and code != EPI_GELU_BWD:
        raise ValueError("gemm_nn: dbias is fused only into the gelu_bwd epilogue")
    if aux_frag:
        if code != EPI_GELU_BWD:
            raise ValueError("gemm_nn: aux_frag is the gelu_bwd epilogue's fragment-ordered GELU' plane")
        ext().gemm(a, b, c, 1, EPI_GELU_BWD_FRAG, None, aux, None, 0.0, 0, M, N, dbias)
        return c
    chunks = _row_chunks(M, 2 * K, 2 * N)
    for r0, r1 in chunks:
        sl = (lambda t: t if t is None or len(chunks) == 1 else t[r0:r1])
        ext().gemm(sl(a), b, sl(c), 1, code, None, sl(aux), None, 0.0, 0, r1 - r0, N, dbias)
    return c


def gemm_tn_acc(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, n_valid: Optional[int] = None):
    """c[N, K] += A[M, N]^T @ B[M, K]  (fp32 c). ``n_valid`` limits the rows of c written."""
    _check2d(a, "A")
    _check2d(b, "B")
    M, N = a.shape
    K = b.shape[1]
    if n_valid is not None:
        N = n_valid
    if c.dtype != torch.float32 or c.shape[0] < N or c.shape[1] != K:
        raise ValueError("gemm_tn_acc: c must be fp32 [N, K]")
    # the reduction runs over M: chunks accumulate into c one after another
    for r0, r1 in _row_chunks(M, 2 * a.shape[1], 2 * K):
        ext().gemm(a[r0:r1], b[r0:r1], c, 2, EPI_NONE, None, None, None, 0.0, 0, N, K)
    return c
