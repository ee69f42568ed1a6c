"""ops/gemm.frag_plane_rowmajor decodes the fragment order the W4 epilogues 6 / 7 use for the GELU'
plane (csrc/kernels/gemm.hip epilogue_staged: per 256 x 256 tile, (wave row wm, wave col wn,
fragment row i, fragment-column pair jp, lane = 16 g + r, jj, 4), lane holding row 16 i + r and
columns 16 (2 jp + jj) + 4 g .. + 3 of its wave's 128 x 128 quadrant).  Built here element by
element from that definition (CPU, no extension needed), partial tiles included."""
import itertools

import pytest
import torch

from mingpt_distributed_amd.ops.gemm import frag_aux_elems, frag_plane_rowmajor


@pytest.mark.parametrize("M,N", [(256, 256), (300, 520), (512, 768)])
def test_fragment_plane_decoder(M, N):
    tm, tn = -(-M // 256), -(-N // 256)
    assert frag_aux_elems(M, N) == tm * tn * 65536
    ref = torch.arange(tm * 256 * tn * 256, dtype=torch.float64).view(tm * 256, tn * 256)
    # the kernel's store order, written out as nested loops (slowest index first)
    rows, cols = [], []
    for a, b, wm, wn, i, jp, lane, jj, e in itertools.product(range(tm), range(tn), range(2), range(2), range(8),
                                                              range(4), range(64), range(2), range(4)):
        rows.append(a * 256 + wm * 128 + 16 * i + (lane & 15))
        cols.append(b * 256 + wn * 128 + 16 * (2 * jp + jj) + 4 * (lane >> 4) + e)
    plane = ref[torch.tensor(rows), torch.tensor(cols)]
    assert torch.equal(frag_plane_rowmajor(plane, M, N), ref[:M, :N])
