"""Static check of the compiled GEMM kernels (no GPU needed): accumulators written by inline-asm
MFMAs must not be read by compiler-placed code (epilogue reads, spills, copies) before the MFMA
result is ready -- hipcc cannot see the latency of an asm MFMA (scripts/mfma_hazards.py)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_gemm_inline_asm_mfma_hazards(tmp_path):
    out = tmp_path / "gemm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
                    "--cuda-device-only", "-S", "-I" + os.path.join(ROOT, "csrc", "include"),
                    os.path.join(ROOT, "csrc", "kernels", "gemm.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "mfma_hazards.py"), str(out), "w4_kernel"],
                       check=True, capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if "early AGPR reads" in l]
    assert lines, r.stdout
    bad = [l for l in lines if not l.rstrip().endswith(": 0 early AGPR reads")]
    assert not bad, "\n".join(bad)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_gemm_asm_lds_reads_waited(tmp_path):
    """Transposing LDS reads are inline asm (so hipcc does not drain the LDS-DMA queue before each
    one); no instruction may read their destination registers before an lgkmcnt(0)."""
    out = tmp_path / "gemm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
                    "--cuda-device-only", "-S", "-I" + os.path.join(ROOT, "csrc", "include"),
                    os.path.join(ROOT, "csrc", "kernels", "gemm.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "mfma_hazards.py"), str(out), "gemm", "--lds"],
                       check=True, capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if "asm LDS results" in l]
    assert len(lines) > 10, r.stdout
    bad = [l for l in lines if not l.rstrip().endswith(": 0 early reads of asm LDS results")]
    assert not bad, "\n".join(bad)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_attention_bwd64_asm_mfma_operands(tmp_path):
    """attn_bwd64_kernel's S / dP~ MFMAs are inline asm (VGPR accumulators): no compiler-placed VALU
    write of any of their operands may land < 2 wait states before one (hipcc does not pad asm),
    and its steady tile loop must hold no scratch access."""
    out = tmp_path / "attn.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-fno-slp-vectorize",
                    "--cuda-device-only", "-S", "-I" + os.path.join(ROOT, "csrc", "include"),
                    os.path.join(ROOT, "csrc", "kernels", "attention_train.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "mfma_hazards.py"), str(out), "attn_bwd64",
                        "--operands"], check=True, capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if "asm-MFMA operands" in l]
    assert len(lines) == 1 and lines[0].rstrip().endswith(": 0 asm-MFMA operands written < 2 wait states before or results read < 12 after"), r.stdout
    # no scratch access inside the steady tile loop: a spill reload there waits vmcnt(0), i.e. for
    # the next tile's in-flight loads / DMA and this tile's dQ stores (measured: 2-8k cycles a tile)
    text = out.read_text()
    m = re.search(r"^(_Z\S*attn_bwd64_kernel\S*):", text, re.M)
    body = text[m.end():text.find(".Lfunc_end", m.end())].split("\n")
    # the work-item loop (Depth=1) around the diagonal-tile and steady-tile loops (Depth=2)
    hdrs = [i for i, l in enumerate(body) if "Loop Header: Depth=2" in l]
    assert len(hdrs) == 2, "expected the diagonal-tile and steady-tile loops inside the item loop"
    labels = {l.split(":")[0].strip(): i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l.strip())}
    # back edges of the steady loop: branches after its header to a label after the diagonal loop's
    back = [(i, labels[mm.group(1)]) for i, l in enumerate(body)
            if (mm := re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)) and i > hdrs[1]
            and hdrs[0] < labels.get(mm.group(1), -1) <= hdrs[1]]
    end, start = max(i for i, _ in back), min(t for _, t in back)
    scratch = [l.strip() for l in body[start:end + 1] if "scratch_" in l]
    assert not scratch, scratch[:5]
