"""Static check of the compiled GEMM kernels (no GPU needed): accumulators written by inline-asm
MFMAs must not be read by compiler-placed code (epilogue reads, spills, copies) before the MFMA
result is ready -- hipcc cannot see the latency of an asm MFMA (scripts/mfma_hazards.py)."""
import os
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
