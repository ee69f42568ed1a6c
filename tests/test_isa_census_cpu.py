"""scripts/isa_census.py on a synthetic kernel listing: the loop span comes from the back edge
(hipcc rotates loops), nested loops are picked by --depth / --loop, instructions are counted by
purpose, and --cold moves the blocks holding a matching instruction out of the hot path."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ASM = """\t.text
_Z6kernelv:
\ts_mov_b32 s0, 0
.LBB0_1:                                ; =>This Loop Header: Depth=1
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]
.LBB0_2:                                ; =>  This Inner Loop Header: Depth=2
\tv_exp_f32_e32 v1, v2
\tv_max3_f32 v3, v4, v5, v6
\tv_add_u32_e32 v7, 16, v7
\tds_read_b128 v[8:11], v7
\ts_cbranch_scc1 .LBB0_2
\tv_cmp_gt_i32_e32 vcc, v1, v2
\tv_cndmask_b32_e32 v3, v4, v5, vcc
\tbuffer_store_dword v1, v2, s[0:3], 0 offen
\ts_cbranch_scc1 .LBB0_1
\ts_endpgm
.Lfunc_end0:
"""


def _run(tmp_path, *args):
    p = tmp_path / "k.s"
    p.write_text(ASM)
    return subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "isa_census.py"), str(p), "kernel", *args],
                          check=True, capture_output=True, text=True).stdout


def test_outer_loop_counts(tmp_path):
    out = _run(tmp_path)
    assert "1 MFMA" in out
    lines = {l.split()[0]: int(l.split()[1]) for l in out.splitlines() if l.startswith("   ")}
    assert lines["mfma"] == 1 and lines["exp"] == 1 and lines["softmax-math"] == 1  # max3 is softmax math
    assert lines["address"] == 1 and lines["compare-sel"] == 2 and lines["lds-read"] == 1
    assert lines["vmem-store"] == 1 and lines["branch"] == 2


def test_inner_loop_and_cold_blocks(tmp_path):
    out = _run(tmp_path, "--depth=2")
    lines = {l.split()[0]: int(l.split()[1]) for l in out.splitlines() if l.startswith("   ")}
    assert "mfma" not in lines and lines["exp"] == 1 and lines["branch"] == 1
    cold = _run(tmp_path, "--cold=v_cmp")
    assert "-- cold blocks" in cold
