"""Build-artifact checks that need no GPU: the in-tree extension (``python build_ext.py``) must not
reference symbols that only it could define (see ``build_ext.anon_undefined``)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import build_ext  # noqa: E402


def test_extension_has_no_unresolvable_internal_symbols():
    so = os.path.join(ROOT, "mingpt_distributed_amd", "_C.so")
    if not os.path.exists(so):
        pytest.skip("extension not built (python build_ext.py)")
    assert build_ext.anon_undefined(so) == []


def test_anon_undefined_flags_a_missing_kernel_stub(tmp_path):
    """A library that calls an anonymous-namespace function it does not define is reported."""
    src = tmp_path / "m.cpp"
    src.write_text("namespace { void kernel_stub(); }\nvoid call() { kernel_stub(); }\n")
    so = tmp_path / "m.so"
    if os.system(f"g++ -shared -fPIC -o {so} {src} 2>/dev/null") != 0:
        pytest.skip("no host C++ compiler")
    bad = build_ext.anon_undefined(str(so))
    assert len(bad) == 1 and "_GLOBAL__N_" in bad[0]
