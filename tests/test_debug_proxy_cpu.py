"""The MINGPT_DEBUG_CHECKS extension proxy (ops/_ext.py) on CPU: error bits map to a named
DeviceCheckError; non-callables and the debug entry points pass through."""
import pytest

from mingpt_distributed_amd.ops import _ext


class _FakeMod:
    VERSION = 3

    def __init__(self):
        self.bits = 0

    def debug_error_bits(self):
        b, self.bits = self.bits, 0
        return b

    def debug_build(self):
        return True

    def embedding_fwd(self, v):
        if v < 0:
            self.bits |= 1
        return v * 2


def test_checked_proxy(monkeypatch):
    import torch

    monkeypatch.setattr(torch.cuda, "synchronize", lambda: None)
    m = _FakeMod()
    p = _ext._Checked(m)
    assert p.VERSION == 3 and p.debug_build()
    assert p.embedding_fwd(4) == 8
    with pytest.raises(_ext.DeviceCheckError, match="embedding_fwd.*token id"):
        p.embedding_fwd(-1)
    assert m.bits == 0
