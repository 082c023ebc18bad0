"""CPU check of the fp8 capture guard: a deferred-update queue left by eager steps is refused
inside a HIP-graph capture instead of being recorded into the graph; before_capture() settles it."""
import pytest
import torch

from paddle2_amd.ops import fp8


def test_queued_updates_refused_while_capturing(monkeypatch):
    m = fp8.FP8TensorMeta(fp8.E4M3)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    monkeypatch.setattr(fp8, "_PENDING", [(m, None)])
    monkeypatch.setattr(fp8, "_PENDING_IDS", {id(m)})
    with pytest.raises(RuntimeError, match="before_capture"):
        fp8.flush_updates()
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setattr(fp8, "update_metas", lambda pairs: None)
    fp8.before_capture()
    assert not fp8._PENDING and not fp8._PENDING_IDS


def test_before_capture_noop_when_empty():
    fp8.before_capture()
    assert not fp8._PENDING
