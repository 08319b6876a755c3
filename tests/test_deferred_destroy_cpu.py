"""Library objects freed while a stream records a hipGraph (Python's garbage
collector can run inside a capture) are destroyed after the capture ends, not
during it (_lib.destroy / flush_deferred)."""
import torch

import distributed_training_amd as D
from distributed_training_amd import _lib as L


def test_destroy_is_parked_while_capturing(monkeypatch):
    plan = D.multi_tensor.TensorListPlan([8, 3], torch.device("cpu"))
    h = plan.handle
    calls = []
    real = L.lib().gs_plan_destroy
    monkeypatch.setattr(L, "_capturing", lambda: True)
    plan.close()
    assert plan.handle is None and L._deferred == [("gs_plan_destroy", h)]
    L.flush_deferred()  # still capturing: nothing runs
    assert len(L._deferred) == 1
    monkeypatch.setattr(L, "_capturing", lambda: False)

    class Spy:
        def __getattr__(self, name):
            if name == "gs_plan_destroy":
                return lambda x: (calls.append(x), real(x))[1]
            return getattr(L._lib, name)

    monkeypatch.setattr(L, "lib", lambda: Spy())
    L.flush_deferred()
    assert calls == [h] and L._deferred == []
