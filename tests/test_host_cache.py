"""The opt-in host-operand device cache (aggregate._OperandCache, TAL_HOST_CACHE_GB): an entry
is reused only while its model is alive and unchanged (data pointers and version counters of
every state tensor); LRU eviction by bytes.  CPU only: the cache logic is device-agnostic."""
import gc

import torch

from topology_aware_learning_amd import aggregate
from topology_aware_learning_amd.aggregate import _OperandCache


def _segs(n):
    return {"f32": torch.zeros(n)}


def test_hit_while_unchanged_miss_after_changes():
    c = _OperandCache(1 << 20)
    m = torch.nn.Linear(4, 3)
    dev = torch.device("cpu")
    sig = _OperandCache.signature(m.state_dict())
    c.put(m, sig, dev, _segs(15))
    assert c.get(m, _OperandCache.signature(m.state_dict()), dev) is not None
    with torch.no_grad():
        m.weight.add_(1.0)  # an optimizer step / copy_ bumps the version counter
    assert c.get(m, _OperandCache.signature(m.state_dict()), dev) is None
    c.put(m, _OperandCache.signature(m.state_dict()), dev, _segs(15))
    m.weight.data = m.weight.data.clone()  # re-pointed storage
    assert c.get(m, _OperandCache.signature(m.state_dict()), dev) is None
    c.put(m, _OperandCache.signature(m.state_dict()), dev, _segs(15))
    assert c.get(m, _OperandCache.signature(m.state_dict()), torch.device("meta")) is None  # other device


def test_entry_dropped_with_its_model():
    c = _OperandCache(1 << 20)
    m = torch.nn.Linear(4, 3)
    c.put(m, _OperandCache.signature(m.state_dict()), torch.device("cpu"), _segs(15))
    assert len(c.entries) == 1 and c.used == 60
    del m
    gc.collect()
    assert len(c.entries) == 0 and c.used == 0


def test_lru_eviction_by_bytes():
    c = _OperandCache(100 * 4)
    ms = [torch.nn.Linear(2, 2) for _ in range(3)]
    for m in ms:
        c.put(m, _OperandCache.signature(m.state_dict()), torch.device("cpu"), _segs(40))
    assert len(c.entries) == 2 and c.used == 320  # the first one evicted
    assert c.get(ms[0], _OperandCache.signature(ms[0].state_dict()), torch.device("cpu")) is None
    assert c.get(ms[2], _OperandCache.signature(ms[2].state_dict()), torch.device("cpu")) is not None
    c.put(ms[0], _OperandCache.signature(ms[0].state_dict()), torch.device("cpu"), _segs(1000))  # > cap
    assert len(c.entries) == 2


def test_pinned_binding_default_and_opt_out(monkeypatch):
    """Pinned binding of CPU models is the default (TAL_HOST_PIN unset); with TAL_HOST_PIN=0 a
    CPU model is never re-pointed to pinned rows (the call packs into staging buffers and
    leaves the model's tensors alone)."""
    from topology_aware_learning_amd.arena import StateLayout

    monkeypatch.delenv("TAL_HOST_PIN", raising=False)
    assert aggregate._pin_enabled()
    m = torch.nn.Linear(3, 2)
    lay = StateLayout.from_state_dict(m.state_dict())
    ptr = m.weight.data_ptr()
    monkeypatch.setenv("TAL_HOST_PIN", "0")
    assert not aggregate._pin_enabled()
    assert aggregate._host_binding(m, lay) is None and m.weight.data_ptr() == ptr
    assert aggregate.bound_row(m) is None
