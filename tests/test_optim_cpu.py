"""FlatAdam vs torch.optim.Adam, state_dict compatibility both ways, the LR schedule."""
import math

import torch
import torch.nn as nn

from mil_nce_howto100m_amd.train.optim import FlatAdam, cosine_schedule_with_warmup


def _params(seed=0):
    torch.manual_seed(seed)
    m = nn.Sequential(nn.Linear(7, 5), nn.Linear(5, 3))
    frozen = nn.Embedding(4, 3)
    frozen.weight.requires_grad_(False)
    return m, frozen


def test_flat_adam_matches_torch_adam():
    m1, f1 = _params()
    m2, f2 = _params()
    p1 = list(m1.parameters()) + [f1.weight]
    p2 = list(m2.parameters()) + [f2.weight]
    o1 = FlatAdam(p1, lr=1e-2)
    o2 = torch.optim.Adam(p2, lr=1e-2)
    for step in range(6):
        x = torch.randn(4, 7)
        for m, o in ((m1, o1), (m2, o2)):
            if isinstance(o, FlatAdam):
                for p in o.trainable:
                    p.grad = torch.zeros_like(p)
            else:
                o.zero_grad()
            m(x).pow(2).sum().backward()
            o.step()
    for a, b in zip(p1, p2):
        assert torch.allclose(a, b, atol=1e-6)


def test_state_dict_roundtrip_with_torch_adam():
    m1, f1 = _params(1)
    p1 = list(m1.parameters()) + [f1.weight]
    o1 = FlatAdam(p1, lr=3e-3)
    for p in o1.trainable:
        p.grad = torch.randn_like(p)
    o1.step()
    sd = o1.state_dict()
    assert len(sd["param_groups"][0]["params"]) == 5
    assert set(sd["state"].keys()) == {0, 1, 2, 3}  # frozen param has no state
    assert set(sd["state"][0].keys()) == {"step", "exp_avg", "exp_avg_sq"}
    # torch Adam accepts it...
    m2, f2 = _params(1)
    o2 = torch.optim.Adam(list(m2.parameters()) + [f2.weight], lr=3e-3)
    o2.load_state_dict(sd)
    # ... and FlatAdam accepts torch's
    m3, f3 = _params(1)
    o3 = FlatAdam(list(m3.parameters()) + [f3.weight], lr=3e-3)
    o3.load_state_dict(o2.state_dict())
    assert o3.step_count == 1
    for k in sd["state"]:
        assert torch.equal(o3.state_dict()["state"][k]["exp_avg"], sd["state"][k]["exp_avg"])


def test_cosine_warmup_schedule_values():
    p = nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    s = cosine_schedule_with_warmup(opt, 10, 110)
    lrs = []
    for _ in range(111):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        s.step()
    assert lrs[0] == 0.0 and abs(lrs[5] - 0.5) < 1e-12 and abs(lrs[10] - 1.0) < 1e-12
    assert abs(lrs[60] - 0.5 * (1 + math.cos(math.pi * 0.5))) < 1e-12
    assert abs(lrs[110]) < 1e-12
