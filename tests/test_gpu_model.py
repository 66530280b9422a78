"""End-to-end: the full HIP path of the model/step against the ATen path with the same weights."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_model_forward_backward_matches_aten():
    from mil_nce_howto100m_amd.models import S3D
    from mil_nce_howto100m_amd.ops import aten
    torch.manual_seed(0)
    m = S3D(512, blocks=["mixed_3b", "mixed_3c", "mixed_4b"]).cuda()
    ref = copy.deepcopy(m).cpu().double()
    v = torch.randint(0, 256, (4, 3, 8, 64, 64), dtype=torch.uint8)
    t = torch.randint(0, 66250, (8, 20))
    ve, te = m(v.cuda(), t.cuda())
    import mil_nce_howto100m_amd.ops as ops_mod
    # oracle: CPU fp64 ATen path with identical parameters
    ver, ter = ref(v.double() / 255.0, t)
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()
    assert rel(ve, ver) < 0.08
    assert rel(te, ter) < 0.02
    # Identical upstream gradients (a fixed random linear functional of the embeddings): the
    # MIL-NCE softmax would amplify the bf16 forward differences into the comparison.
    gv = torch.randn(ve.shape, dtype=torch.float64)
    gt = torch.randn(te.shape, dtype=torch.float64)
    ((ve.double() * gv.cuda()).sum() + (te.double() * gt.cuda()).sum()).backward()
    ((ver * gv).sum() + (ter * gt).sum()).backward()
    errs = []
    for (n1, p1), (n2, p2) in zip(m.named_parameters(), ref.named_parameters()):
        if p2.grad is None:
            continue
        assert p1.grad is not None, n1
        errs.append((n1, rel(p1.grad, p2.grad), p2.grad.norm().item()))
    for n, e, g in errs:
        print(f"{n:45s} rel_err={e:.4f} |g|={g:.3e}")
    bad = [(n, e) for n, e, g in errs if e > 0.12]
    assert not bad, bad


def test_bench_step_runs():
    import subprocess, sys, json, os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--batch_per_gpu", "8", "--size", "64", "--num_frames", "8"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["value"] > 0 and out["n_gpus"] == 1
