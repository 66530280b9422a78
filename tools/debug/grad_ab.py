"""Debug: per-parameter gradient differences HIP vs ATen (train-mode BN, softened logits)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_gpu_training as T
from mil_nce_howto100m_amd import ops
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips

extra = ["--batch_size", "32", "--num_frames", "16", "--video_size", "96", "--num_candidates", "4"]
mode = sys.argv[1] if len(sys.argv) > 1 else "train"
res = {}
soft = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
batch0 = None
for name, aten, direct in (("hip", False, True), ("hip_nodirect", False, False), ("aten", True, True),
                           ("cpu", True, True)):
    tr, args = T._trainer(extra, seed=5)
    if name == "cpu":
        from mil_nce_howto100m_amd.parallel import dist as pdist
        from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
        ctx = pdist.DistContext(device=torch.device("cpu"))
        pdist.set_context(ctx)
        seed_everything(5, 0)
        tr = Trainer(args, build_model(args, ctx.device), ctx, 1000)
    T._soften(tr, soft)
    if not direct:
        for p in tr.bucketer.params:
            p._milnce_flat_grad = False
    if batch0 is None:
        batch0 = SyntheticClips(32, 16, 96, 4, args.max_words, args.vocab_size, device=torch.device("cuda")).batch(0)
    batch = {k: (v.cpu() if name == "cpu" else v) for k, v in batch0.items()}
    with (ops.force_aten() if aten else T._Null()):
        getattr(tr.model, mode)()
        tr.bucketer.zero()
        loss = tr.forward_loss(batch)
        loss.backward()
    torch.cuda.synchronize()
    res[name] = (float(loss), {n: (p.grad.detach().double().clone() if p.grad is not None else None)
                               for n, p in tr.model.named_parameters() if p.requires_grad})
    print(name, "loss", res[name][0], flush=True)
ref = res["cpu"][1]
rel = lambda x, r: ((x - r).norm() / (r.norm() + 1e-30)).item()  # noqa: E731
rows = []
for n in ref:
    r = ref[n].cpu()
    rows.append((rel(res["hip"][1][n].cpu(), r), rel(res["hip_nodirect"][1][n].cpu(), r),
                 rel(res["aten"][1][n].cpu(), r), r.norm().item(), n))
rows.sort(reverse=True)
for r in rows[:30]:
    print(f"vs cpu-fp32: hip {r[0]:8.4f} nodirect {r[1]:8.4f} aten-bf16 {r[2]:8.4f} |g| {r[3]:10.3e}  {r[4]}")
for i, nm in enumerate(("hip", "hip_nodirect", "aten")):
    print("median rel vs cpu", nm, sorted(r[i] for r in rows)[len(rows) // 2])
