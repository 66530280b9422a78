import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.config import get_args
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
from mil_nce_howto100m_amd.parallel import dist as pdist
from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
from mil_nce_howto100m_amd.ops import hip_ops as h
args = get_args(argv=["--batch_size", "4", "--num_frames", "8", "--video_size", "64", "--num_candidates", "2",
                      "--blocks", "mixed_3b,mixed_3c", "--word2vec_path", "", "--vocab_size", "1000"])
ctx = pdist.DistContext(device=torch.device("cuda", 0))
data = SyntheticClips(4, 8, 64, 2, 20, 1000, device=ctx.device)
order = [d == "1" for d in (sys.argv[1] if len(sys.argv) > 1 else "101")]
flats, trs = [], []
for direct in order:
    seed_everything(1, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
    for p in tr.bucketer.params:
        p._milnce_flat_grad = direct
    tr.model.eval()
    tr.bucketer.zero()
    for _ in range(2):
        tr.forward_loss(data.batch(0)).backward()
    torch.cuda.synchronize()
    flats.append(tr.bucketer.flat.clone())
    trs.append(tr)
names = {id(p): n for n, p in trs[0].model.named_parameters()}
for i in range(1, len(flats)):
    bad = []
    for p in trs[0].bucketer.params:
        o = trs[0].bucketer.offsets[id(p)]
        a, b = flats[0][o:o + p.numel()], flats[i][o:o + p.numel()]
        if not torch.allclose(a, b, rtol=1e-5, atol=1e-6):
            bad.append((names[id(p)], ((a - b).norm() / (a.norm() + 1e-30)).item()))
    print(f"run 0 ({order[0]}) vs run {i} ({order[i]}): {len(bad)} params differ", bad[:12], flush=True)
print("plans with 4-wave:", sorted({(k[0][1:], p.k, p.impl, p.d_impl) for k, p in h._PLANS.items()
                                   if p.impl in (16, 17) or p.d_impl in (16, 17)}))
