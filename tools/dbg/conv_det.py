"""Record every conv forward / dgrad output of three identical eval-mode model steps and report
the calls whose outputs differ between the runs (with their plan and kernel variant)."""
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
seed_everything(1, 0)
tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
tr.model.eval()
rec = []
of, od, ob = h.conv_forward_raw, h.conv_dgrad, h.conv_dgrad_bnbwd


def fwd(x, wp, plan, stats, pro=None, shift=None):
    xin = x.clone() if x.stride()[-1] != 0 else None
    y = of(x, wp, plan, stats, pro, shift)
    rec.append(("fwd", plan.k, plan.Cin, plan.Cout, plan.impl, plan.grid_m, xin, y.clone(), pro is not None))
    return y


def dg(dy, wd, plan, producer_bn=None):
    dx = od(dy, wd, plan, producer_bn)
    rec.append(("dgrad", plan.k, plan.Cin, plan.Cout, plan.d_impl, plan.d_grid_m, dy.clone(), dx.clone(), False))
    return dx


def dgb(dz, wd, plan, producer_bn, y, ss, coef, dy_out, impl=0, grid=0, dx=None):
    r = ob(dz, wd, plan, producer_bn, y, ss, coef, dy_out, impl, grid, dx)
    rec.append(("dgradbn", plan.k, plan.Cin, plan.Cout, impl or plan.d_impl, grid or plan.d_grid_m, dz.clone(),
                r.clone(), True))
    return r


h.conv_forward_raw, h.conv_dgrad, h.conv_dgrad_bnbwd = fwd, dg, dgb
state = {k: v.clone() for k, v in tr.model.state_dict().items()}
runs = []
for rep in range(3):
    tr.model.load_state_dict(state)
    tr.bucketer.zero()
    rec.clear()
    tr.forward_loss(data.batch(0)).backward()
    torch.cuda.synchronize()
    runs.append(list(rec))
a, b = runs[1], runs[2]
print("calls", len(a), len(b))
for i, (ra, rb) in enumerate(zip(a, b)):
    in_same = ra[6] is None or rb[6] is None or torch.equal(ra[6], rb[6])
    out_same = torch.equal(ra[7], rb[7])
    if not (in_same and out_same):
        print(i, ra[0], ra[1], ra[2], ra[3], "impl", ra[4], "grid", ra[5], "pro", ra[8], "input same", in_same,
              "output same", out_same, flush=True)
