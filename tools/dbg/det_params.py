"""Which parameters / buffers differ between two identical train-mode runs (determinism check)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mil_nce_howto100m_amd.config import get_args  # noqa: E402
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips  # noqa: E402
from mil_nce_howto100m_amd.ops import grad_sink  # noqa: E402
from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.parallel import dist as pdist  # noqa: E402
from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything  # noqa: E402

args = get_args(argv=["--batch_size", "4", "--num_frames", "8", "--video_size", "64", "--num_candidates", "2",
                      "--blocks", "mixed_3b,mixed_3c,mixed_4b", "--word2vec_path", "", "--vocab_size", "1000"])
ctx = pdist.DistContext(device=torch.device("cuda", 0))
data = SyntheticClips(4, 8, 64, 2, 20, 1000, device=ctx.device)


def run():
    seed_everything(1, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
    for p in tr.bucketer.params:
        p._milnce_flat_grad = True
    tr.model.train()
    for step in range(2):
        tr.bucketer.zero()
        h.zero_arena_begin(ctx.device)
        tr.forward_loss(data.batch(step)).backward()
        h.zero_arena_end()
        grad_sink.drain()
    torch.cuda.synchronize()
    g = {n: p.grad.clone() for n, p in tr.model.named_parameters() if p.grad is not None}
    b = {n: t.clone().float() for n, t in tr.model.named_buffers()}
    return g, b


(g1, b1), (g2, b2) = run(), run()
for n in g1:
    if not torch.equal(g1[n], g2[n]):
        print("grad", n, (g1[n] - g2[n]).abs().max().item(), g1[n].abs().max().item())
for n in b1:
    if not torch.equal(b1[n], b2[n]):
        print("buffer", n, (b1[n] - b2[n]).abs().max().item())
print("done")
