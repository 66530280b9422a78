"""Loss of a fresh model on one synthetic batch (GPU), for A/B checks of fused paths."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mil_nce_howto100m_amd.config import get_args
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
from mil_nce_howto100m_amd.parallel import dist as pdist
from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ctx = pdist.init_distributed("nccl", "auto")
args = get_args(argv=["--batch_size", str(b), "--word2vec_path", "", "--lr", "0.001", "--warmup_steps", "10000"])
data = SyntheticClips(b, 16, 200, 4, 20, 66250, device=ctx.device)
seed_everything(1, 0)
tr = Trainer(args, build_model(args, ctx.device), ctx, 100)
tr.model.train()
with torch.no_grad():
    for i in range(2):
        print("fuse", os.environ.get("MILNCE_FUSE_STEM_POOL", "1"), "bs", b, "loss", float(tr.forward_loss(data.batch(i))))
for i in range(3):
    print("step", i, float(tr.train_step(data.batch(i))))
