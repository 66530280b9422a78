"""Parameters whose gradients reach them through autograd's AccumulateGrad in a flagship training
step (each such accumulation into the flat gradient buffer is one elementwise-add launch), as
opposed to the kernels writing the flat buffer directly."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    b = 32
    args = get_args(argv=["--word2vec_path", "", "--batch_size", str(b), "--num_frames", "16", "--video_size", "200",
                          "--num_candidates", "4"])
    ctx = pdist.DistContext(device=torch.device("cuda", 0))
    pdist.set_context(ctx)
    seed_everything(1, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 1000)
    data = SyntheticClips(b, 16, 200, 4, args.max_words, args.vocab_size, device=torch.device("cuda"))
    for i in range(2):
        tr.train_step(data.batch(i))
    hits = {}
    hs = [p.register_post_accumulate_grad_hook(lambda p, n=n: hits.__setitem__(n, hits.get(n, 0) + 1))
          for n, p in tr.model.named_parameters() if p.requires_grad]
    tr.train_step(data.batch(2))
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    print(f"{len(hits)} of {sum(1 for p in tr.model.parameters() if p.requires_grad)} parameters via AccumulateGrad")
    for n, c in sorted(hits.items()):
        print(f"  {c}  {n}")


if __name__ == "__main__":
    main()
