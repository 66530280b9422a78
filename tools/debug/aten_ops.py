"""Which ATen ops (not HIP-kernel calls) run inside one flagship training step, with their Python
call sites: the step's small elementwise / copy launches (rocprof shows them as
vectorized_elementwise_kernel / copyBuffer)."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mil_nce_howto100m_amd.config import get_args
    from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
    b = int(os.environ.get("B", "64"))
    args = get_args(argv=["--word2vec_path", "", "--batch_size", str(b), "--num_frames", "16", "--video_size", "200",
                          "--num_candidates", "4"])
    ctx = pdist.DistContext(device=torch.device("cuda", 0))
    pdist.set_context(ctx)
    seed_everything(1, 0)
    tr = Trainer(args, build_model(args, ctx.device), ctx, 1000)
    data = SyntheticClips(b, 16, 200, 4, args.max_words, args.vocab_size, device=torch.device("cuda"))
    for i in range(2):
        tr.train_step(data.batch(i))
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        tr.train_step(data.batch(2))
        torch.cuda.synchronize()
    names = {"aten::add_", "aten::add", "aten::copy_", "aten::cat", "aten::fill_", "aten::zero_", "aten::mul",
             "aten::to", "aten::_to_copy", "aten::sum", "aten::mm", "aten::addmm", "aten::clone"}
    rows = []
    for e in prof.key_averages(group_by_stack_n=6):
        if e.key in names:
            st = [f for f in (e.stack or []) if "torch/" not in f][:3]
            dev = "cuda" if e.device_type is not None and "CUDA" in str(e.device_type) else ""
            rows.append((e.count, e.key, " <- ".join(st)))
    for n, k, st in sorted(rows, reverse=True)[:50]:
        print(f"{n:4d}  {k:16s} {st}")


if __name__ == "__main__":
    main()
