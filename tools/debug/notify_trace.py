"""Debug: where do parameter-ready notifications come from on the HIP path?"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch
from mil_nce_howto100m_amd.config import get_args
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
from mil_nce_howto100m_amd.parallel import dist as pdist
from mil_nce_howto100m_amd.parallel.ddp import GradBucketer
from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
from mil_nce_howto100m_amd.ops import grad_sink

ctx = pdist.init_distributed("nccl", "cuda")
args = get_args(argv=["--batch_size", "4", "--num_frames", "8", "--video_size", "64", "--num_candidates", "2",
                      "--word2vec_path", "", "--warmup_steps", "1"])
seed_everything(3, 0)
tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
names = {id(p): n for n, p in tr.model.named_parameters()}
bk = GradBucketer(list(tr.model.parameters()), world_size=2, bucket_bytes=2 << 20)
tr.bucketer = bk
tr.optimizer.bind_flat_grad(bk.flat, bk.offsets)
stacks = collections.defaultdict(list)


def on_grad(p, src):
    stacks[id(p)].append(src + " | " + " <- ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-6:-1]))


for h in bk._hooks:
    h.remove()
for p in bk.params:
    p.register_post_accumulate_grad_hook(lambda p: on_grad(p, "hook"))
grad_sink.set_sink(lambda p: on_grad(p, "sink"))
bk._launch = lambda i: None
data = SyntheticClips(4, 8, 64, 2, args.max_words, args.vocab_size, device=ctx.device)
for step in range(2):
    stacks.clear()
    tr.bucketer.zero()
    loss = tr.forward_loss(data.batch(step))
    loss.backward()
    torch.cuda.synchronize()
    cnt = collections.Counter(len(v) for v in stacks.values())
    print("step", step, "notify-count histogram", dict(cnt), "missing", len(bk.params) - len(stacks))
    shown = 0
    for k, v in stacks.items():
        if len(v) != 1 and shown < 6:
            shown += 1
            print(names[k])
            for s in v:
                print("    ", s)
