import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.config import get_args
from mil_nce_howto100m_amd.data.synthetic import SyntheticClips
from mil_nce_howto100m_amd.parallel import dist as pdist
from mil_nce_howto100m_amd.train.engine import Trainer, build_model, seed_everything
from mil_nce_howto100m_amd.ops import grad_sink
args = get_args(argv=["--batch_size", "4", "--num_frames", "8", "--video_size", "64", "--num_candidates", "2",
                      "--blocks", "mixed_3b,mixed_3c", "--word2vec_path", "", "--vocab_size", "1000"])
ctx = pdist.DistContext(device=torch.device("cuda", 0))
data = SyntheticClips(4, 8, 64, 2, 20, 1000, device=ctx.device)
seed_everything(1, 0)
tr = Trainer(args, build_model(args, ctx.device), ctx, 10)
tr.model.eval()
tr.bucketer.zero()
calls = []
orig = grad_sink.drain
def drain():
    import threading
    calls.append((threading.current_thread().name, torch.cuda.current_stream().cuda_stream, len(grad_sink._PENDING)))
    orig()
grad_sink.drain = drain
for i in range(2):
    tr.forward_loss(data.batch(0)).backward()
    print("pass", i, "pending after backward:", grad_sink.pending(), "drain calls:", calls,
          "main stream", torch.cuda.current_stream().cuda_stream, flush=True)
    calls.clear()
