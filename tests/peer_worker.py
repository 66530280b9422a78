"""One rank of tests/test_gpu_peer.py: the one-shot peer-write all-gather (parallel/peer.py)
between two processes sharing cuda:0 over IPC-mapped receive buffers, against the known rank-major
result, plus the comm probe's timing of both gather paths. argv: OUTDIR."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    out = sys.argv[1]
    from mil_nce_howto100m_amd.parallel import dist as pdist
    from mil_nce_howto100m_amd.parallel.peer import PeerAllGather
    ctx = pdist.init_distributed("gloo", "cuda")
    W, r = ctx.world_size, ctx.rank
    dev = ctx.device
    pg = PeerAllGather()
    res = {"rank": r, "checks": 0}
    for rows, cols, dt in ((5, 512, torch.float32), (16, 64, torch.bfloat16), (3, 8, torch.float32)):
        for call in range(3):  # both receive buffers, then the first again
            x = (torch.arange(rows * cols, device=dev, dtype=torch.float32).view(rows, cols) + 1000 * r + 7 * call)
            got = pg.gather(x.to(dt))
            want = torch.cat([(torch.arange(rows * cols, device=dev, dtype=torch.float32).view(rows, cols)
                               + 1000 * q + 7 * call).to(dt) for q in range(W)])
            assert got.shape == (W * rows, cols) and torch.equal(got, want), (rows, cols, dt, call)
            res["checks"] += 1
    # through the model-facing entry point: rank-major gather, local-slice backward
    pdist.set_emb_gather("peer")
    v = torch.full((2, 16), float(r), device=dev, requires_grad=True)
    t = torch.full((4, 16), 10.0 + r, device=dev, requires_grad=True)
    gv, gt = pdist.all_gather_embeddings(v, t, ctx)
    (gv.sum() * 2 + gt.sum() * 3).backward()
    assert torch.equal(gv[:, 0].cpu(), torch.tensor([0.0, 0.0, 1.0, 1.0]))
    assert torch.equal(gt[:, 0].cpu(), torch.tensor([10.0] * 4 + [11.0] * 4))
    assert torch.equal(v.grad.cpu(), torch.full((2, 16), 2.0))
    assert torch.equal(t.grad.cpu(), torch.full((4, 16), 3.0))
    from mil_nce_howto100m_amd.parallel.comm_probe import probe
    res["comm"] = probe(1 << 20, [(0, 1 << 19), (1 << 19, 1 << 20)], 768, 512, torch.float32, dev, reps=5)
    torch.cuda.synchronize()
    with open(os.path.join(out, f"peer_r{r}.json"), "w") as f:
        json.dump(res, f)
    pdist.destroy()


if __name__ == "__main__":
    main()
