"""Training engine: one process per GPU, the MIL-NCE step, epochs, checkpoint/resume.

The step (``main_distributed.py:226-241`` ``TrainOneBatch``) is:

    zero flat grads -> [broadcast BN buffers from rank 0] -> forward (S3D-G + text tower)
    -> all-gather video+text embeddings (one collective, local-slice backward)
    -> MIL-NCE over the global batch (computed redundantly on every rank, like the reference)
    -> backward (bucketed RCCL all-reduce issued as buckets fill) -> wait buckets
    -> fused Adam (HIP, grad scale folded in) -> cosine LR step

Differences from the reference, all deliberate: the loss is returned as a device tensor and
only synchronised every ``n_display`` steps (the reference's per-step ``loss.item()``,
``main_distributed.py:241``, is a host sync); the seed reaches every rank.
"""
from __future__ import annotations

import os
import random
import time
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from .. import ops
from ..losses import build_loss
from ..models import S3D
from ..parallel import bucket_plan
from ..parallel import dist as pdist
from ..parallel.ddp import BufferBroadcaster, GradBucketer, broadcast_parameters
from ..utils import MainStream, StepTimer, Watchdog
from . import checkpoint as ckpt
from .logging import MetricsLogger, log, train_line
from .optim import FlatAdam, FlatSGD, cosine_schedule_with_warmup


def seed_everything(seed: int, rank: int = 0) -> None:
    random.seed(seed + rank)
    np.random.seed((seed + rank) % (2 ** 32))
    torch.manual_seed(seed)  # same weights on every rank before the rank-0 broadcast


def build_model(args, device: torch.device) -> S3D:
    blocks = [b for b in (getattr(args, "blocks", "") or "").split(",") if b]
    model = S3D(args.num_class, space_to_depth=False,
                word2vec_path=args.word2vec_path if os.path.isfile(args.word2vec_path or "") else "",
                init=args.weight_init, token_to_word_path=getattr(args, "token_to_word_path", ""),
                vocab_size=getattr(args, "vocab_size", 66250), blocks=blocks)
    if args.pretrain_cnn_path:
        sd = ckpt.load_checkpoint(args.pretrain_cnn_path)
        if "state_dict" in sd:
            sd = sd["state_dict"]
        ckpt.load_model_weights(model, sd, strict=True)
    return model.to(device)


class Trainer:
    def __init__(self, args, model: S3D, ctx: pdist.DistContext, steps_per_epoch: int):
        self.args, self.model, self.ctx = args, model, ctx
        self.device = ctx.device
        # the reference overwrites --rank / --world-size with the process's own (main_distributed.py:46-47,69)
        args.rank, args.world_size = ctx.rank, ctx.world_size
        pdist.set_emb_gather(getattr(args, "emb_gather", "rccl"))
        broadcast_parameters(model, ctx.world_size)
        params = list(model.parameters())
        scale = 1.0 / ctx.world_size if getattr(args, "grad_scale", "reference") == "reference" else 1.0
        if args.optimizer == "adam":
            self.optimizer = FlatAdam(params, lr=args.lr, grad_scale=scale)
        elif args.optimizer == "sgd":
            self.optimizer = FlatSGD(params, lr=args.lr, momentum=args.momemtum, grad_scale=scale)
        else:
            raise ValueError(args.optimizer)
        bucket_mb = getattr(args, "bucket_mb", "auto")
        tail = None
        if bucket_mb == "auto":  # link-aware sizes (parallel/bucket_plan.py), measured at N > 1
            grad_bytes = 4 * sum(p.numel() for p in params if p.requires_grad)
            self.comm_plan = bucket_plan.auto_plan(grad_bytes, ctx.world_size, self.device)
            bucket_bytes, tail = self.comm_plan.bucket_bytes, self.comm_plan.tail_bytes
        else:
            self.comm_plan = None
            bucket_bytes = int(float(bucket_mb) * (1 << 20))
        self.bucketer = GradBucketer(params, ctx.world_size, bucket_bytes, tail_bytes=tail,
                                     verify=bool(getattr(args, "verify_buckets", 0)) or None,
                                     comm_dtype=(torch.bfloat16 if getattr(args, "grad_comm_dtype", "fp32") == "bf16"
                                                 else torch.float32))
        self.optimizer.bind_flat_grad(self.bucketer.flat, self.bucketer.offsets)
        self.buffers = BufferBroadcaster(model, ctx.world_size) if getattr(args, "broadcast_buffers", 1) else None
        self.scheduler = cosine_schedule_with_warmup(self.optimizer, args.warmup_steps,
                                                     steps_per_epoch * args.epochs)
        self.criterion = build_loss(args)
        self.global_step = 0
        self.timer = StepTimer(bool(getattr(args, "phase_timers", 0)), self.device)
        # kernel autotuning (first use of each conv shape) decided by rank 0 for every rank
        from ..ops import tune_sync
        self._tune_synced = ctx.world_size > 1 and tune_sync.configure_from_process_group()

    def tune_region(self):
        """Context of a DP step: every kernel-variant choice made inside is rank 0's (ops/tune_sync)."""
        from ..ops import tune_sync
        return tune_sync.region(self._tune_synced)

    # ---------------------------------------------------------------------------------
    def forward_loss(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        video = batch["video"]
        text = batch["text"]
        text = text.reshape(-1, text.shape[-1])
        with self.timer.phase("forward"):
            video_embd, text_embd = self.model(video, text)
        with self.timer.phase("all_gather"):
            video_embd, text_embd = pdist.all_gather_embeddings(video_embd, text_embd, self.ctx)
        with self.timer.phase("loss"):
            return self._loss(batch, video_embd, text_embd)

    def _loss(self, batch, video_embd, text_embd) -> torch.Tensor:
        name = getattr(self.args, "loss", "milnce")
        if name == "milnce":
            return self.criterion(video_embd, text_embd)
        # soft-DTW family: sequences of seq_len clips, one caption per clip (BASELINE config 4)
        n = getattr(self.args, "seq_len", 8)
        v = video_embd.view(-1, n, video_embd.shape[-1])
        t = text_embd.view(-1, n, text_embd.shape[-1])
        if name == "sdtw_cidm":
            start = batch["start"]
            if self.ctx.world_size > 1:
                out = start.new_empty((self.ctx.world_size,) + tuple(start.shape))
                torch.distributed.all_gather_into_tensor(out, start.contiguous())
                start = out.view(-1, start.shape[-1])
            return self.criterion(v, t, start)
        out = self.criterion(v, t)
        return sum(out) if isinstance(out, tuple) else out

    def train_step(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        fault = getattr(self.args, "fault_at_step", -1)
        if fault >= 0 and self.global_step == fault:
            raise RuntimeError(f"injected fault at step {fault} (--fault_at_step)")
        self.model.train()
        self.bucketer.zero()
        if self.buffers is not None:
            with self.timer.phase("broadcast_buffers"):
                self.buffers()
        chunks = self.grad_cache_chunks(video_batch=batch["video"])
        arena = self.ctx.device.type == "cuda" and ops.use_hip(self.bucketer.flat)
        if arena:
            from ..ops import hip_ops
            hip_ops.zero_arena_begin(self.ctx.device)
        try:
            with self.tune_region():
                if chunks > 1:
                    loss = self._grad_cache_backward(batch, chunks)
                else:
                    loss = self.forward_loss(batch)
                    with self.timer.phase("backward"):
                        loss.backward()
        finally:
            if arena:
                hip_ops.zero_arena_end()
                # the cold-cache flush buffer lives only through the step that tuned (a no-op when
                # nothing was tuned; a resumed run or a new shape tunes at any global_step)
                hip_ops.release_tuning_buffers()
        with self.timer.phase("allreduce_wait"):
            self.bucketer.finish()
        with self.timer.phase("optimizer"):
            self.optimizer.step()
            self.scheduler.step()
        self.global_step += 1
        return loss.detach()

    # Peak memory of the one-shot bf16 step per clip, measured on MI355X (profiles/r3_configs_4_5.md):
    # 203.5 GiB at 1024 clips of 32 x 200^2 (BASELINE config 5), i.e. ~0.199 GiB per clip at 32 x 200^2;
    # activations scale with frames x pixels. The auto mode keeps 10 % of the device in reserve.
    GIB_PER_CLIP_32F200 = 203.5 / 1024

    def grad_cache_chunks(self, video_batch: Optional[torch.Tensor] = None) -> int:
        """Micro-batches of the step: --grad_cache_chunks if set (0/1: one-shot), else (-1) the
        reference's one-shot step whenever its activations fit the device, else the fewest
        GradCache chunks that do. Resolved once, on the first batch, and collectively: every rank
        uses the largest count any rank needs (GradCache normalises BatchNorm per micro-batch, so
        ranks with different counts would contribute gradients of different BN statistics)."""
        req = int(getattr(self.args, "grad_cache_chunks", 0) or 0)
        if req >= 0:
            return req
        if getattr(self, "_auto_chunks", None) is not None:
            return self._auto_chunks
        chunks = 0
        short = ""  # this rank cannot fit one clip: raised on EVERY rank after the collective
        if video_batch is not None:
            v = video_batch
            b = v.shape[0]
            t, h, w = (v.shape[1], v.shape[2], v.shape[3]) if v.shape[-1] in (3, 4) and v.dim() == 5 else \
                (v.shape[2], v.shape[3], v.shape[4])
            est = self.GIB_PER_CLIP_32F200 * b * (t / 32.0) * (h * w / 200.0 ** 2) * 2 ** 30
            budget = self._memory_budget()
            if budget is not None:
                if budget <= est / b:
                    short = (f"{budget / 2 ** 30:.2f} GiB left for the step, less than one clip's activations "
                             f"({est / b / 2 ** 30:.3f} GiB)")
                    chunks = -1  # the max over ranks below is inf: every rank raises
                elif est > budget:
                    chunks = int(min(b, -(-est // budget)))
        if self.ctx.world_size > 1:
            # (a rank that raised before this collective would leave its peers waiting in it)
            chunks = pdist.all_reduce_max(float("inf") if chunks < 0 else float(chunks))
        if chunks < 0 or chunks == float("inf"):
            why = short or "another rank has less than one clip's activations of device memory left"
            raise RuntimeError(f"--grad_cache_chunks -1: {why}; free device memory or lower --batch_size")
        chunks = int(chunks)
        self._auto_chunks = chunks if chunks > 1 else 0
        if self.ctx.is_main and getattr(self.args, "checkpoint_dir", ""):  # a real run's log, not bench / tests
            log(f"grad_cache_chunks -1 resolved to {self._auto_chunks} "
                f"({'one-shot step' if self._auto_chunks == 0 else 'GradCache micro-batches'})", self.args, 0)
        return self._auto_chunks

    def _memory_budget(self) -> Optional[float]:
        """Bytes this step may still allocate while keeping 10 % of the device free (None: no device
        memory model, e.g. CPU)."""
        if self.device.type != "cuda":
            return None
        free, total = torch.cuda.mem_get_info(self.device)
        return 0.9 * total - (total - free)

    def _grad_cache_backward(self, batch: Dict[str, torch.Tensor], chunks: int) -> torch.Tensor:
        """GradCache two-pass step: the loss still sees every rank's
        full local batch as negatives, but activations are only held for one micro-batch.

        1. embeddings of all micro-batches without an autograd graph (BN running statistics
           are restored afterwards, so they advance once per micro-batch as in pass 2);
        2. all-gather + loss + backward to the (local) embeddings only;
        3. per micro-batch: re-forward with the graph, backward the cached embedding gradient
           (gradient all-reduce is issued during the last micro-batch only).
        BatchNorm sees micro-batch statistics, the usual gradient-accumulation semantics.
        """
        video, text = batch["video"], batch["text"]
        b = video.shape[0]
        bounds = [(i * b // chunks, (i + 1) * b // chunks) for i in range(chunks)]
        bounds = [(s, e) for s, e in bounds if e > s]
        bufs = [t for t in self.model.buffers()]
        saved = [t.clone() for t in bufs]
        with torch.no_grad(), self.timer.phase("gc_embed"):
            vs, ts = [], []
            for s, e in bounds:
                v, t = self.model(video[s:e], text[s:e].reshape(-1, text.shape[-1]))
                vs.append(v)
                ts.append(t)
            for t, v in zip(bufs, saved):
                t.copy_(v)
        ve = torch.cat(vs).detach().requires_grad_(True)
        te = torch.cat(ts).detach().requires_grad_(True)
        with self.timer.phase("all_gather"):
            vg, tg = pdist.all_gather_embeddings(ve, te, self.ctx)
        with self.timer.phase("loss"):
            loss = self._loss(batch, vg, tg)
        loss.backward()
        k = text.shape[1] if text.dim() == 3 else 1
        with self.timer.phase("backward"):
            for i, (s, e) in enumerate(bounds):
                self.bucketer.set_sync(i == len(bounds) - 1)
                v, t = self.model(video[s:e], text[s:e].reshape(-1, text.shape[-1]))
                surrogate = (v * ve.grad[s:e].to(v.dtype)).sum() + (t * te.grad[s * k:e * k].to(t.dtype)).sum()
                surrogate.backward()
            self.bucketer.set_sync(True)
        return loss

    # ---------------------------------------------------------------------------------
    def state(self, epoch: int, step_in_epoch: int = 0) -> dict:
        """Reference checkpoint dict; a mid-epoch checkpoint adds ``step_in_epoch``."""
        st = {"epoch": epoch, "state_dict": ckpt.model_state_dict(self.model),
              "optimizer": self.optimizer.state_dict(), "scheduler": self.scheduler.state_dict()}
        if step_in_epoch:
            st["step_in_epoch"] = step_in_epoch
        return st

    def load_state(self, state: dict) -> int:
        ckpt.load_model_weights(self.model, state["state_dict"], strict=True)
        self.optimizer.load_state_dict(state["optimizer"])
        self.scheduler.load_state_dict(state["scheduler"])
        self.global_step = int(self.scheduler.last_epoch)
        return int(state["epoch"])


def checkpoint_dir_of(args) -> str:
    return os.path.join(getattr(args, "checkpoint_root", "checkpoint") or "checkpoint", args.checkpoint_dir)


def run_training(args, ctx: Optional[pdist.DistContext] = None) -> Dict[str, float]:
    """Epoch loop of main_distributed.py:185-200 over the synthetic or the HowTo100M feed."""
    from ..data.loader import build_train_feed

    ctx = ctx or pdist.context()
    seed_everything(args.seed, ctx.rank)
    # batch_size is per node; divided across the node's GPUs like main_distributed.py:88.
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world_size)))
    local_bs = max(1, args.batch_size // max(1, local_world))
    feed = build_train_feed(args, ctx, local_bs)
    steps_per_epoch = feed.steps_per_epoch
    model = build_model(args, ctx.device)
    trainer = Trainer(args, model, ctx, steps_per_epoch)
    metrics = MetricsLogger(getattr(args, "log_jsonl", ""), ctx.rank)
    cdir = checkpoint_dir_of(args)
    if ctx.is_main and args.checkpoint_dir:
        os.makedirs(cdir, exist_ok=True)
    pdist.barrier()
    start_epoch = args.start_epoch
    start_step = 0
    if args.resume:
        path = ckpt.get_last_checkpoint(cdir)
        if path:
            log("=> loading checkpoint '{}'".format(path), args, ctx.rank)
            state = ckpt.load_checkpoint(path, map_location=ctx.device)
            start_epoch = trainer.load_state(state)
            start_step = int(state.get("step_in_epoch", 0))
            log("=> loaded checkpoint '{}' (epoch {})".format(path, start_epoch), args, ctx.rank)
        else:
            log("=> no checkpoint found at '{}'".format(cdir), args, ctx.rank)
    total_bs = local_bs * ctx.world_size  # clips per step over all ranks
    log("Starting training loop for rank: {}, total batch size: {}".format(ctx.rank, total_bs), args, ctx.rank)
    watchdog = Watchdog(getattr(args, "watchdog_s", 0.0), ctx.rank,
                        dump_dir=getattr(args, "log_root", "log") or "log").start()
    eval_every = max(1, total_bs // 512)  # main_distributed.py:188
    try:
        with MainStream(ctx.device):  # the steps on a high-priority stream (utils/streams.py)
            return _epochs(args, ctx, trainer, feed, metrics, cdir, watchdog, start_epoch, start_step,
                           steps_per_epoch, total_bs, eval_every)
    finally:
        watchdog.stop()


def _epochs(args, ctx, trainer, feed, metrics, cdir, watchdog, start_epoch, start_step, steps_per_epoch, total_bs,
            eval_every) -> Dict[str, float]:
    """The epoch loop of run_training (main_distributed.py:185-200)."""
    last = {}
    for epoch in range(start_epoch, args.epochs):
        if args.evaluate and epoch % eval_every == 0 and not (epoch == start_epoch and start_step):
            from .evaluation import evaluate_hmdb_during_training
            res = evaluate_hmdb_during_training(args, ctx, trainer.model)
            if ctx.is_main and res:
                metrics.write(epoch=epoch, step=trainer.global_step, hmdb=res)
        running = torch.zeros((), device=ctx.device)
        t0 = time.time()
        first = start_step if epoch == start_epoch else 0
        for i, batch in enumerate(feed.epoch(epoch, first), start=first):
            running += trainer.train_step(batch)
            watchdog.beat(trainer.global_step)
            if (i + 1) % args.n_display == 0:
                avg = float(running.item()) / args.n_display  # the only host sync
                d = time.time() - t0
                lr = trainer.optimizer.param_groups[0]["lr"]
                if args.verbose:
                    log(train_line(epoch + 1, d, total_bs * float(i) / max(1, feed.epoch_len), avg, lr), args,
                        ctx.rank)
                metrics.write(epoch=epoch + 1, step=trainer.global_step, loss=avg, lr=lr,
                              pairs_per_s=total_bs * args.n_display / max(d, 1e-9),
                              phase_ms=trainer.timer.summary())
                last = {"loss": avg, "lr": lr}
                running.zero_()
                t0 = time.time()
            if (args.ckpt_every_steps and trainer.global_step % args.ckpt_every_steps == 0
                    and i + 1 < steps_per_epoch):
                # mid-epoch checkpoint: same file family (epoch%04d of the epoch in progress),
                # plus step_in_epoch so --resume continues from the next step
                if ctx.is_main:
                    ckpt.save_checkpoint(trainer.state(epoch, i + 1), cdir, epoch)
                pdist.barrier()
        if ctx.is_main:
            ckpt.save_checkpoint(trainer.state(epoch + 1), cdir, epoch + 1)
        pdist.barrier()
        if getattr(args, "stop_epoch", 0) and epoch + 1 >= args.stop_epoch:
            break
    return last
