"""Test helper: instruments a GradBucketer to check gradient-bucket readiness."""
import torch


class BucketRecorder:
    """Wraps a GradBucketer: records per-parameter readiness reports and snapshots each bucket's
    flat slice at the moment its all-reduce is issued (stream order == what RCCL would read)."""

    def __init__(self, bucketer):
        self.b = bucketer
        self.notes = {}
        self.snaps = {}
        self.issued_in_finish = []
        self._in_finish = False
        orig_on_grad, orig_launch, orig_finish = bucketer._on_grad, bucketer._launch, bucketer.finish

        def on_grad(p):
            if self.b.sync_enabled:
                self.notes[id(p)] = self.notes.get(id(p), 0) + 1
            orig_on_grad(p)

        def launch(i):
            s, e = self.b.buckets[i]
            assert i not in self.snaps, f"bucket {i} issued twice"
            if self.b.flat.is_cuda:
                # what the bucket's all-reduce reads: the bucketer issues it from a stream that
                # waits for the compute stream and the side stream's deferred writes (grad_sink.join)
                from mil_nce_howto100m_amd.ops import grad_sink
                st = torch.cuda.Stream(device=self.b.flat.device)
                st.wait_stream(torch.cuda.current_stream(self.b.flat.device))
                grad_sink.join(st)
                with torch.cuda.stream(st):
                    self.snaps[i] = self.b.flat[s:e].clone()
                torch.cuda.current_stream(self.b.flat.device).wait_stream(st)
            else:
                self.snaps[i] = self.b.flat[s:e].clone()
            if self._in_finish:
                self.issued_in_finish.append(i)
            orig_launch(i)

        def finish():
            self._in_finish = True
            orig_finish()
            self._in_finish = False

        # hooks registered in the constructor hold the bound method: route through the wrapper
        bucketer._on_grad = on_grad
        bucketer._launch = launch
        bucketer.finish = finish
        from mil_nce_howto100m_amd.ops import grad_sink
        grad_sink.set_sink(on_grad)
        for h in bucketer._hooks:
            h.remove()
        bucketer._hooks = [p.register_post_accumulate_grad_hook(on_grad) for p in bucketer.params]

    def check(self):
        b = self.b
        assert sorted(self.snaps) == list(range(len(b.buckets)))
        assert not self.issued_in_finish, f"buckets never became ready: {self.issued_in_finish}"
        # a parameter may report more than once (in-place HIP gradient write + autograd's
        # post-accumulate hook); the bucketer must count it once -- the snapshots catch an
        # early issue -- but every parameter has to report
        missing = [tuple(p.shape) for p in b.params if self.notes.get(id(p), 0) == 0]
        assert not missing, f"{len(missing)} params never reported ready: {missing[:12]}"
        return self.snaps
