"""Model structure, parameter/checkpoint compatibility and NDHWC-vs-NCDHW parity (CPU)."""
import os
import tempfile

import torch

from mil_nce_howto100m_amd.models import S3D
from mil_nce_howto100m_amd.train import checkpoint as ckpt

import ref_s3d


def test_param_counts_and_keys_match_reference():
    m = S3D(512)
    assert sum(p.numel() for p in m.parameters()) == 31_190_408
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == 11_315_408
    sd = m.state_dict()
    assert len(sd) == 537
    suffix = {}
    for k in sd:
        s = k.rsplit(".", 1)[1]
        suffix[s] = suffix.get(s, 0) + 1
    assert suffix == {"weight": 193, "bias": 116, "running_mean": 76, "running_var": 76,
                      "num_batches_tracked": 76}
    assert tuple(sd["conv_2c.conv1.weight"].shape) == (192, 64, 1, 3, 3)
    assert tuple(sd["conv_2c.conv2.weight"].shape) == (192, 192, 3, 1, 1)
    assert tuple(sd["text_module.word_embd.weight"].shape) == (66250, 300)
    assert not m.text_module.word_embd.weight.requires_grad
    assert len(list(m.parameters())) == 309


def test_space_to_depth_variant_params():
    m = S3D(512, space_to_depth=True)
    assert sum(p.numel() for p in m.parameters()) == 31_211_336
    assert tuple(m.state_dict()["conv1.conv1.weight"].shape) == (64, 24, 2, 4, 4)


def test_forward_matches_ncdhw_oracle_train_and_eval():
    torch.manual_seed(0)
    m = S3D(512).double()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    v = torch.rand(2, 3, 8, 64, 64, dtype=torch.float64)
    t = torch.randint(0, 66250, (4, 20))
    ve, te = m(v, t)
    assert ve.shape == (2, 512) and te.shape == (4, 512)
    ref_v = ref_s3d.s3d_video(sd, v, training=True)
    ref_t = ref_s3d.s3d_text(sd, t)
    assert torch.allclose(ve, ref_v, rtol=1e-8, atol=1e-9)
    assert torch.allclose(te, ref_t, rtol=1e-8, atol=1e-9)
    m.eval()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    f = m(v, None, mode="video", mixed5c=True)
    assert f.shape == (2, 1024)
    assert torch.allclose(f, ref_s3d.s3d_video(sd, v, training=False, mixed5c=True), rtol=1e-8, atol=1e-9)


def test_uint8_native_input_equals_float_reference_input():
    torch.manual_seed(1)
    m = S3D(512, blocks=["mixed_3b"]).double().eval()
    u8 = torch.randint(0, 256, (2, 8, 32, 32, 4), dtype=torch.uint8)
    u8[..., 3] = 0
    a = m(u8, None, mode="video")
    b = m(u8[..., :3].permute(0, 4, 1, 2, 3).double() / 255.0, None, mode="video")
    assert torch.allclose(a.double(), b, rtol=1e-5, atol=1e-6)


def test_checkpoint_roundtrip_reference_format():
    torch.manual_seed(2)
    m = S3D(512, blocks=["mixed_3b"])
    opt = torch.optim.Adam(m.parameters(), 1e-3)
    with tempfile.TemporaryDirectory() as d:
        state = {"epoch": 3, "state_dict": ckpt.model_state_dict(m), "optimizer": opt.state_dict(),
                 "scheduler": {"last_epoch": 0}}
        for e in range(1, 14):
            ckpt.save_checkpoint(state, d, e)
        files = sorted(os.listdir(d))
        assert files[0] == "epoch0004.pth.tar" and files[-1] == "epoch0013.pth.tar" and len(files) == 10
        assert ckpt.get_last_checkpoint(d).endswith("epoch0013.pth.tar")
        loaded = ckpt.load_checkpoint(ckpt.get_last_checkpoint(d))
        assert all(k.startswith("module.") for k in loaded["state_dict"])
        m2 = S3D(512, blocks=["mixed_3b"])
        ckpt.load_model_weights(m2, loaded["state_dict"])
        for (k1, v1), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
            assert k1 == k2 and torch.equal(v1, v2)
        # a plain nn.Module with the reference's names loads it strictly (DataParallel-style)
        plain = torch.nn.DataParallel(S3D(512, blocks=["mixed_3b"]))
        plain.load_state_dict(loaded["state_dict"], strict=True)


def test_space_to_depth_forward_matches_ncdhw_oracle():
    """The public-weights (space-to-depth) variant: s2d input transform, [2,4,4] conv1 with pad
    (1,2,2), BN+ReLU over the uncropped output, crop [1:, 1:, 1:] (s3dg.py:248-253, 267-272);
    fp64 against an independent NCDHW oracle, train and eval mode."""
    torch.manual_seed(4)
    m = S3D(512, space_to_depth=True, blocks=["mixed_3b", "mixed_3c"]).double()
    v = torch.rand(2, 3, 8, 64, 64, dtype=torch.float64)
    for training in (True, False):
        m.train(training)
        sd = {k: x.clone() for k, x in m.state_dict().items()}
        f = m(v, None, mode="video", mixed5c=True)
        ref = ref_s3d.s3d_video(sd, v, training=training, mixed5c=True)
        assert torch.allclose(f, ref, rtol=1e-8, atol=1e-9), (training, (f - ref).abs().max())


def test_main_stream_on_cpu_is_a_no_op():
    """utils/streams.py MainStream does nothing for a CPU device (the gloo / CPU runs)."""
    from mil_nce_howto100m_amd.utils import MainStream
    with MainStream(torch.device("cpu")) as ms:
        assert not ms.enabled and ms.priority == 0
